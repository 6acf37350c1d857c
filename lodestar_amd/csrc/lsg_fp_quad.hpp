// Quad backend: 381-bit Montgomery arithmetic with one Fp element per 4-lane quad.
//
// Lane q (0..3) of a quad holds limbs 3q, 3q+1, 3q+2 of the element (32-bit limbs, little
// endian), so all 12 limbs are live and a wave64 carries sixteen independent field elements
// (sixteen signature sets).  Compared with one element per 16-lane row (lsg_fp_lane.hpp,
// four elements per wave, lanes 12..15 idle) a Montgomery product issues about half the
// instructions per element and a field addition about a quarter.
//
// Montgomery multiplication is CIOS with the i-loop over time; every lane runs its three
// limbs of the j-loop:
//   b_i   : DPP quad_perm broadcast from lane i/3 (register i%3 is a compile-time choice)
//   m     : quad broadcast of limb 0 (lane 0) times n0'
//   a_j b_i and m p_j : one v_mad_u64_u32 each
//   /2^32 : limbs 1,2 move down inside the lane (register renaming), limb 0 of lane q+1
//           arrives by a DPP quad shift
// Carries are deferred per limb in two 32-bit words (ca from the a*b column, cb from the m*p
// column), exactly as in the row backend, so every v_mad_u64_u32 addend stays < 2^33.  The
// carries of a limb stay at the same limb index across the shift, so nothing but the limb
// values crosses lanes inside the loop.  Carry resolution and the conditional subtraction
// of p propagate inside the lane with add/sub-with-carry chains and across the four lanes
// with a carry-lookahead on s_ballot masks ((G|P)+G)^(G|P)^G, with the top lane of every
// quad masked out so that quads never interact.
#pragma once
#include "lsg_constants.hpp"

#define LSG_QUAD_MODE 1
#define LSG_GROUP 4  // lanes per field element
// the generic layers built on this backend are device-only code
#undef LSG_INL
#define LSG_INL __device__ __forceinline__
#undef LSG_NOINL
#define LSG_NOINL __device__ __noinline__

LSG_DEVI uint32_t qidx() { return __lane_id() & 3u; }
LSG_DEVI uint32_t qbase() { return __lane_id() & 60u; }

LSG_DEVI uint32_t sel4(uint32_t q, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return q == 0 ? a : (q == 1 ? b : (q == 2 ? c : d));
}

struct fp_t {
  uint32_t l0, l1, l2;
  fp_t() = default;
  LSG_DEVI fp_t(const fpc_t& c) {
    uint32_t q = qidx();
    l0 = sel4(q, c.l[0], c.l[3], c.l[6], c.l[9]);
    l1 = sel4(q, c.l[1], c.l[4], c.l[7], c.l[10]);
    l2 = sel4(q, c.l[2], c.l[5], c.l[8], c.l[11]);
  }
  LSG_DEVI fp_t(uint32_t a, uint32_t b, uint32_t c) : l0(a), l1(b), l2(c) {}
};
// lane-q limbs of a 12-limb literal array
LSG_DEVI fp_t fp_from_arr(const uint32_t* c) {
  uint32_t q = qidx();
  return fp_t(sel4(q, c[0], c[3], c[6], c[9]), sel4(q, c[1], c[4], c[7], c[10]), sel4(q, c[2], c[5], c[8], c[11]));
}

// ---- DPP helpers (control codes must be immediates)
template <int CTRL>
LSG_DEVI uint32_t qdpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
}
// value of lane s of the quad
template <int S>
LSG_DEVI uint32_t qbcast(uint32_t x) {
  return qdpp<S * 0x55>(x);
}
LSG_DEVI uint32_t qshift_down(uint32_t x) { return qdpp<0xF9>(x); }  // lane q <- lane q+1 (3 <- 3)
LSG_DEVI uint32_t qshift_up(uint32_t x) { return qdpp<0x90>(x); }    // lane q <- lane q-1 (0 <- 0)

// ---- carry lookahead over the quads of a wave.  g: this lane produces a carry out of its
// top limb by itself; p: this lane passes an incoming carry through.  Returns the carry into
// this lane; *out (if given) gets the carry out of the quad's top lane.
constexpr uint64_t LSG_QTOP = 0x8888888888888888ull;
LSG_DEVI bool quad_carry(bool g, bool p, bool* out) {
  uint64_t G = __ballot(g), P = __ballot(p);
  uint64_t Gm = G & ~LSG_QTOP, Am = (G | P) & ~LSG_QTOP;
  uint64_t cin = (Am + Gm) ^ Am ^ Gm;
  uint32_t l = __lane_id();
  if (out) {
    uint32_t t = qbase() + 3;
    bool ct = (cin >> t) & 1u;
    *out = ((G >> t) & 1u) || (((P >> t) & 1u) && ct);
  }
  return (cin >> l) & 1u;
}
LSG_DEVI bool quad_none(bool pred) { return ((__ballot(pred) >> qbase()) & 0xfull) == 0; }

// p limbs of this lane (LDS copy; see lsg_lane_setup)
__shared__ uint32_t lsg_lds_p[12];
LSG_DEVI void lsg_lane_setup() {
  uint32_t l = __lane_id();
  if (l < 12) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 12; k++) v = (l == (uint32_t)k) ? LSG_P[k] : v;  // literals, no memory
    lsg_lds_p[l] = v;
  }
}
LSG_DEVI fp_t p_limbs() {
  uint32_t q = qidx();
  return fp_t(lsg_lds_p[3 * q], lsg_lds_p[3 * q + 1], lsg_lds_p[3 * q + 2]);
}

// a + c_in (c_in in {0,1}) over the lane's three limbs; *co = carry out of the lane
LSG_DEVI fp_t lane_add_bit(const fp_t& a, uint32_t cin, uint32_t* co) {
  uint32_t c = 0;
  fp_t r;
  r.l0 = __builtin_addc(a.l0, cin, 0u, &c);
  r.l1 = __builtin_addc(a.l1, 0u, c, &c);
  r.l2 = __builtin_addc(a.l2, 0u, c, &c);
  *co = c;
  return r;
}
LSG_DEVI fp_t lane_sub_bit(const fp_t& a, uint32_t bin, uint32_t* bo) {
  uint32_t b = 0;
  fp_t r;
  r.l0 = __builtin_subc(a.l0, bin, 0u, &b);
  r.l1 = __builtin_subc(a.l1, 0u, b, &b);
  r.l2 = __builtin_subc(a.l2, 0u, b, &b);
  *bo = b;
  return r;
}
LSG_DEVI bool lane_all_ones(const fp_t& a) { return (a.l0 & a.l1 & a.l2) == 0xffffffffu; }
LSG_DEVI bool lane_all_zero(const fp_t& a) { return (a.l0 | a.l1 | a.l2) == 0u; }

// full 384-bit a + b (no overflow beyond limb 11 for the inputs used here)
LSG_DEVI fp_t quad_add_raw(const fp_t& a, const fp_t& b) {
  uint32_t c = 0;
  fp_t s;
  s.l0 = __builtin_addc(a.l0, b.l0, 0u, &c);
  s.l1 = __builtin_addc(a.l1, b.l1, c, &c);
  s.l2 = __builtin_addc(a.l2, b.l2, c, &c);
  bool cin = quad_carry(c != 0, lane_all_ones(s), nullptr);
  uint32_t dummy;
  return lane_add_bit(s, cin ? 1u : 0u, &dummy);
}
// a - b; *neg = (a < b)
LSG_DEVI fp_t quad_sub_raw(const fp_t& a, const fp_t& b, bool* neg) {
  uint32_t br = 0;
  fp_t d;
  d.l0 = __builtin_subc(a.l0, b.l0, 0u, &br);
  d.l1 = __builtin_subc(a.l1, b.l1, br, &br);
  d.l2 = __builtin_subc(a.l2, b.l2, br, &br);
  bool bin = quad_carry(br != 0, lane_all_zero(d), neg);
  uint32_t dummy;
  return lane_sub_bit(d, bin ? 1u : 0u, &dummy);
}

// z < 2p -> z mod p
LSG_DEVI fp_t quad_reduce_once(const fp_t& z, const fp_t& p) {
  bool neg;
  fp_t d = quad_sub_raw(z, p, &neg);
  return neg ? z : d;
}

// N independent Montgomery products, interleaved (N chains in flight per lane, three limbs each)
template <int N>
LSG_DEVI void quad_mont_mul_n(const fp_t* a, const fp_t* b, fp_t* r) {
  const fp_t p = p_limbs();
  const bool top = qidx() == 3;
  uint32_t x[N][3], ca[N][3], cb[N][3];
#pragma unroll
  for (int k = 0; k < N; k++)
#pragma unroll
    for (int j = 0; j < 3; j++) x[k][j] = ca[k][j] = cb[k][j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
#pragma unroll
    for (int k = 0; k < N; k++) {
      const uint32_t bsrc = (i % 3 == 0) ? b[k].l0 : ((i % 3 == 1) ? b[k].l1 : b[k].l2);
      uint32_t bi;
      if (i / 3 == 0) bi = qbcast<0>(bsrc);
      else if (i / 3 == 1) bi = qbcast<1>(bsrc);
      else if (i / 3 == 2) bi = qbcast<2>(bsrc);
      else bi = qbcast<3>(bsrc);
      const uint32_t av[3] = {a[k].l0, a[k].l1, a[k].l2};
      const uint32_t pv[3] = {p.l0, p.l1, p.l2};
      uint32_t t2l[3], t2h[3], sh[3];
#pragma unroll
      for (int j = 0; j < 3; j++) {
        uint32_t tl = x[k][j] + ca[k][j];
        uint32_t th = tl < ca[k][j];
        uint64_t s = (uint64_t)av[j] * bi + (((uint64_t)th << 32) | tl);
        uint32_t sl = (uint32_t)s;
        sh[j] = (uint32_t)(s >> 32);
        t2l[j] = sl + cb[k][j];
        t2h[j] = t2l[j] < cb[k][j];
      }
      const uint32_t m = qbcast<0>(t2l[0]) * LSG_N0P;
      uint32_t ul[3];
#pragma unroll
      for (int j = 0; j < 3; j++) {
        uint64_t u = (uint64_t)m * pv[j] + (((uint64_t)t2h[j] << 32) | t2l[j]);
        ul[j] = (uint32_t)u;
        cb[k][j] = (uint32_t)(u >> 32);
        ca[k][j] = sh[j];
      }
      const uint32_t up = qshift_down(ul[0]);
      x[k][0] = ul[1];
      x[k][1] = ul[2];
      x[k][2] = top ? 0u : up;
    }
  }
  // resolve the deferred carries: value = sum_J (x_J + ca_J + cb_J) 2^(32 J) < 2p
#pragma unroll
  for (int k = 0; k < N; k++) {
    uint64_t y0 = (uint64_t)x[k][0] + ca[k][0] + cb[k][0];
    uint64_t y1 = (uint64_t)x[k][1] + ca[k][1] + cb[k][1] + (y0 >> 32);
    uint64_t y2 = (uint64_t)x[k][2] + ca[k][2] + cb[k][2] + (y1 >> 32);
    // lane carry-out (<= 3) goes to limb 0 of the next lane
    uint32_t hin = qshift_up((uint32_t)(y2 >> 32));
    hin = qidx() == 0 ? 0u : hin;
    fp_t z((uint32_t)y0, (uint32_t)y1, (uint32_t)y2);
    uint32_t c = 0;
    z.l0 = __builtin_addc(z.l0, hin, 0u, &c);
    z.l1 = __builtin_addc(z.l1, 0u, c, &c);
    z.l2 = __builtin_addc(z.l2, 0u, c, &c);
    bool cin = quad_carry(c != 0, lane_all_ones(z), nullptr);
    uint32_t dummy;
    z = lane_add_bit(z, cin ? 1u : 0u, &dummy);
    r[k] = quad_reduce_once(z, p);
  }
}

LSG_DEVNOINL fp_t quad_mont_mul(fp_t a, fp_t b) {
  fp_t r;
  quad_mont_mul_n<1>(&a, &b, &r);
  return r;
}
struct lsg_fp2x_t {
  fp_t a, b;
};
struct lsg_fp3x_t {
  fp_t a, b, c;
};
LSG_DEVNOINL lsg_fp2x_t quad_mont_mul2(fp_t a0, fp_t b0, fp_t a1, fp_t b1) {
  fp_t aa[2] = {a0, a1}, bb[2] = {b0, b1}, r[2];
  quad_mont_mul_n<2>(aa, bb, r);
  return lsg_fp2x_t{r[0], r[1]};
}
LSG_DEVNOINL lsg_fp3x_t quad_mont_mul3(fp_t a0, fp_t b0, fp_t a1, fp_t b1, fp_t a2, fp_t b2) {
  fp_t aa[3] = {a0, a1, a2}, bb[3] = {b0, b1, b2}, r[3];
  quad_mont_mul_n<3>(aa, bb, r);
  return lsg_fp3x_t{r[0], r[1], r[2]};
}

LSG_DEVNOINL fp_t quad_add(fp_t a, fp_t b) { return quad_reduce_once(quad_add_raw(a, b), p_limbs()); }
LSG_DEVNOINL fp_t quad_sub(fp_t a, fp_t b) {
  bool neg;
  fp_t d = quad_sub_raw(a, b, &neg);
  fp_t e = quad_add_raw(d, p_limbs());
  return neg ? e : d;
}

// ------------------------------------------------------------------ Fp API
LSG_DEVI fp_t fp_zero() { return fp_t(0u, 0u, 0u); }
LSG_INL fp_t fp_canonical(const fp_t& a) { return a; }  // values are kept fully reduced
LSG_DEVI bool fp_is_zero(const fp_t& a) { return quad_none(!lane_all_zero(a)); }
LSG_DEVI bool fp_eq(const fp_t& a, const fp_t& b) {
  return quad_none(((a.l0 ^ b.l0) | (a.l1 ^ b.l1) | (a.l2 ^ b.l2)) != 0u);
}
LSG_DEVI fp_t fp_select(bool c, const fp_t& a, const fp_t& b) {
  return fp_t(c ? a.l0 : b.l0, c ? a.l1 : b.l1, c ? a.l2 : b.l2);
}
LSG_DEVI fp_t fp_add(const fp_t& a, const fp_t& b) { return quad_add(a, b); }
LSG_DEVI fp_t fp_sub(const fp_t& a, const fp_t& b) { return quad_sub(a, b); }
LSG_DEVI fp_t fp_neg(const fp_t& a) { return quad_sub(fp_zero(), a); }
LSG_DEVI fp_t fp_mul(const fp_t& a, const fp_t& b) { return quad_mont_mul(a, b); }
#ifndef LSG_QUAD_MUL_WIDTH
#define LSG_QUAD_MUL_WIDTH 1  // chains per call: 1 keeps the leaf inside v0..v39
#endif
LSG_DEVI void fp_mul2(fp_t& r0, fp_t& r1, const fp_t& a0, const fp_t& b0, const fp_t& a1, const fp_t& b1) {
#if LSG_QUAD_MUL_WIDTH >= 2
  lsg_fp2x_t r = quad_mont_mul2(a0, b0, a1, b1);
  r0 = r.a;
  r1 = r.b;
#else
  fp_t t = quad_mont_mul(a0, b0);
  r1 = quad_mont_mul(a1, b1);
  r0 = t;
#endif
}
LSG_DEVI void fp_mul3(fp_t& r0, fp_t& r1, fp_t& r2, const fp_t& a0, const fp_t& b0, const fp_t& a1, const fp_t& b1,
                      const fp_t& a2, const fp_t& b2) {
#if LSG_QUAD_MUL_WIDTH >= 3
  lsg_fp3x_t r = quad_mont_mul3(a0, b0, a1, b1, a2, b2);
  r0 = r.a;
  r1 = r.b;
  r2 = r.c;
#else
  fp_t t0 = quad_mont_mul(a0, b0);
  fp_t t1 = quad_mont_mul(a1, b1);
  r2 = quad_mont_mul(a2, b2);
  r0 = t0;
  r1 = t1;
#endif
}
// nine products: three interleaved triples (three limbs x three chains per lane in flight)
LSG_DEVI void fp_mul9(fp_t* r, const fp_t* a, const fp_t* b) {
#pragma unroll
  for (int g = 0; g < 9; g += 3) fp_mul3(r[g], r[g + 1], r[g + 2], a[g], b[g], a[g + 1], b[g + 1], a[g + 2], b[g + 2]);
}

// ---- canonical predicates and byte I/O (quad-uniform results)
LSG_DEVI bool fp_canon_gt_half(const fp_t& c) {
  bool neg;
  (void)quad_sub_raw(fp_from_arr(LSG_HALF_P_CANON), c, &neg);  // borrow of HALF - c
  return neg;
}
LSG_DEVI bool fp_canon_lt_p(const fp_t& c) {
  bool neg;
  (void)quad_sub_raw(c, p_limbs(), &neg);  // borrow of c - p
  return neg;
}
LSG_DEVI uint32_t fp_canon_parity(const fp_t& c) { return qbcast<0>(c.l0) & 1u; }

LSG_DEVI uint32_t be32(const uint8_t* q) {
  return ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
}
// the number formed by the 4*nlimbs big-endian bytes at b
LSG_DEVI fp_t fp_from_be_bytes(const uint8_t* b, int nlimbs) {
  int J = 3 * (int)qidx();
  uint32_t v0 = J < nlimbs ? be32(b + 4 * (nlimbs - 1 - J)) : 0u;
  uint32_t v1 = J + 1 < nlimbs ? be32(b + 4 * (nlimbs - 2 - J)) : 0u;
  uint32_t v2 = J + 2 < nlimbs ? be32(b + 4 * (nlimbs - 3 - J)) : 0u;
  return fp_t(v0, v1, v2);
}
LSG_DEVI void put_be32(uint8_t* q, uint32_t v) {
  q[0] = (uint8_t)(v >> 24);
  q[1] = (uint8_t)(v >> 16);
  q[2] = (uint8_t)(v >> 8);
  q[3] = (uint8_t)v;
}
LSG_DEVI void fp_to_be48(uint8_t* b, const fp_t& a) {
  int J = 3 * (int)qidx();
  put_be32(b + 44 - 4 * J, a.l0);
  put_be32(b + 40 - 4 * J, a.l1);
  put_be32(b + 36 - 4 * J, a.l2);
}
// clear the 3 ZCash flag bits (top of limb 11 = lane 3, register 2)
LSG_DEVI fp_t fp_mask_flags(const fp_t& a) { return fp_t(a.l0, a.l1, qidx() == 3 ? (a.l2 & 0x1fffffffu) : a.l2); }
LSG_DEVI fp_t fp_or_flags(const fp_t& a, uint32_t flags) {
  return fp_t(a.l0, a.l1, qidx() == 3 ? (a.l2 | (flags << 24)) : a.l2);
}

// ---- item-major global storage: a value of type T (a struct of W/3 fp_t) for item i lives at
// mem[(i*W + k)*4 + q], k = 0..W-1 (16 contiguous bytes per quad and word)
template <class T>
LSG_DEVI T lane_load(const uint32_t* __restrict__ mem, size_t item) {
  constexpr int W = sizeof(T) / 4;
  uint32_t w[W];
  const uint32_t* p = mem + item * W * 4 + qidx();
#pragma unroll
  for (int k = 0; k < W; k++) w[k] = p[k * 4];
  T v;
  __builtin_memcpy(&v, w, sizeof(T));
  return v;
}
template <class T>
LSG_DEVI void lane_store(uint32_t* __restrict__ mem, size_t item, const T& v) {
  constexpr int W = sizeof(T) / 4;
  uint32_t w[W];
  __builtin_memcpy(w, &v, sizeof(T));
  uint32_t* p = mem + item * W * 4 + qidx();
#pragma unroll
  for (int k = 0; k < W; k++) p[k * 4] = w[k];
}
template <class T>
constexpr size_t lane_words() {
  return sizeof(T) / 4 * 4;  // u32 words per item in global memory
}
