// Lane backend: limb-parallel 381-bit Montgomery arithmetic for gfx950.
//
// One Fp element lives in one 16-lane DPP row: lane j (0..11) holds 32-bit limb j, lanes
// 12..15 hold 0.  A wave64 therefore carries four independent field elements (four
// signature sets), so a 4096-set batch occupies 1024 waves -- one per SIMD -- instead of the
// 64 waves a thread-per-set layout would give, and an Fp12 costs 12 VGPRs instead of 144.
//
// Montgomery multiplication is CIOS with the i-loop across time and the j-loop across lanes:
//   b_i   : DPP row_newbcast:i          m : row_newbcast:0 of (column 0) * n0'
//   a_j b_i, m p_j : one v_mad_u64_u32 each, per lane
//   the /2^32 shift of CIOS is a DPP row_shl:1 (lane j <- lane j+1)
// Carries are deferred in two 32-bit words per lane (ca from the a*b column, cb from the
// m*p column) so that every v_mad_u64_u32 addend stays < 2^33 and nothing overflows.  The
// final carry resolve and the conditional subtraction of p use a carry-lookahead on ballot
// masks: with G = lanes that generate and P = lanes that propagate a carry (disjoint),
// ((G|P) + G) ^ (G|P) ^ G is the carry INTO every lane, computed on the scalar unit for all
// four rows of the wave at once (rows cannot interact: lanes 12..15 never generate or
// propagate).
#pragma once
#include "lsg_constants.hpp"

#define LSG_LANE_MODE 1
#define LSG_GROUP 16  // lanes per field element
// the generic layers built on this backend are device-only code
#undef LSG_INL
#define LSG_INL __device__ __forceinline__
#undef LSG_NOINL
#define LSG_NOINL __device__ __noinline__

LSG_DEVI uint32_t lane16() { return __lane_id() & 15u; }
LSG_DEVI uint32_t row_base() { return __lane_id() & 48u; }

struct fp_t {
  uint32_t v;
  fp_t() = default;
  LSG_DEVI fp_t(const fpc_t& c) {
    uint32_t j = lane16();
    v = j < 12 ? c.l[j] : 0u;
  }
  LSG_DEVI explicit fp_t(uint32_t x) : v(x) {}
};

// ---- DPP helpers (control codes must be immediates)
template <int CTRL, bool BC>
LSG_DEVI uint32_t dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, BC);
}
LSG_DEVI uint32_t row_bcast(uint32_t x, int i) {
  switch (i) {
    case 0: return dpp<0x150, false>(x);
    case 1: return dpp<0x151, false>(x);
    case 2: return dpp<0x152, false>(x);
    case 3: return dpp<0x153, false>(x);
    case 4: return dpp<0x154, false>(x);
    case 5: return dpp<0x155, false>(x);
    case 6: return dpp<0x156, false>(x);
    case 7: return dpp<0x157, false>(x);
    case 8: return dpp<0x158, false>(x);
    case 9: return dpp<0x159, false>(x);
    case 10: return dpp<0x15a, false>(x);
    default: return dpp<0x15b, false>(x);
  }
}
LSG_DEVI uint32_t row_shl1(uint32_t x) { return dpp<0x101, true>(x); }  // lane j <- lane j+1 (15 <- 0)
LSG_DEVI uint32_t row_shr1(uint32_t x) { return dpp<0x111, true>(x); }  // lane j <- lane j-1 (0 <- 0)

// carry-lookahead over the wave: bit k of the result = carry INTO lane k
LSG_DEVI uint64_t carry_into(bool g, bool p) {
  uint64_t G = __ballot(g);
  uint64_t A = G | __ballot(p);
  return (A + G) ^ A ^ G;
}
LSG_DEVI uint32_t lane_bit(uint64_t m) { return (uint32_t)(m >> __lane_id()) & 1u; }
LSG_DEVI bool row_bit(uint64_t m, uint32_t k) { return ((m >> (row_base() + k)) & 1u) != 0; }
LSG_DEVI bool row_none(bool pred) { return ((__ballot(pred) >> row_base()) & 0xffffull) == 0; }

// The modulus limb p_j is needed by every add/sub/reduce: a global-memory load there put
// ~500 cycles of latency on each field addition.  Every lane kernel calls lsg_lane_setup()
// first; each wave writes the 16 limbs itself (identical values), and LDS operations of one
// wave complete in order, so no barrier is needed before p_limb() reads them.
__shared__ uint32_t lsg_lds_p[16];
LSG_DEVI void lsg_lane_setup() {
  uint32_t j = lane16();
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 12; k++) v = (j == (uint32_t)k) ? LSG_P[k] : v;  // literals, no memory
  lsg_lds_p[j] = v;
}
LSG_DEVI uint32_t p_limb() { return lsg_lds_p[lane16()]; }

// z < 2p (normalized limbs) -> z mod p
LSG_DEVI uint32_t lane_reduce_once(uint32_t z, uint32_t pj) {
  uint32_t j = lane16();
  uint64_t B = carry_into(z < pj, z == pj && j < 12);
  uint32_t d = z - pj - lane_bit(B);
  uint32_t r = row_bit(B, 12) ? z : d;  // borrow out of limb 11 <=> z < p
  return j < 12 ? r : 0u;
}

// N independent Montgomery products, interleaved so that one wave keeps N dependency
// chains in flight (the per-row chain is latency-bound: mad -> add -> DPP -> mul -> mad -> DPP).
template <int N>
LSG_DEVI void lane_mont_mul_n(const uint32_t* a, const uint32_t* b, uint32_t* r) {
  const uint32_t pj = p_limb();
  uint32_t x[N], ca[N], cb[N];
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = ca[k] = cb[k] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
#pragma unroll
    for (int k = 0; k < N; k++) {
      uint32_t bi = row_bcast(b[k], i);
      // 33-bit addends built with a 32-bit add + carry bit (v_add_co / v_addc), no zero-extends
      uint32_t tl = x[k] + ca[k];
      uint32_t th = tl < ca[k];
      uint64_t s = (uint64_t)a[k] * bi + (((uint64_t)th << 32) | tl);
      uint32_t sl = (uint32_t)s;
      uint32_t t2l = sl + cb[k];
      uint32_t t2h = t2l < cb[k];
      uint32_t m = row_bcast(t2l, 0) * LSG_N0P;
      uint64_t u = (uint64_t)m * pj + (((uint64_t)t2h << 32) | t2l);
      x[k] = row_shl1((uint32_t)u);
      ca[k] = (uint32_t)(s >> 32);
      cb[k] = (uint32_t)(u >> 32);
    }
  }
  // resolve the deferred carries: value = sum_j (x_j + ca_j + cb_j) 2^(32 j) < 2p
#pragma unroll
  for (int k = 0; k < N; k++) {
    uint64_t y = (uint64_t)x[k] + ca[k] + cb[k];
    uint64_t z = (uint64_t)(uint32_t)y + row_shr1((uint32_t)(y >> 32));
    uint32_t zl = (uint32_t)z;
    zl += lane_bit(carry_into((z >> 32) != 0, zl == 0xffffffffu));
    r[k] = lane_reduce_once(zl, pj);
  }
}

typedef uint32_t lsg_u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t lsg_u32x4 __attribute__((ext_vector_type(4)));

LSG_DEVNOINL uint32_t lane_mont_mul(uint32_t a, uint32_t b) {
  uint32_t r;
  lane_mont_mul_n<1>(&a, &b, &r);
  return r;
}
LSG_DEVNOINL lsg_u32x2 lane_mont_mul2(lsg_u32x2 a, lsg_u32x2 b) {
  uint32_t aa[2] = {a.x, a.y}, bb[2] = {b.x, b.y}, r[2];
  lane_mont_mul_n<2>(aa, bb, r);
  lsg_u32x2 o;
  o.x = r[0];
  o.y = r[1];
  return o;
}
LSG_DEVNOINL lsg_u32x4 lane_mont_mul3(lsg_u32x4 a, lsg_u32x4 b) {
  uint32_t aa[3] = {a.x, a.y, a.z}, bb[3] = {b.x, b.y, b.z}, r[3];
  lane_mont_mul_n<3>(aa, bb, r);
  lsg_u32x4 o;
  o.x = r[0];
  o.y = r[1];
  o.z = r[2];
  o.w = 0;
  return o;
}

typedef uint32_t lsg_u32x16 __attribute__((ext_vector_type(16)));
// nine independent products (three Fp2 Karatsuba products) per call
LSG_DEVNOINL lsg_u32x16 lane_mont_mul9(lsg_u32x16 a, lsg_u32x16 b) {
  uint32_t aa[9], bb[9], r[9];
#pragma unroll
  for (int k = 0; k < 9; k++) {
    aa[k] = a[k];
    bb[k] = b[k];
  }
  lane_mont_mul_n<9>(aa, bb, r);
  lsg_u32x16 o;
#pragma unroll
  for (int k = 0; k < 16; k++) o[k] = k < 9 ? r[k] : 0u;
  return o;
}

// ---- one item per wave: the four rows of a wave hold the same item, and a batch of N
// independent products (fp_mul_list, lsg_tower.hpp) is split over them: row q computes
// products q, q + 4, ... (M = ceil(N/4) per row, in one interleaved call where possible),
// then every row collects all N results with ds_bpermute.  Everything outside the batches
// runs replicated in the four rows, so every row keeps the whole item state.  The serial
// per-group stages (final exponentiation, signature-side Miller loop) have one item per
// group: a row per item left three quarters of their one wave idle.
#ifndef LSG_ROWS_PER_ITEM
#define LSG_ROWS_PER_ITEM 4
#endif
#if LSG_ROWS_PER_ITEM == 4
#define LSG_ROW_SPLIT 1
LSG_DEVI uint32_t row_q() { return (__lane_id() >> 4) & 3u; }
// M independent products of lane values, in as few interleaved leaf calls as possible
template <int M>
LSG_DEVI void lane_mul_chunks(uint32_t* o, const uint32_t* a, const uint32_t* b) {
  int k = 0;
#pragma unroll
  for (; k + 9 <= M; k += 9) {
    lsg_u32x16 x, y;
#pragma unroll
    for (int t = 0; t < 16; t++) {
      x[t] = t < 9 ? a[k + t] : 0u;
      y[t] = t < 9 ? b[k + t] : 0u;
    }
    lsg_u32x16 z = lane_mont_mul9(x, y);
#pragma unroll
    for (int t = 0; t < 9; t++) o[k + t] = z[t];
  }
#pragma unroll
  for (; k + 3 <= M; k += 3) {
    lsg_u32x4 x, y;
    x.x = a[k];
    x.y = a[k + 1];
    x.z = a[k + 2];
    x.w = 0;
    y.x = b[k];
    y.y = b[k + 1];
    y.z = b[k + 2];
    y.w = 0;
    lsg_u32x4 z = lane_mont_mul3(x, y);
    o[k] = z.x;
    o[k + 1] = z.y;
    o[k + 2] = z.z;
  }
  if (M - k == 2) {
    lsg_u32x2 x, y;
    x.x = a[k];
    x.y = a[k + 1];
    y.x = b[k];
    y.y = b[k + 1];
    lsg_u32x2 z = lane_mont_mul2(x, y);
    o[k] = z.x;
    o[k + 1] = z.y;
  } else if (M - k == 1) {
    o[k] = lane_mont_mul(a[k], b[k]);
  }
}
template <int N>
LSG_DEVI void lane_mul_rows(uint32_t* r, const uint32_t* x, const uint32_t* y) {
  constexpr int M = (N + 3) / 4;
  const uint32_t q = row_q();
  uint32_t a[M], b[M], o[M];
#pragma unroll
  for (int j = 0; j < M; j++) {
    // row q's operands of product 4j + q (a row past the end repeats product 4j)
    uint32_t av = x[4 * j], bv = y[4 * j];
#pragma unroll
    for (int t = 1; t < 4; t++) {
      if (4 * j + t < N) {
        av = q == (uint32_t)t ? x[4 * j + t] : av;
        bv = q == (uint32_t)t ? y[4 * j + t] : bv;
      }
    }
    a[j] = av;
    b[j] = bv;
  }
  lane_mul_chunks<M>(o, a, b);
  const int l16 = (int)lane16();
#pragma unroll
  for (int k = 0; k < N; k++)
    r[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((l16 + 16 * (k & 3)) << 2, (int)o[k >> 2]);
}
#endif

LSG_DEVI uint32_t lane_add(uint32_t a, uint32_t b) {
  uint64_t s = (uint64_t)a + b;
  uint32_t z = (uint32_t)s;
  z += lane_bit(carry_into((s >> 32) != 0, z == 0xffffffffu));
  return lane_reduce_once(z, p_limb());
}

LSG_DEVI uint32_t lane_sub(uint32_t a, uint32_t b) {
  uint32_t j = lane16();
  uint64_t B = carry_into(a < b, a == b && j < 12);
  uint32_t d = a - b - lane_bit(B);
  bool neg = row_bit(B, 12);
  uint64_t s = (uint64_t)d + p_limb();
  uint32_t e = (uint32_t)s;
  e += lane_bit(carry_into((s >> 32) != 0, e == 0xffffffffu && j < 12));
  uint32_t r = neg ? e : d;
  return j < 12 ? r : 0u;
}

// ------------------------------------------------------------------ Fp API
LSG_DEVI fp_t fp_zero() { return fp_t(0u); }
LSG_DEVI bool fp_is_zero(const fp_t& a) { return row_none(a.v != 0); }
LSG_DEVI bool fp_eq(const fp_t& a, const fp_t& b) { return row_none(a.v != b.v); }
LSG_DEVI fp_t fp_select(bool c, const fp_t& a, const fp_t& b) { return fp_t(c ? a.v : b.v); }
LSG_DEVI fp_t fp_add(const fp_t& a, const fp_t& b) { return fp_t(lane_add(a.v, b.v)); }
LSG_DEVI fp_t fp_sub(const fp_t& a, const fp_t& b) { return fp_t(lane_sub(a.v, b.v)); }
LSG_DEVI fp_t fp_neg(const fp_t& a) { return fp_t(lane_sub(0u, a.v)); }
LSG_DEVI fp_t fp_canonical(const fp_t& a) { return a; }  // values are kept fully reduced
LSG_DEVI fp_t fp_mul(const fp_t& a, const fp_t& b) { return fp_t(lane_mont_mul(a.v, b.v)); }
LSG_DEVI void fp_mul9(fp_t* r, const fp_t* a, const fp_t* b) {
  lsg_u32x16 x, y;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    x[k] = k < 9 ? a[k].v : 0u;
    y[k] = k < 9 ? b[k].v : 0u;
  }
  lsg_u32x16 o = lane_mont_mul9(x, y);
#pragma unroll
  for (int k = 0; k < 9; k++) r[k] = fp_t(o[k]);
}
// two / three independent products with interleaved chains
LSG_DEVI void fp_mul2(fp_t& r0, fp_t& r1, const fp_t& a0, const fp_t& b0, const fp_t& a1, const fp_t& b1) {
  lsg_u32x2 a, b;
  a.x = a0.v;
  a.y = a1.v;
  b.x = b0.v;
  b.y = b1.v;
  lsg_u32x2 r = lane_mont_mul2(a, b);
  r0 = fp_t(r.x);
  r1 = fp_t(r.y);
}
LSG_DEVI void fp_mul3(fp_t& r0, fp_t& r1, fp_t& r2, const fp_t& a0, const fp_t& b0, const fp_t& a1, const fp_t& b1,
                      const fp_t& a2, const fp_t& b2) {
  lsg_u32x4 a, b;
  a.x = a0.v;
  a.y = a1.v;
  a.z = a2.v;
  a.w = 0;
  b.x = b0.v;
  b.y = b1.v;
  b.z = b2.v;
  b.w = 0;
  lsg_u32x4 r = lane_mont_mul3(a, b);
  r0 = fp_t(r.x);
  r1 = fp_t(r.y);
  r2 = fp_t(r.z);
}

#ifdef LSG_ROW_SPLIT
template <int N>
LSG_DEVI void fp_mul_list_rows(fp_t* r, const fp_t* x, const fp_t* y) {
  uint32_t xv[N], yv[N], rv[N];
#pragma unroll
  for (int k = 0; k < N; k++) {
    xv[k] = x[k].v;
    yv[k] = y[k].v;
  }
  lane_mul_rows<N>(rv, xv, yv);
#pragma unroll
  for (int k = 0; k < N; k++) r[k] = fp_t(rv[k]);
}
#endif

// ---- canonical predicates and byte I/O (row-uniform results)
LSG_DEVI bool fp_canon_gt_half(const fp_t& c) {
  uint32_t j = lane16();
  uint32_t h = j < 12 ? LSG_HALF_P_CANON[j] : 0u;
  return row_bit(carry_into(h < c.v, h == c.v && j < 12), 12);  // borrow of HALF - c
}
LSG_DEVI bool fp_canon_lt_p(const fp_t& c) {
  uint32_t j = lane16();
  uint32_t pj = p_limb();
  return row_bit(carry_into(c.v < pj, c.v == pj && j < 12), 12);  // borrow of c - p
}
LSG_DEVI uint32_t fp_canon_parity(const fp_t& c) { return row_bcast(c.v, 0) & 1u; }

LSG_DEVI fp_t fp_from_be_bytes(const uint8_t* b, int nlimbs) {
  uint32_t j = lane16();
  uint32_t v = 0;
  if ((int)j < nlimbs) {
    const uint8_t* q = b + 4 * (nlimbs - 1 - (int)j);
    v = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
  return fp_t(v);
}
LSG_DEVI void fp_to_be48(uint8_t* b, const fp_t& a) {
  uint32_t j = lane16();
  if (j < 12) {
    uint8_t* q = b + 44 - 4 * j;
    q[0] = (uint8_t)(a.v >> 24);
    q[1] = (uint8_t)(a.v >> 16);
    q[2] = (uint8_t)(a.v >> 8);
    q[3] = (uint8_t)a.v;
  }
}
LSG_DEVI fp_t fp_mask_flags(const fp_t& a) { return fp_t(lane16() == 11 ? (a.v & 0x1fffffffu) : a.v); }
// OR ZCash flag bits into the most significant byte (canonical value, for serialization)
LSG_DEVI fp_t fp_or_flags(const fp_t& a, uint32_t flags) {
  return fp_t(lane16() == 11 ? (a.v | (flags << 24)) : a.v);
}

// ---- item-major global storage of lane-form values: a value of type T (a struct of W
// fp_t) for item i lives at mem[(i*W + k)*16 + lane], k = 0..W-1 (coalesced 64-byte rows).
template <class T>
LSG_DEVI T lane_load(const uint32_t* __restrict__ mem, size_t item) {
  constexpr int W = sizeof(T) / 4;
  uint32_t w[W];
  const uint32_t* p = mem + item * W * 16 + lane16();
#pragma unroll
  for (int k = 0; k < W; k++) w[k] = p[k * 16];
  T v;
  __builtin_memcpy(&v, w, sizeof(T));
  return v;
}
template <class T>
LSG_DEVI void lane_store(uint32_t* __restrict__ mem, size_t item, const T& v) {
  constexpr int W = sizeof(T) / 4;
  uint32_t w[W];
  __builtin_memcpy(w, &v, sizeof(T));
  uint32_t* p = mem + item * W * 16 + lane16();
#pragma unroll
  for (int k = 0; k < W; k++) p[k * 16] = w[k];
}
template <class T>
constexpr size_t lane_words() {
  return sizeof(T) / 4 * 16;  // u32 words per item in global memory
}
