// Element backend: one thread holds a whole Fp element (12 x u32 Montgomery limbs).
// Used by the host build of the math (tests/native/hostcheck.hip) so that every stage of the
// generic tower / curve / pairing code can be checked against the oracle on a CPU; the
// product kernels use the limb-parallel backend (lsg_fp_lane.hpp) instead.
#pragma once
#include "lsg_constants.hpp"

#define LSG_ELEM_MODE 1

typedef fpc_t fp_t;

LSG_INL fp_t fp_zero() {
  fp_t r;
  for (int i = 0; i < 12; i++) r.l[i] = 0;
  return r;
}

LSG_INL bool fp_is_zero(const fp_t& a) {
  uint32_t acc = 0;
  for (int i = 0; i < 12; i++) acc |= a.l[i];
  return acc == 0;
}

LSG_INL bool fp_eq(const fp_t& a, const fp_t& b) {
  uint32_t acc = 0;
  for (int i = 0; i < 12; i++) acc |= a.l[i] ^ b.l[i];
  return acc == 0;
}

LSG_INL fp_t fp_select(bool c, const fp_t& a, const fp_t& b) {
  fp_t r;
  for (int i = 0; i < 12; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

LSG_INL fp_t fp_reduce_once(const fp_t& a) {
  fp_t s;
  uint32_t br = 0;
  for (int i = 0; i < 12; i++) s.l[i] = __builtin_subc(a.l[i], LSG_P[i], br, &br);
  return br ? a : s;
}

LSG_INL fp_t fp_add(const fp_t& a, const fp_t& b) {
  fp_t r;
  uint32_t c = 0;
  for (int i = 0; i < 12; i++) r.l[i] = __builtin_addc(a.l[i], b.l[i], c, &c);
  return fp_reduce_once(r);
}

LSG_INL fp_t fp_sub(const fp_t& a, const fp_t& b) {
  fp_t r, s;
  uint32_t br = 0;
  for (int i = 0; i < 12; i++) r.l[i] = __builtin_subc(a.l[i], b.l[i], br, &br);
  uint32_t c = 0;
  for (int i = 0; i < 12; i++) s.l[i] = __builtin_addc(r.l[i], LSG_P[i], c, &c);
  return br ? s : r;
}

LSG_INL fp_t fp_neg(const fp_t& a) { return fp_sub(fp_zero(), a); }
LSG_INL fp_t fp_canonical(const fp_t& a) { return a; }  // values are kept fully reduced

#ifdef LSG_COUNT_MULS  // host build only: exact Fp-multiplication counts per stage
extern unsigned long long lsg_mul_count;
#define LSG_COUNT_MUL() (lsg_mul_count++)
#else
#define LSG_COUNT_MUL() ((void)0)
#endif

// Montgomery product, "no-carry" CIOS (valid since p[11] < 2^31 - 1); inputs < p.
LSG_NOINL fp_t fp_mul(fp_t a, fp_t b) {
  LSG_COUNT_MUL();
  uint32_t t[12];
  for (int j = 0; j < 12; j++) t[j] = 0;
  for (int i = 0; i < 12; i++) {
    uint64_t s = (uint64_t)a.l[0] * b.l[i] + t[0];
    t[0] = (uint32_t)s;
    uint64_t A = s >> 32;
    uint32_t m = t[0] * LSG_N0P;
    uint64_t C = ((uint64_t)m * LSG_P[0] + t[0]) >> 32;
    for (int j = 1; j < 12; j++) {
      s = (uint64_t)a.l[j] * b.l[i] + t[j] + A;
      A = s >> 32;
      uint64_t s2 = (uint64_t)m * LSG_P[j] + (uint32_t)s + C;
      t[j - 1] = (uint32_t)s2;
      C = s2 >> 32;
    }
    t[11] = (uint32_t)(C + A);
  }
  fp_t r;
  for (int j = 0; j < 12; j++) r.l[j] = t[j];
  return fp_reduce_once(r);
}

LSG_INL void fp_mul2(fp_t& r0, fp_t& r1, const fp_t& a0, const fp_t& b0, const fp_t& a1, const fp_t& b1) {
  r0 = fp_mul(a0, b0);
  r1 = fp_mul(a1, b1);
}
LSG_INL void fp_mul9(fp_t* r, const fp_t* a, const fp_t* b) {
  for (int k = 0; k < 9; k++) r[k] = fp_mul(a[k], b[k]);
}
LSG_INL void fp_mul3(fp_t& r0, fp_t& r1, fp_t& r2, const fp_t& a0, const fp_t& b0, const fp_t& a1, const fp_t& b1,
                     const fp_t& a2, const fp_t& b2) {
  r0 = fp_mul(a0, b0);
  r1 = fp_mul(a1, b1);
  r2 = fp_mul(a2, b2);
}

// ---- canonical (non-Montgomery) predicates and byte I/O
LSG_INL bool fp_canon_gt_half(const fp_t& c) {
  uint32_t br = 0;
  for (int i = 0; i < 12; i++) (void)__builtin_subc(LSG_HALF_P_CANON[i], c.l[i], br, &br);
  return br != 0;
}
LSG_INL bool fp_canon_lt_p(const fp_t& c) {
  uint32_t br = 0;
  for (int i = 0; i < 12; i++) (void)__builtin_subc(c.l[i], LSG_P[i], br, &br);
  return br != 0;
}
LSG_INL uint32_t fp_canon_parity(const fp_t& c) { return c.l[0] & 1u; }

// the number formed by the 4*nlimbs big-endian bytes at b
LSG_INL fp_t fp_from_be_bytes(const uint8_t* b, int nlimbs) {
  fp_t r = fp_zero();
  for (int i = 0; i < nlimbs; i++) {
    const uint8_t* q = b + 4 * (nlimbs - 1 - i);
    r.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
  return r;
}
LSG_INL void fp_to_be48(uint8_t* b, const fp_t& a) {
  for (int i = 0; i < 12; i++) {
    uint8_t* q = b + 44 - 4 * i;
    q[0] = (uint8_t)(a.l[i] >> 24);
    q[1] = (uint8_t)(a.l[i] >> 16);
    q[2] = (uint8_t)(a.l[i] >> 8);
    q[3] = (uint8_t)a.l[i];
  }
}
// clear the 3 ZCash flag bits (top of limb 11)
LSG_INL fp_t fp_mask_flags(const fp_t& a) {
  fp_t r = a;
  r.l[11] &= 0x1fffffffu;
  return r;
}
LSG_INL fp_t fp_or_flags(const fp_t& a, uint32_t flags) {
  fp_t r = a;
  r.l[11] |= flags << 24;
  return r;
}
