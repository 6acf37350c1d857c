// BLS12-381 base-field tower for gfx950: Fp (12 x u32 Montgomery limbs), Fp2, Fp6, Fp12.
//
// Replaces the field layer of supranational blst (un-vendored; reached through
// @chainsafe/blst@0.2.8, /root/reference/yarn.lock:492-497) that
// packages/beacon-node/src/chain/bls/maybeBatch.ts:18,37 drives.  Written for the
// 32-bit integer VALU: every 32x32->64 multiply-accumulate is a v_mad_u64_u32.
//
// Tower (same as the oracle, oracle/fields.py):
//   Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3-(1+u)), Fp12 = Fp6[w]/(w^2-v).
// All values are kept fully reduced (< p) in Montgomery form, so two equal field
// elements are equal limb for limb and every stage is bit-comparable with the oracle.
//
// Code-size policy: Montgomery multiplication is a real (non-inlined) function so the
// Fp12 / G2 code built on it stays within the instruction cache; additions inline.
#pragma once
#include <stdint.h>

#define LSG_INL __host__ __device__ __forceinline__
#define LSG_NOINL __host__ __device__ __noinline__
#define LSG_CONST static constexpr

struct fp_t {
  uint32_t l[12];
};
struct fp2_t {
  fp_t c0, c1;
};
struct fp6_t {
  fp2_t c0, c1, c2;
};
struct fp12_t {
  fp6_t c0, c1;
};

#include "lsg_constants.hpp"

// ------------------------------------------------------------------ Fp
LSG_INL fp_t fp_zero() {
  fp_t r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = 0;
  return r;
}

LSG_INL fp_t fp_one() { return FP_ONE; }

LSG_INL bool fp_is_zero(const fp_t& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc |= a.l[i];
  return acc == 0;
}

LSG_INL bool fp_eq(const fp_t& a, const fp_t& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc |= a.l[i] ^ b.l[i];
  return acc == 0;
}

LSG_INL fp_t fp_select(bool c, const fp_t& a, const fp_t& b) {
  fp_t r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

// r = a - p if a >= p else a   (a < 2p)
LSG_INL fp_t fp_reduce_once(const fp_t& a) {
  fp_t s;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s.l[i] = __builtin_subc(a.l[i], LSG_P[i], br, &br);
  return br ? a : s;
}

LSG_INL fp_t fp_add(const fp_t& a, const fp_t& b) {
  fp_t r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = __builtin_addc(a.l[i], b.l[i], c, &c);
  return fp_reduce_once(r);  // a + b < 2p < 2^382: no carry out of limb 11
}

LSG_INL fp_t fp_sub(const fp_t& a, const fp_t& b) {
  fp_t r, s;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = __builtin_subc(a.l[i], b.l[i], br, &br);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s.l[i] = __builtin_addc(r.l[i], LSG_P[i], c, &c);
  return br ? s : r;
}

LSG_INL fp_t fp_dbl(const fp_t& a) { return fp_add(a, a); }

LSG_INL fp_t fp_neg(const fp_t& a) {
  fp_t r;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = __builtin_subc(LSG_P[i], a.l[i], br, &br);
  return fp_is_zero(a) ? a : r;
}

// Montgomery product a*b/R mod p, "no-carry" CIOS (valid since p[11] < 2^31 - 1).
// Inputs: a, b < p.  The call boundary uses 12-wide vectors, which the AMDGPU calling
// convention passes and returns in VGPRs (a struct return would go through scratch).
typedef uint32_t lsg_u32x12 __attribute__((ext_vector_type(12)));

LSG_NOINL lsg_u32x12 fp_mul_core(lsg_u32x12 a, lsg_u32x12 b) {
  uint32_t t[12];
#pragma unroll
  for (int j = 0; j < 12; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t s = (uint64_t)a[0] * b[i] + t[0];
    t[0] = (uint32_t)s;
    uint64_t A = s >> 32;
    uint32_t m = t[0] * LSG_N0P;
    uint64_t C = ((uint64_t)m * LSG_P[0] + t[0]) >> 32;
#pragma unroll
    for (int j = 1; j < 12; j++) {
      s = (uint64_t)a[j] * b[i] + t[j] + A;
      A = s >> 32;
      uint64_t s2 = (uint64_t)m * LSG_P[j] + (uint32_t)s + C;
      t[j - 1] = (uint32_t)s2;
      C = s2 >> 32;
    }
    t[11] = (uint32_t)(C + A);
  }
  // conditional final subtraction
  uint32_t d[12];
  uint32_t br = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) d[j] = __builtin_subc(t[j], LSG_P[j], br, &br);
  lsg_u32x12 r;
#pragma unroll
  for (int j = 0; j < 12; j++) r[j] = br ? t[j] : d[j];
  return r;
}

LSG_INL fp_t fp_mul(const fp_t& a, const fp_t& b) {
  lsg_u32x12 x, y;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    x[i] = a.l[i];
    y[i] = b.l[i];
  }
  lsg_u32x12 r = fp_mul_core(x, y);
  fp_t o;
#pragma unroll
  for (int i = 0; i < 12; i++) o.l[i] = r[i];
  return o;
}

LSG_INL fp_t fp_sqr(const fp_t& a) { return fp_mul(a, a); }

LSG_INL fp_t fp_to_mont(const fp_t& a) { return fp_mul(a, FP_R2); }
LSG_INL fp_t fp_from_mont(const fp_t& a) { return fp_mul(a, FP_ONE_CANON); }

// a^e for a fixed public exponent (12 limbs, MSB first square-and-multiply; the exponent
// is the same for every lane, so the branch is uniform).
LSG_NOINL fp_t fp_pow_fixed(fp_t a, const uint32_t* e) {
  fp_t r = FP_ONE;
  bool started = false;
  for (int w = 11; w >= 0; w--) {
    uint32_t word = e[w];
    for (int b = 31; b >= 0; b--) {
      if (started) r = fp_sqr(r);
      if ((word >> b) & 1u) {
        r = started ? fp_mul(r, a) : a;
        started = true;
      }
    }
  }
  return r;
}

LSG_INL fp_t fp_inv(const fp_t& a) { return fp_pow_fixed(a, LSG_EXP_P_MINUS_2); }  // inv(0) = 0

// canonical (non-Montgomery) comparisons / parity
LSG_INL bool fp_canon_gt_half(const fp_t& canon) {
  // canon > (p-1)/2 ?
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) (void)__builtin_subc(LSG_HALF_P_CANON[i], canon.l[i], br, &br);
  return br != 0;
}

// ------------------------------------------------------------------ Fp2
LSG_INL fp2_t fp2_make(const fp_t& a, const fp_t& b) {
  fp2_t r;
  r.c0 = a;
  r.c1 = b;
  return r;
}
LSG_INL fp2_t fp2_zero() { return fp2_make(fp_zero(), fp_zero()); }
LSG_INL fp2_t fp2_one() { return fp2_make(FP_ONE, fp_zero()); }
LSG_INL bool fp2_is_zero(const fp2_t& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
LSG_INL bool fp2_eq(const fp2_t& a, const fp2_t& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
LSG_INL fp2_t fp2_select(bool c, const fp2_t& a, const fp2_t& b) {
  return fp2_make(fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1));
}
LSG_INL fp2_t fp2_add(const fp2_t& a, const fp2_t& b) { return fp2_make(fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)); }
LSG_INL fp2_t fp2_sub(const fp2_t& a, const fp2_t& b) { return fp2_make(fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)); }
LSG_INL fp2_t fp2_dbl(const fp2_t& a) { return fp2_add(a, a); }
LSG_INL fp2_t fp2_neg(const fp2_t& a) { return fp2_make(fp_neg(a.c0), fp_neg(a.c1)); }
LSG_INL fp2_t fp2_conj(const fp2_t& a) { return fp2_make(a.c0, fp_neg(a.c1)); }

LSG_INL fp2_t fp2_mul(const fp2_t& a, const fp2_t& b) {
  fp_t t0 = fp_mul(a.c0, b.c0);
  fp_t t1 = fp_mul(a.c1, b.c1);
  fp_t t2 = fp_mul(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return fp2_make(fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1));
}

LSG_INL fp2_t fp2_sqr(const fp2_t& a) {
  // (a0 + a1)(a0 - a1), 2 a0 a1
  fp_t t0 = fp_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
  fp_t t1 = fp_mul(a.c0, a.c1);
  return fp2_make(t0, fp_dbl(t1));
}

LSG_INL fp2_t fp2_mul_fp(const fp2_t& a, const fp_t& k) { return fp2_make(fp_mul(a.c0, k), fp_mul(a.c1, k)); }

// (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
LSG_INL fp2_t fp2_mul_xi(const fp2_t& a) { return fp2_make(fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)); }

LSG_INL fp_t fp2_norm(const fp2_t& a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }

LSG_INL fp2_t fp2_inv(const fp2_t& a) {
  fp_t ni = fp_inv(fp2_norm(a));
  return fp2_make(fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni)));
}

// 12 * a (for b3 = 3 * 4(1+u) multiplications)
LSG_INL fp_t fp_mul12(const fp_t& a) {
  fp_t a2 = fp_dbl(a);
  fp_t a4 = fp_dbl(a2);
  fp_t a8 = fp_dbl(a4);
  return fp_add(a8, a4);
}
LSG_INL fp2_t fp2_mul_b3(const fp2_t& a) {
  fp2_t t = fp2_mul_xi(a);
  return fp2_make(fp_mul12(t.c0), fp_mul12(t.c1));
}

// RFC 9380 sgn0 for Fp2 (a in Montgomery form)
LSG_INL uint32_t fp2_sgn0(const fp2_t& a) {
  fp_t c0 = fp_from_mont(a.c0), c1 = fp_from_mont(a.c1);
  uint32_t sign0 = c0.l[0] & 1u;
  uint32_t zero0 = fp_is_zero(c0) ? 1u : 0u;
  uint32_t sign1 = c1.l[0] & 1u;
  return sign0 | (zero0 & sign1);
}

// ZCash "lexicographically largest" flag of y in Fp2 (Montgomery form)
LSG_INL bool fp2_lexi_largest(const fp2_t& y) {
  fp_t c0 = fp_from_mont(y.c0), c1 = fp_from_mont(y.c1);
  return fp_is_zero(c1) ? fp_canon_gt_half(c0) : fp_canon_gt_half(c1);
}

// Square root in Fp2 via the norm: two fixed Fp exponentiations.
//   n = a0^2 + a1^2, s = sqrt(n);  c = (a0 + s)/2 (c = a0 if that is 0);  t = c^((p-3)/4)
//   c square:      root = (c t, a1 t / 2)
//   c non-square:  root = (a1 t / 2, -c t)
// Returns false when a is not a square.  Which of the two roots comes out does not matter:
// every caller fixes the sign afterwards.
LSG_INL bool fp2_sqrt(fp2_t& out, const fp2_t& a) {
  fp_t n = fp2_norm(a);
  fp_t s = fp_pow_fixed(n, LSG_EXP_P_PLUS_1_DIV_4);
  bool ok = fp_eq(fp_sqr(s), n);
  fp_t c = fp_mul(fp_add(a.c0, s), FP_HALF);
  c = fp_select(fp_is_zero(c), a.c0, c);
  fp_t t = fp_pow_fixed(c, LSG_EXP_P_MINUS_3_DIV_4);
  fp_t ct = fp_mul(c, t);
  bool c_sq = fp_eq(fp_mul(ct, t), FP_ONE) || fp_is_zero(c);
  fp_t h = fp_mul(fp_mul(a.c1, t), FP_HALF);
  fp2_t r = c_sq ? fp2_make(ct, h) : fp2_make(h, fp_neg(ct));
  ok = ok && fp2_eq(fp2_sqr(r), a);
  out = r;
  return ok;
}

// ------------------------------------------------------------------ Fp6
LSG_INL fp6_t fp6_make(const fp2_t& a, const fp2_t& b, const fp2_t& c) {
  fp6_t r;
  r.c0 = a;
  r.c1 = b;
  r.c2 = c;
  return r;
}
LSG_INL fp6_t fp6_zero() { return fp6_make(fp2_zero(), fp2_zero(), fp2_zero()); }
LSG_INL fp6_t fp6_one() { return fp6_make(fp2_one(), fp2_zero(), fp2_zero()); }
LSG_INL fp6_t fp6_add(const fp6_t& a, const fp6_t& b) {
  return fp6_make(fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2));
}
LSG_INL fp6_t fp6_sub(const fp6_t& a, const fp6_t& b) {
  return fp6_make(fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2));
}
LSG_INL fp6_t fp6_neg(const fp6_t& a) { return fp6_make(fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)); }

// (a0 + a1 v + a2 v^2)(b0 + b1 v + b2 v^2), schoolbook as in oracle/fields.py:f6_mul
LSG_NOINL fp6_t fp6_mul(fp6_t a, fp6_t b) {
  fp2_t t0 = fp2_mul(a.c0, b.c0);
  fp2_t t1 = fp2_mul(a.c1, b.c1);
  fp2_t t2 = fp2_mul(a.c2, b.c2);
  fp2_t c0 = fp2_add(t0, fp2_mul_xi(fp2_add(fp2_mul(a.c1, b.c2), fp2_mul(a.c2, b.c1))));
  fp2_t c1 = fp2_add(fp2_add(fp2_mul(a.c0, b.c1), fp2_mul(a.c1, b.c0)), fp2_mul_xi(t2));
  fp2_t c2 = fp2_add(fp2_add(fp2_mul(a.c0, b.c2), t1), fp2_mul(a.c2, b.c0));
  return fp6_make(c0, c1, c2);
}

LSG_INL fp6_t fp6_mul_v(const fp6_t& a) { return fp6_make(fp2_mul_xi(a.c2), a.c0, a.c1); }

// (a0 + a1 v + a2 v^2)(b0 + b1 v)   -- oracle/pairing.py:f6_mul_01
LSG_NOINL fp6_t fp6_mul_01(fp6_t a, fp2_t b0, fp2_t b1) {
  fp2_t t0 = fp2_mul(a.c0, b0);
  fp2_t t1 = fp2_mul(a.c1, b1);
  fp2_t c0 = fp2_add(fp2_mul_xi(fp2_mul(a.c2, b1)), t0);
  fp2_t c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b0, b1)), t0), t1);
  fp2_t c2 = fp2_add(fp2_mul(a.c2, b0), t1);
  return fp6_make(c0, c1, c2);
}

// (a0 + a1 v + a2 v^2)(b1 v)   -- oracle/pairing.py:f6_mul_1
LSG_INL fp6_t fp6_mul_1(const fp6_t& a, const fp2_t& b1) {
  return fp6_make(fp2_mul_xi(fp2_mul(a.c2, b1)), fp2_mul(a.c0, b1), fp2_mul(a.c1, b1));
}

LSG_NOINL fp6_t fp6_inv(fp6_t a) {
  fp2_t t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  fp2_t t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  fp2_t t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  fp2_t den = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  fp2_t di = fp2_inv(den);
  return fp6_make(fp2_mul(t0, di), fp2_mul(t1, di), fp2_mul(t2, di));
}

// ------------------------------------------------------------------ Fp12
LSG_INL fp12_t fp12_make(const fp6_t& a, const fp6_t& b) {
  fp12_t r;
  r.c0 = a;
  r.c1 = b;
  return r;
}
LSG_INL fp12_t fp12_one() { return fp12_make(fp6_one(), fp6_zero()); }
LSG_INL bool fp12_is_one(const fp12_t& a) {
  return fp2_eq(a.c0.c0, fp2_one()) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) && fp2_is_zero(a.c1.c0) &&
         fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
}
LSG_INL fp12_t fp12_conj(const fp12_t& a) { return fp12_make(a.c0, fp6_neg(a.c1)); }

LSG_NOINL fp12_t fp12_mul(fp12_t a, fp12_t b) {
  fp6_t t0 = fp6_mul(a.c0, b.c0);
  fp6_t t1 = fp6_mul(a.c1, b.c1);
  fp6_t c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), t0), t1);
  fp6_t c0 = fp6_add(t0, fp6_mul_v(t1));
  return fp12_make(c0, c1);
}

// (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w
LSG_NOINL fp12_t fp12_sqr(fp12_t a) {
  fp6_t t = fp6_mul(a.c0, a.c1);
  fp6_t c0 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1))), t), fp6_mul_v(t));
  return fp12_make(c0, fp6_add(t, t));
}

// f * ((l00 + l01 v) + (l11 v) w)   -- oracle/pairing.py:f12_mul_line
LSG_NOINL fp12_t fp12_mul_line(fp12_t f, fp2_t l00, fp2_t l01, fp2_t l11) {
  fp6_t t0 = fp6_mul_01(f.c0, l00, l01);
  fp6_t t1 = fp6_mul_1(f.c1, l11);
  fp6_t s = fp6_add(f.c0, f.c1);
  fp6_t c1 = fp6_sub(fp6_sub(fp6_mul_01(s, l00, fp2_add(l01, l11)), t0), t1);
  fp6_t c0 = fp6_add(t0, fp6_mul_v(t1));
  return fp12_make(c0, c1);
}

LSG_NOINL fp12_t fp12_inv(fp12_t a) {
  fp6_t t = fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_v(fp6_mul(a.c1, a.c1)));
  fp6_t ti = fp6_inv(t);
  return fp12_make(fp6_mul(a.c0, ti), fp6_neg(fp6_mul(a.c1, ti)));
}

// a^p : coefficient of w^j is conj(c_j) * gamma1_j; w^j order (c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2)
LSG_NOINL fp12_t fp12_frob(fp12_t a) {
  fp12_t r;
  r.c0.c0 = fp2_conj(a.c0.c0);
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), FROB1_G1);
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), FROB1_G2);
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), FROB1_G3);
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), FROB1_G4);
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), FROB1_G5);
  return r;
}

LSG_NOINL fp12_t fp12_frob2(fp12_t a) {
  fp12_t r;
  r.c0.c0 = a.c0.c0;
  r.c1.c0 = fp2_mul(a.c1.c0, FROB2_G1);
  r.c0.c1 = fp2_mul(a.c0.c1, FROB2_G2);
  r.c1.c1 = fp2_mul(a.c1.c1, FROB2_G3);
  r.c0.c2 = fp2_mul(a.c0.c2, FROB2_G4);
  r.c1.c2 = fp2_mul(a.c1.c2, FROB2_G5);
  return r;
}
