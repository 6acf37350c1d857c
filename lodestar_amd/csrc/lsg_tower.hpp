// BLS12-381 extension tower, generic over the Fp backend (include lsg_fp_lane.hpp or
// lsg_fp_elem.hpp first).
//
// Replaces the field layer of supranational blst (un-vendored; reached through
// @chainsafe/blst@0.2.8, /root/reference/yarn.lock:492-497) that
// packages/beacon-node/src/chain/bls/maybeBatch.ts:18,37 drives.
//   Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3-(1+u)), Fp12 = Fp6[w]/(w^2-v)
// Same tower and the same formulas as the oracle (oracle/fields.py, oracle/pairing.py).
// Values are kept fully reduced (< p) in Montgomery form, so equal field elements are equal
// limb for limb and every stage is bit-comparable with the oracle.
#pragma once

#ifndef LSG_BIGFN
#define LSG_BIGFN LSG_NOINL
#endif

// ------------------------------------------------------------------ Fp (backend-generic)
LSG_INL fp_t fp_one() { return fp_t(FP_ONE); }
LSG_INL fp_t fp_dbl(const fp_t& a) { return fp_add(a, a); }
LSG_INL fp_t fp_sqr(const fp_t& a) { return fp_mul(a, a); }
LSG_INL fp_t fp_to_mont(const fp_t& a) { return fp_mul(a, fp_t(FP_R2)); }
LSG_INL fp_t fp_from_mont(const fp_t& a) { return fp_mul(a, fp_t(FP_ONE_CANON)); }
LSG_INL fp_t fp_from_be48(const uint8_t* b) { return fp_from_be_bytes(b, 12); }

// a^e for a fixed public exponent (MSB-first square-and-multiply; uniform branches)
LSG_BIGFN fp_t fp_pow_fixed(fp_t a, const uint32_t* e) {
  fp_t r = fp_one();
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

LSG_INL fp_t fp_mul12(const fp_t& a) {
  fp_t a2 = fp_dbl(a);
  fp_t a4 = fp_dbl(a2);
  fp_t a8 = fp_dbl(a4);
  return fp_add(a8, a4);
}

// ------------------------------------------------------------------ Fp2
struct fp2_t {
  fp_t c0, c1;
  fp2_t() = default;
  LSG_INL fp2_t(const fp_t& a, const fp_t& b) : c0(a), c1(b) {}
  LSG_INL fp2_t(const fp2c_t& c) : c0(c.c0), c1(c.c1) {}
};
struct fp6_t {
  fp2_t c0, c1, c2;
};
struct fp12_t {
  fp6_t c0, c1;
};

LSG_INL fp2_t fp2_make(const fp_t& a, const fp_t& b) { return fp2_t(a, b); }
LSG_INL fp2_t fp2_zero() { return fp2_t(fp_zero(), fp_zero()); }
LSG_INL fp2_t fp2_one() { return fp2_t(fp_one(), fp_zero()); }
LSG_INL bool fp2_is_zero(const fp2_t& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
LSG_INL bool fp2_eq(const fp2_t& a, const fp2_t& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
LSG_INL fp2_t fp2_select(bool c, const fp2_t& a, const fp2_t& b) {
  return fp2_t(fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1));
}
LSG_INL fp2_t fp2_add(const fp2_t& a, const fp2_t& b) { return fp2_t(fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)); }
LSG_INL fp2_t fp2_sub(const fp2_t& a, const fp2_t& b) { return fp2_t(fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)); }
LSG_INL fp2_t fp2_dbl(const fp2_t& a) { return fp2_add(a, a); }
LSG_INL fp2_t fp2_neg(const fp2_t& a) { return fp2_t(fp_neg(a.c0), fp_neg(a.c1)); }
LSG_INL fp2_t fp2_conj(const fp2_t& a) { return fp2_t(a.c0, fp_neg(a.c1)); }

// Karatsuba: 3 Fp multiplications
LSG_INL fp2_t fp2_mul(const fp2_t& a, const fp2_t& b) {
  fp_t t0 = fp_mul(a.c0, b.c0);
  fp_t t1 = fp_mul(a.c1, b.c1);
  fp_t t2 = fp_mul(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return fp2_t(fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1));
}

// (a0 + a1)(a0 - a1), 2 a0 a1
LSG_INL fp2_t fp2_sqr(const fp2_t& a) {
  fp_t t0 = fp_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
  fp_t t1 = fp_mul(a.c0, a.c1);
  return fp2_t(t0, fp_dbl(t1));
}

LSG_INL fp2_t fp2_mul_fp(const fp2_t& a, const fp_t& k) { return fp2_t(fp_mul(a.c0, k), fp_mul(a.c1, k)); }

// (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
LSG_INL fp2_t fp2_mul_xi(const fp2_t& a) { return fp2_t(fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)); }

LSG_INL fp_t fp2_norm(const fp2_t& a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }

LSG_INL fp2_t fp2_inv(const fp2_t& a) {
  fp_t ni = fp_inv(fp2_norm(a));
  return fp2_t(fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni)));
}

// 12 a (for b3 = 3 * 4(1+u))
LSG_INL fp2_t fp2_mul_b3(const fp2_t& a) {
  fp2_t t = fp2_mul_xi(a);
  return fp2_t(fp_mul12(t.c0), fp_mul12(t.c1));
}

// RFC 9380 sgn0 for Fp2 (a in Montgomery form)
LSG_INL uint32_t fp2_sgn0(const fp2_t& a) {
  fp_t c0 = fp_from_mont(a.c0), c1 = fp_from_mont(a.c1);
  uint32_t sign0 = fp_canon_parity(c0);
  uint32_t zero0 = fp_is_zero(c0) ? 1u : 0u;
  uint32_t sign1 = fp_canon_parity(c1);
  return sign0 | (zero0 & sign1);
}

// ZCash "lexicographically largest" flag of y in Fp2 (Montgomery form)
LSG_INL bool fp2_lexi_largest(const fp2_t& y) {
  fp_t c0 = fp_from_mont(y.c0), c1 = fp_from_mont(y.c1);
  return fp_is_zero(c1) ? fp_canon_gt_half(c0) : fp_canon_gt_half(c1);
}

// Square root in Fp2 via the norm (two fixed Fp exponentiations):
//   n = a0^2 + a1^2, s = sqrt(n);  c = (a0 + s)/2 (c = a0 if that is 0);  t = c^((p-3)/4)
//   c square:      root = (c t, a1 t / 2)
//   c non-square:  root = (a1 t / 2, -c t)
// Returns false when a is not a square.  Callers fix the root's sign afterwards.
LSG_BIGFN bool fp2_sqrt(fp2_t& out, fp2_t a) {
  fp_t n = fp2_norm(a);
  fp_t s = fp_pow_fixed(n, LSG_EXP_P_PLUS_1_DIV_4);
  bool ok = fp_eq(fp_sqr(s), n);
  fp_t c = fp_mul(fp_add(a.c0, s), fp_t(FP_HALF));
  c = fp_select(fp_is_zero(c), a.c0, c);
  fp_t t = fp_pow_fixed(c, LSG_EXP_P_MINUS_3_DIV_4);
  fp_t ct = fp_mul(c, t);
  bool c_sq = fp_eq(fp_mul(ct, t), fp_one()) || fp_is_zero(c);
  fp_t h = fp_mul(fp_mul(a.c1, t), fp_t(FP_HALF));
  fp2_t r = c_sq ? fp2_t(ct, h) : fp2_t(h, fp_neg(ct));
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

// schoolbook as oracle/fields.py:f6_mul
LSG_BIGFN fp6_t fp6_mul(fp6_t a, fp6_t b) {
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
LSG_BIGFN fp6_t fp6_mul_01(fp6_t a, fp2_t b0, fp2_t b1) {
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

LSG_BIGFN fp6_t fp6_inv(fp6_t a) {
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

LSG_BIGFN fp12_t fp12_mul(fp12_t a, fp12_t b) {
  fp6_t t0 = fp6_mul(a.c0, b.c0);
  fp6_t t1 = fp6_mul(a.c1, b.c1);
  fp6_t c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), t0), t1);
  fp6_t c0 = fp6_add(t0, fp6_mul_v(t1));
  return fp12_make(c0, c1);
}

// (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w
LSG_BIGFN fp12_t fp12_sqr(fp12_t a) {
  fp6_t t = fp6_mul(a.c0, a.c1);
  fp6_t c0 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1))), t), fp6_mul_v(t));
  return fp12_make(c0, fp6_add(t, t));
}

// f * ((l00 + l01 v) + (l11 v) w)   -- oracle/pairing.py:f12_mul_line
LSG_BIGFN fp12_t fp12_mul_line(fp12_t f, fp2_t l00, fp2_t l01, fp2_t l11) {
  fp6_t t0 = fp6_mul_01(f.c0, l00, l01);
  fp6_t t1 = fp6_mul_1(f.c1, l11);
  fp6_t s = fp6_add(f.c0, f.c1);
  fp6_t c1 = fp6_sub(fp6_sub(fp6_mul_01(s, l00, fp2_add(l01, l11)), t0), t1);
  fp6_t c0 = fp6_add(t0, fp6_mul_v(t1));
  return fp12_make(c0, c1);
}

LSG_BIGFN fp12_t fp12_inv(fp12_t a) {
  fp6_t t = fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_v(fp6_mul(a.c1, a.c1)));
  fp6_t ti = fp6_inv(t);
  return fp12_make(fp6_mul(a.c0, ti), fp6_neg(fp6_mul(a.c1, ti)));
}

// a^p : coefficient of w^j is conj(c_j) * gamma1_j; w^j order (c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2)
LSG_BIGFN fp12_t fp12_frob(fp12_t a) {
  fp12_t r;
  r.c0.c0 = fp2_conj(a.c0.c0);
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), FROB1_G1);
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), FROB1_G2);
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), FROB1_G3);
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), FROB1_G4);
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), FROB1_G5);
  return r;
}

LSG_BIGFN fp12_t fp12_frob2(fp12_t a) {
  fp12_t r;
  r.c0.c0 = a.c0.c0;
  r.c1.c0 = fp2_mul(a.c1.c0, FROB2_G1);
  r.c0.c1 = fp2_mul(a.c0.c1, FROB2_G2);
  r.c1.c1 = fp2_mul(a.c1.c1, FROB2_G3);
  r.c0.c2 = fp2_mul(a.c0.c2, FROB2_G4);
  r.c1.c2 = fp2_mul(a.c1.c2, FROB2_G5);
  return r;
}
