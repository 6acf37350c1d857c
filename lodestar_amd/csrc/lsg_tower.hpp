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
// canonical plain integer in [0, p) (fp_canonical is the identity for the fully reduced
// backends; the lazy pair backend reduces here)
LSG_INL fp_t fp_from_mont(const fp_t& a) { return fp_canonical(fp_mul(a, fp_t(FP_ONE_CANON))); }
LSG_INL fp_t fp_from_be48(const uint8_t* b) { return fp_from_be_bytes(b, 12); }

// a^e for a fixed public exponent e (12 little-endian words): left-to-right sliding window
// of width 4 over the odd powers a, a^3, ..., a^15.  For the 379-381-bit exponents of the
// square roots and inversions that is ~380 squarings and ~75 multiplications instead of
// ~380 + popcount(e) (~190).  The window schedule depends on e only, so every lane of a
// wave takes the same branches; the table entry is picked with selects (no indexed
// register access).
LSG_BIGFN fp_t fp_pow_fixed(fp_t a, const uint32_t* e) {
#ifdef LSG_POW_LEAF
  return pair_pow_fixed(a, e);
#else
  fp_t T[8];  // T[k] = a^(2k+1)
  T[0] = a;
  const fp_t a2 = fp_sqr(a);
#pragma unroll
  for (int k = 1; k < 8; k++) T[k] = fp_mul(T[k - 1], a2);
  int i = 383;
  while (i >= 0 && !((e[i >> 5] >> (i & 31)) & 1u)) i--;
  fp_t r = fp_one();
  bool started = false;
  while (i >= 0) {
    if (!((e[i >> 5] >> (i & 31)) & 1u)) {  // started: the top bit is a window
      r = fp_sqr(r);
      i--;
      continue;
    }
    int j = i - 3 < 0 ? 0 : i - 3;  // window e[i..j] ends in a set bit
    while (!((e[j >> 5] >> (j & 31)) & 1u)) j++;
    uint32_t v = 0;
    for (int t = i; t >= j; t--) v = (v << 1) | ((e[t >> 5] >> (t & 31)) & 1u);
    if (started)
      for (int t = i; t >= j; t--) r = fp_sqr(r);
    fp_t tv = T[0];
#pragma unroll
    for (int k = 1; k < 8; k++) tv = fp_select(v == (uint32_t)(2 * k + 1), T[k], tv);
    r = started ? fp_mul(r, tv) : tv;
    started = true;
    i = j - 1;
  }
  return r;
#endif
}

// a^e for the three fixed exponents by id (LSG_POW_INV p-2, LSG_POW_SQRT (p+1)/4,
// LSG_POW_SQRT34 (p-3)/4); the pair backend runs the compile-time plan (pair_pow_plan)
#ifndef LSG_POW_IDS
enum { LSG_POW_INV = 0, LSG_POW_SQRT = 1, LSG_POW_SQRT34 = 2 };
#endif
LSG_BIGFN fp_t fp_pow_id(fp_t a, int id) {
#ifdef LSG_POW_PLAN
  return pair_pow_plan(a, id);
#else
  return fp_pow_fixed(a, id == LSG_POW_INV ? LSG_EXP_P_MINUS_2
                         : id == LSG_POW_SQRT ? LSG_EXP_P_PLUS_1_DIV_4 : LSG_EXP_P_MINUS_3_DIV_4);
#endif
}

LSG_INL fp_t fp_inv(const fp_t& a) { return fp_pow_id(a, LSG_POW_INV); }  // inv(0) = 0

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
#ifdef LSG_FP2_LEAF
  const fp_duo d = pair_fp2_mul(a.c0, a.c1, b.c0, b.c1);
  return fp2_t(d.x, d.y);
#else
  fp_t t0, t1, t2;
  fp_mul3(t0, t1, t2, a.c0, b.c0, a.c1, b.c1, fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return fp2_t(fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1));
#endif
}

// (a0 + a1)(a0 - a1), 2 a0 a1
LSG_INL fp2_t fp2_sqr(const fp2_t& a) {
#ifdef LSG_FP2_LEAF
  const fp_duo d = pair_fp2_sqr(a.c0, a.c1);
  return fp2_t(d.x, d.y);
#else
  fp_t t0, t1;
  fp_mul2(t0, t1, fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1), a.c0, a.c1);
  return fp2_t(t0, fp_dbl(t1));
#endif
}

LSG_INL fp2_t fp2_mul_fp(const fp2_t& a, const fp_t& k) {
  fp_t r0, r1;
  fp_mul2(r0, r1, a.c0, k, a.c1, k);
  return fp2_t(r0, r1);
}

// ---- batched products: independent Montgomery chains interleaved 9 at a time
// (fp_mul9 is one call with nine dependency chains in flight; the tail uses mul3/mul2/mul)
template <int N>
LSG_INL void fp_mul_list(fp_t* r, const fp_t* x, const fp_t* y) {
#ifdef LSG_ROW_SPLIT
#ifndef LSG_SPLIT_MIN
#define LSG_SPLIT_MIN 4
#endif
  if (N >= LSG_SPLIT_MIN) {  // the rows (lane pairs) of a wave share one item: split the batch
    fp_mul_list_rows<N>(r, x, y);
    return;
  }
#endif
#pragma unroll
  for (int g = 0; g + 9 <= N; g += 9) fp_mul9(r + g, x + g, y + g);
  constexpr int T = N % 9, B = N - T;
#pragma unroll
  for (int g = B; g + 3 <= N; g += 3) fp_mul3(r[g], r[g + 1], r[g + 2], x[g], y[g], x[g + 1], y[g + 1], x[g + 2], y[g + 2]);
  constexpr int B2 = B + (T / 3) * 3;
  if (N - B2 == 2) fp_mul2(r[B2], r[B2 + 1], x[B2], y[B2], x[B2 + 1], y[B2 + 1]);
  if (N - B2 == 1) r[B2] = fp_mul(x[B2], y[B2]);
}

// K independent Fp2 products a[k] * b[k] (Karatsuba, 3K Fp products)
template <int K>
LSG_INL void fp2_mul_n(fp2_t* r, const fp2_t* a, const fp2_t* b) {
  fp_t x[3 * K], y[3 * K], z[3 * K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    x[3 * k] = a[k].c0;
    y[3 * k] = b[k].c0;
    x[3 * k + 1] = a[k].c1;
    y[3 * k + 1] = b[k].c1;
    x[3 * k + 2] = fp_add(a[k].c0, a[k].c1);
    y[3 * k + 2] = fp_add(b[k].c0, b[k].c1);
  }
  fp_mul_list<3 * K>(z, x, y);
#pragma unroll
  for (int k = 0; k < K; k++)
    r[k] = fp2_t(fp_sub(z[3 * k], z[3 * k + 1]), fp_sub(fp_sub(z[3 * k + 2], z[3 * k]), z[3 * k + 1]));
}

// K independent Fp2 squarings (2K Fp products)
template <int K>
LSG_INL void fp2_sqr_n(fp2_t* r, const fp2_t* a) {
  fp_t x[2 * K], y[2 * K], z[2 * K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    x[2 * k] = fp_add(a[k].c0, a[k].c1);
    y[2 * k] = fp_sub(a[k].c0, a[k].c1);
    x[2 * k + 1] = a[k].c0;
    y[2 * k + 1] = a[k].c1;
  }
  fp_mul_list<2 * K>(z, x, y);
#pragma unroll
  for (int k = 0; k < K; k++) r[k] = fp2_t(z[2 * k], fp_dbl(z[2 * k + 1]));
}

// (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
LSG_INL fp2_t fp2_mul_xi(const fp2_t& a) { return fp2_t(fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)); }

LSG_INL fp_t fp2_norm(const fp2_t& a) {
  fp_t s0, s1;
  fp_mul2(s0, s1, a.c0, a.c0, a.c1, a.c1);
  return fp_add(s0, s1);
}

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
// Any square root s of n works (the two cases cover both signs).  Returns false when a is
// not a square.  Callers fix the root's sign afterwards.
// Stage 1: the norm's candidate root s = n^((p+1)/4); *is_sq = (s^2 == n).
LSG_INL fp_t fp2_norm_sqrt_candidate(const fp2_t& a, bool* is_sq) {
  fp_t n = fp2_norm(a);
  fp_t s = fp_pow_id(n, LSG_POW_SQRT);
  *is_sq = fp_eq(fp_sqr(s), n);
  return s;
}
// Stage 2: the root of a from a square root s of N(a).
LSG_BIGFN bool fp2_sqrt_with_norm_root(fp2_t& out, fp2_t a, fp_t s) {
  fp_t c = fp_mul(fp_add(a.c0, s), fp_t(FP_HALF));
  c = fp_select(fp_is_zero(c), a.c0, c);
  fp_t t = fp_pow_id(c, LSG_POW_SQRT34);
  fp_t ct = fp_mul(c, t);
  bool c_sq = fp_eq(fp_mul(ct, t), fp_one()) || fp_is_zero(c);
  fp_t h = fp_mul(fp_mul(a.c1, t), fp_t(FP_HALF));
  fp2_t r = c_sq ? fp2_t(ct, h) : fp2_t(h, fp_neg(ct));
  out = r;
  return fp2_eq(fp2_sqr(r), a);
}
LSG_BIGFN bool fp2_sqrt(fp2_t& out, fp2_t a) {
  bool ok;
  fp_t s = fp2_norm_sqrt_candidate(a, &ok);
  bool r = fp2_sqrt_with_norm_root(out, a, s);
  return ok && r;
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

// Karatsuba Fp6 product in two halves so that several Fp6 products can share batched
// Fp2 multiplications: prep writes the 6 Fp2 operand pairs, fin combines the 6 products.
// Same value as oracle/fields.py:f6_mul.
LSG_INL void fp6_mul_prep(fp2_t* A, fp2_t* B, const fp6_t& a, const fp6_t& b) {
  A[0] = a.c0;
  B[0] = b.c0;
  A[1] = a.c1;
  B[1] = b.c1;
  A[2] = a.c2;
  B[2] = b.c2;
  A[3] = fp2_add(a.c1, a.c2);
  B[3] = fp2_add(b.c1, b.c2);
  A[4] = fp2_add(a.c0, a.c1);
  B[4] = fp2_add(b.c0, b.c1);
  A[5] = fp2_add(a.c0, a.c2);
  B[5] = fp2_add(b.c0, b.c2);
}
LSG_INL fp6_t fp6_mul_fin(const fp2_t* V) {
  fp2_t c0 = fp2_add(V[0], fp2_mul_xi(fp2_sub(fp2_sub(V[3], V[1]), V[2])));
  fp2_t c1 = fp2_add(fp2_sub(fp2_sub(V[4], V[0]), V[1]), fp2_mul_xi(V[2]));
  fp2_t c2 = fp2_add(fp2_sub(fp2_sub(V[5], V[0]), V[2]), V[1]);
  fp6_t r;
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
  return r;
}
#ifdef LSG_LEAN_TOWER
// Quad backend: an Fp takes three VGPRs, so the products are issued one Fp2 product (three
// interleaved Montgomery chains) at a time instead of in wide batches; same values.
LSG_BIGFN fp6_t fp6_mul(fp6_t a, fp6_t b) {
  fp2_t v0 = fp2_mul(a.c0, b.c0);
  fp2_t v1 = fp2_mul(a.c1, b.c1);
  fp2_t v2 = fp2_mul(a.c2, b.c2);
  fp2_t c0 = fp2_add(v0, fp2_mul_xi(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), v1), v2)));
  fp2_t c1 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), v0), v1), fp2_mul_xi(v2));
  fp2_t c2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), v0), v2), v1);
  return fp6_make(c0, c1, c2);
}
#else
LSG_BIGFN fp6_t fp6_mul(fp6_t a, fp6_t b) {
  fp2_t A[6], B[6], V[6];
  fp6_mul_prep(A, B, a, b);
  fp2_mul_n<6>(V, A, B);
  return fp6_mul_fin(V);
}
#endif

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

#ifdef LSG_LEAN_TOWER
LSG_BIGFN fp12_t fp12_mul(fp12_t a, fp12_t b) {
  fp6_t t0 = fp6_mul(a.c0, b.c0);
  fp6_t t1 = fp6_mul(a.c1, b.c1);
  fp6_t t2 = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1));
  return fp12_make(fp6_add(t0, fp6_mul_v(t1)), fp6_sub(fp6_sub(t2, t0), t1));
}
LSG_BIGFN fp12_t fp12_sqr(fp12_t a) {
  fp6_t t = fp6_mul(a.c0, a.c1);
  fp6_t u = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  return fp12_make(fp6_sub(fp6_sub(u, t), fp6_mul_v(t)), fp6_add(t, t));
}
#else
// Karatsuba over Fp6: the three Fp6 products (18 Fp2 products) are issued as one batch
LSG_BIGFN fp12_t fp12_mul(fp12_t a, fp12_t b) {
  fp2_t A[18], B[18], V[18];
  fp6_mul_prep(A, B, a.c0, b.c0);
  fp6_mul_prep(A + 6, B + 6, a.c1, b.c1);
  fp6_mul_prep(A + 12, B + 12, fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1));
  fp2_mul_n<18>(V, A, B);
  fp6_t t0 = fp6_mul_fin(V), t1 = fp6_mul_fin(V + 6), t2 = fp6_mul_fin(V + 12);
  return fp12_make(fp6_add(t0, fp6_mul_v(t1)), fp6_sub(fp6_sub(t2, t0), t1));
}

// (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w; both Fp6 products in one batch
LSG_BIGFN fp12_t fp12_sqr(fp12_t a) {
  fp2_t A[12], B[12], V[12];
  fp6_mul_prep(A, B, a.c0, a.c1);
  fp6_mul_prep(A + 6, B + 6, fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  fp2_mul_n<12>(V, A, B);
  fp6_t t = fp6_mul_fin(V), u = fp6_mul_fin(V + 6);
  return fp12_make(fp6_sub(fp6_sub(u, t), fp6_mul_v(t)), fp6_add(t, t));
}
#endif

// (a + b t)^2 in Fp4 = Fp2[t]/(t^2 - xi)  -- oracle/pairing.py:_fp4_square
LSG_INL void fp4_square(fp2_t& c0, fp2_t& c1, const fp2_t& a, const fp2_t& b) {
  fp2_t t0 = fp2_sqr(a);
  fp2_t t1 = fp2_sqr(b);
  c0 = fp2_add(fp2_mul_xi(t1), t0);
  c1 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(a, b)), t0), t1);
}

// Granger-Scott squaring for f in the cyclotomic subgroup -- oracle/pairing.py:f12_cyclotomic_sqr
// (the three Fp4 squarings = 9 Fp2 squarings issued as one batch)
LSG_BIGFN fp12_t fp12_cyclotomic_sqr(fp12_t f) {
  fp2_t z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2, z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
#ifdef LSG_LEAN_TOWER
  fp2_t t0, t1, u0, u1, t2, t3;
  fp4_square(t0, t1, z0, z1);
  fp4_square(u0, u1, z2, z3);
  fp4_square(t2, t3, z4, z5);
#else
  fp2_t S[9], Q[9];
  S[0] = z0;
  S[1] = z1;
  S[2] = fp2_add(z0, z1);
  S[3] = z2;
  S[4] = z3;
  S[5] = fp2_add(z2, z3);
  S[6] = z4;
  S[7] = z5;
  S[8] = fp2_add(z4, z5);
  fp2_sqr_n<9>(Q, S);
  // fp4_square(a, b): c0 = xi b^2 + a^2, c1 = (a + b)^2 - a^2 - b^2
  fp2_t t0 = fp2_add(fp2_mul_xi(Q[1]), Q[0]);
  fp2_t t1 = fp2_sub(fp2_sub(Q[2], Q[0]), Q[1]);
  fp2_t u0 = fp2_add(fp2_mul_xi(Q[4]), Q[3]);
  fp2_t u1 = fp2_sub(fp2_sub(Q[5], Q[3]), Q[4]);
  fp2_t t2 = fp2_add(fp2_mul_xi(Q[7]), Q[6]);
  fp2_t t3 = fp2_sub(fp2_sub(Q[8], Q[6]), Q[7]);
#endif
  z0 = fp2_sub(t0, z0);
  z0 = fp2_add(fp2_add(z0, z0), t0);
  z1 = fp2_add(t1, z1);
  z1 = fp2_add(fp2_add(z1, z1), t1);
  t0 = u0;
  t1 = u1;
  z4 = fp2_sub(t0, z4);
  z4 = fp2_add(fp2_add(z4, z4), t0);
  z5 = fp2_add(t1, z5);
  z5 = fp2_add(fp2_add(z5, z5), t1);
  t0 = fp2_mul_xi(t3);
  z2 = fp2_add(t0, z2);
  z2 = fp2_add(fp2_add(z2, z2), t0);
  z3 = fp2_sub(t2, z3);
  z3 = fp2_add(fp2_add(z3, z3), t2);
#ifdef LSG_PAIR_MODE
  // the output carries 2x the input additively (3t - 2z): bound lazy values so chains of
  // squarings (exp by x) do not grow them without limit
  fp2_t* zs[6] = {&z0, &z1, &z2, &z3, &z4, &z5};
  for (int k = 0; k < 6; k++) *zs[k] = fp2_t(fp_tame(zs[k]->c0), fp_tame(zs[k]->c1));
#endif
  return fp12_make(fp6_make(z0, z4, z3), fp6_make(z2, z1, z5));
}

// f * ((l00 + l01 v) + (l11 v) w)   -- oracle/pairing.py:f12_mul_line
// fp6_mul_01(f0, l00, l01), fp6_mul_01(f0 + f1, l00, l01 + l11) and fp6_mul_1(f1, l11):
// 13 independent Fp2 products issued as one batch.
LSG_BIGFN fp12_t fp12_mul_line(fp12_t f, fp2_t l00, fp2_t l01, fp2_t l11) {
#ifdef LSG_LEAN_TOWER
  fp6_t t0 = fp6_mul_01(f.c0, l00, l01);
  fp6_t u = fp6_mul_01(fp6_add(f.c0, f.c1), l00, fp2_add(l01, l11));
  fp6_t t1 = fp6_mul_1(f.c1, l11);
  return fp12_make(fp6_add(t0, fp6_mul_v(t1)), fp6_sub(fp6_sub(u, t0), t1));
#else
  const fp6_t& a = f.c0;
  const fp6_t& c = f.c1;
  fp6_t s = fp6_add(f.c0, f.c1);
  fp2_t m = fp2_add(l01, l11);
  fp2_t A[13], B[13], V[13];
  // fp6_mul_01(a, l00, l01): a0 b0, a1 b1, a2 b1, (a0+a1)(b0+b1), a2 b0
  A[0] = a.c0; B[0] = l00;
  A[1] = a.c1; B[1] = l01;
  A[2] = a.c2; B[2] = l01;
  A[3] = fp2_add(a.c0, a.c1); B[3] = fp2_add(l00, l01);
  A[4] = a.c2; B[4] = l00;
  // fp6_mul_01(s, l00, m)
  A[5] = s.c0; B[5] = l00;
  A[6] = s.c1; B[6] = m;
  A[7] = s.c2; B[7] = m;
  A[8] = fp2_add(s.c0, s.c1); B[8] = fp2_add(l00, m);
  A[9] = s.c2; B[9] = l00;
  // fp6_mul_1(c, l11): c2 b1, c0 b1, c1 b1
  A[10] = c.c2; B[10] = l11;
  A[11] = c.c0; B[11] = l11;
  A[12] = c.c1; B[12] = l11;
  fp2_mul_n<13>(V, A, B);
  fp6_t t0 = fp6_make(fp2_add(fp2_mul_xi(V[2]), V[0]), fp2_sub(fp2_sub(V[3], V[0]), V[1]), fp2_add(V[4], V[1]));
  fp6_t u = fp6_make(fp2_add(fp2_mul_xi(V[7]), V[5]), fp2_sub(fp2_sub(V[8], V[5]), V[6]), fp2_add(V[9], V[6]));
  fp6_t t1 = fp6_make(fp2_mul_xi(V[10]), V[11], V[12]);
  return fp12_make(fp6_add(t0, fp6_mul_v(t1)), fp6_sub(fp6_sub(u, t0), t1));
#endif
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
