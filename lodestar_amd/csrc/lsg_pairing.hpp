// Optimal-ate Miller loop and final exponentiation for gfx950.  Replaces blst's
// miller_loop_n / final_exp used by Pairing.commit()/finalverify() under
// @chainsafe/blst verifyMultipleAggregateSignatures and verify
// (packages/beacon-node/src/chain/bls/maybeBatch.ts:18,37).
// Operation-for-operation mirror of oracle/pairing.py (dbl_step, add_step,
// f12_mul_line, miller_loop_fast, final_exp_fast), so per-pair Miller values are
// bit-comparable with the oracle.
#pragma once
#include "lsg_curve.hpp"

struct line_t {
  fp2_t l00, l01, l11;
};

// T <- 2T; returns the line unevaluated: (3b'Z^2 - Y^2, 3X^2, -2YZ); at P it is
// (l00, l01 xP, l11 yP) (line_eval)
LSG_BIGFN line_t ml_dbl_step_raw(g2p_t& T) {
  fp2_t t0 = fp2_sqr(T.Y);
  fp2_t t1 = fp2_mul(T.Y, T.Z);
  fp2_t t2 = fp2_mul_b3(fp2_sqr(T.Z));
  fp2_t XX = fp2_sqr(T.X);
  line_t L;
  L.l00 = fp2_sub(t2, t0);
  L.l01 = fp2_add(fp2_add(XX, XX), XX);
  L.l11 = fp2_neg(fp2_add(t1, t1));
  fp2_t Z3 = fp2_add(t0, t0);
  Z3 = fp2_add(Z3, Z3);
  Z3 = fp2_add(Z3, Z3);
  fp2_t X3 = fp2_mul(t2, Z3);
  fp2_t Y3 = fp2_add(t0, t2);
  Z3 = fp2_mul(t1, Z3);
  fp2_t u1 = fp2_add(t2, t2);
  fp2_t u2 = fp2_add(u1, t2);
  fp2_t s0 = fp2_sub(t0, u2);
  Y3 = fp2_mul(s0, Y3);
  Y3 = fp2_add(X3, Y3);
  fp2_t v1 = fp2_mul(T.X, T.Y);
  X3 = fp2_mul(s0, v1);
  X3 = fp2_add(X3, X3);
  T.X = X3;
  T.Y = Y3;
  T.Z = Z3;
  return L;
}

// T <- T + Q; theta = Y - yQ Z, delta = X - xQ Z; unevaluated line (delta yQ - theta xQ,
// theta, -delta); at P: (l00, theta xP, -delta yP)
LSG_BIGFN line_t ml_add_step_raw(g2p_t& T, g2a_t Q) {
  fp2_t theta = fp2_sub(T.Y, fp2_mul(Q.y, T.Z));
  fp2_t delta = fp2_sub(T.X, fp2_mul(Q.x, T.Z));
  line_t L;
  L.l00 = fp2_sub(fp2_mul(delta, Q.y), fp2_mul(theta, Q.x));
  L.l01 = theta;
  L.l11 = fp2_neg(delta);
  fp2_t C = fp2_sqr(theta);
  fp2_t D = fp2_sqr(delta);
  fp2_t E = fp2_mul(D, delta);
  fp2_t F = fp2_mul(T.Z, C);
  fp2_t G = fp2_mul(T.X, D);
  fp2_t H = fp2_sub(fp2_add(E, F), fp2_add(G, G));
  fp2_t X3 = fp2_mul(delta, H);
  fp2_t Y3 = fp2_sub(fp2_mul(theta, fp2_sub(G, H)), fp2_mul(E, T.Y));
  fp2_t Z3 = fp2_mul(E, T.Z);
  T.X = X3;
  T.Y = Y3;
  T.Z = Z3;
  return L;
}

// an unevaluated line at the G1 point P = (xP, yP)
LSG_INL line_t line_eval(line_t L, const fp_t& xP, const fp_t& yP) {
  L.l01 = fp2_mul_fp(L.l01, xP);
  L.l11 = fp2_mul_fp(L.l11, yP);
  return L;
}

#ifdef LSG_ROW_SPLIT
// Rows of a wave sharing one item (lsg_fp_lane.hpp): the steps above with their independent
// products issued as batches for the rows to split (identical values: the row backend keeps
// every value fully reduced).  Doubling: round 1 Y^2, YZ, Z^2, X^2, XY; round 2 the point's
// four products and the line evaluation at P.
LSG_INL line_t ml_dbl_step_rows(g2p_t& T, const fp_t& xP, const fp_t& yP) {
  fp_t x[16], y[16], z[16];
  kar_prep(x, y, 0, T.Y, T.Y);
  kar_prep(x, y, 3, T.Y, T.Z);
  kar_prep(x, y, 6, T.Z, T.Z);
  kar_prep(x, y, 9, T.X, T.X);
  kar_prep(x, y, 12, T.X, T.Y);
  fp_mul_list<15>(z, x, y);
  const fp2_t t0 = kar_fin(z, 0), t1 = kar_fin(z, 3), t2 = fp2_mul_b3(kar_fin(z, 6)), XX = kar_fin(z, 9),
              v1 = kar_fin(z, 12);
  line_t L;
  L.l00 = fp2_sub(t2, t0);
  const fp2_t l01 = fp2_add(fp2_add(XX, XX), XX), l11 = fp2_neg(fp2_add(t1, t1));
  const fp2_t z8 = fp2_dbl(fp2_dbl(fp2_dbl(t0)));
  const fp2_t y3 = fp2_add(t0, t2);
  const fp2_t s0 = fp2_sub(t0, fp2_add(fp2_add(t2, t2), t2));
  kar_prep(x, y, 0, t2, z8);
  kar_prep(x, y, 3, t1, z8);
  kar_prep(x, y, 6, s0, y3);
  kar_prep(x, y, 9, s0, v1);
  x[12] = l01.c0;
  y[12] = xP;
  x[13] = l01.c1;
  y[13] = xP;
  x[14] = l11.c0;
  y[14] = yP;
  x[15] = l11.c1;
  y[15] = yP;
  fp_mul_list<16>(z, x, y);
  const fp2_t X3 = kar_fin(z, 0);
  T.X = fp2_dbl(kar_fin(z, 9));
  T.Y = fp2_add(X3, kar_fin(z, 6));
  T.Z = kar_fin(z, 3);
  L.l01 = fp2_t(z[12], z[13]);
  L.l11 = fp2_t(z[14], z[15]);
  return L;
}
// Addition: four rounds (Q Z; the line and C, D; E, F, G and the evaluation; the outputs)
LSG_INL line_t ml_add_step_rows(g2p_t& T, const g2a_t& Q, const fp_t& xP, const fp_t& yP) {
  fp_t x[13], y[13], z[13];
  kar_prep(x, y, 0, Q.y, T.Z);
  kar_prep(x, y, 3, Q.x, T.Z);
  fp_mul_list<6>(z, x, y);
  const fp2_t theta = fp2_sub(T.Y, kar_fin(z, 0)), delta = fp2_sub(T.X, kar_fin(z, 3));
  kar_prep(x, y, 0, delta, Q.y);
  kar_prep(x, y, 3, theta, Q.x);
  kar_prep(x, y, 6, theta, theta);
  kar_prep(x, y, 9, delta, delta);
  fp_mul_list<12>(z, x, y);
  line_t L;
  L.l00 = fp2_sub(kar_fin(z, 0), kar_fin(z, 3));
  const fp2_t C = kar_fin(z, 6), D = kar_fin(z, 9), l11 = fp2_neg(delta);
  kar_prep(x, y, 0, D, delta);
  kar_prep(x, y, 3, T.Z, C);
  kar_prep(x, y, 6, T.X, D);
  x[9] = theta.c0;
  y[9] = xP;
  x[10] = theta.c1;
  y[10] = xP;
  x[11] = l11.c0;
  y[11] = yP;
  x[12] = l11.c1;
  y[12] = yP;
  fp_mul_list<13>(z, x, y);
  const fp2_t E = kar_fin(z, 0), F = kar_fin(z, 3), G = kar_fin(z, 6);
  L.l01 = fp2_t(z[9], z[10]);
  L.l11 = fp2_t(z[11], z[12]);
  const fp2_t H = fp2_sub(fp2_add(E, F), fp2_add(G, G));
  kar_prep(x, y, 0, delta, H);
  kar_prep(x, y, 3, theta, fp2_sub(G, H));
  kar_prep(x, y, 6, E, T.Y);
  kar_prep(x, y, 9, E, T.Z);
  fp_mul_list<12>(z, x, y);
  T.X = kar_fin(z, 0);
  T.Y = fp2_sub(kar_fin(z, 3), kar_fin(z, 6));
  T.Z = kar_fin(z, 9);
  return L;
}
LSG_INL line_t ml_dbl_step(g2p_t& T, fp_t xP, fp_t yP) { return ml_dbl_step_rows(T, xP, yP); }
LSG_INL line_t ml_add_step(g2p_t& T, g2a_t Q, fp_t xP, fp_t yP) { return ml_add_step_rows(T, Q, xP, yP); }
#else
// T <- 2T; line = (3b'Z^2 - Y^2, 3X^2 xP, -2YZ yP)
LSG_INL line_t ml_dbl_step(g2p_t& T, fp_t xP, fp_t yP) { return line_eval(ml_dbl_step_raw(T), xP, yP); }

// T <- T + Q; line = (delta yQ - theta xQ, theta xP, -delta yP)
LSG_INL line_t ml_add_step(g2p_t& T, g2a_t Q, fp_t xP, fp_t yP) {
  return line_eval(ml_add_step_raw(T, Q), xP, yP);
}
#endif

// f_{|x|,Q}(P) conjugated (x < 0).  P affine G1, Q affine G2, both finite.
LSG_BIGFN fp12_t miller_loop(g1a_t P, g2a_t Q) {
  const uint64_t xa = ((uint64_t)LSG_X_ABS_HI << 32) | LSG_X_ABS_LO;
  g2p_t T = proj_from_aff(Q);
  line_t L = ml_dbl_step(T, P.x, P.y);
  fp12_t f;
  f.c0 = fp6_make(L.l00, L.l01, fp2_zero());
  f.c1 = fp6_make(fp2_zero(), L.l11, fp2_zero());
  // bit 62 of |x| is 1
  L = ml_add_step(T, Q, P.x, P.y);
  f = fp12_mul_line(f, L.l00, L.l01, L.l11);
  for (int b = 61; b >= 0; b--) {
    f = fp12_sqr(f);
    L = ml_dbl_step(T, P.x, P.y);
    f = fp12_mul_line(f, L.l00, L.l01, L.l11);
    if ((xa >> b) & 1u) {
      L = ml_add_step(T, Q, P.x, P.y);
      f = fp12_mul_line(f, L.l00, L.l01, L.l11);
    }
  }
  return fp12_conj(f);
}

LSG_INL fp12_t fp12_from_line(const line_t& L) {
  fp12_t f;
  f.c0 = fp6_make(L.l00, L.l01, fp2_zero());
  f.c1 = fp6_make(fp2_zero(), L.l11, fp2_zero());
  return f;
}
LSG_INL fp12_t fp12_select(bool c, const fp12_t& a, const fp12_t& b) {
  fp12_t r;
  r.c0 = fp6_make(fp2_select(c, a.c0.c0, b.c0.c0), fp2_select(c, a.c0.c1, b.c0.c1), fp2_select(c, a.c0.c2, b.c0.c2));
  r.c1 = fp6_make(fp2_select(c, a.c1.c0, b.c1.c0), fp2_select(c, a.c1.c1, b.c1.c1), fp2_select(c, a.c1.c2, b.c1.c2));
  return r;
}

// Multi-Miller loop over K pairs sharing one f and its squarings (blst miller_loop_n):
// returns prod_{k: use[k]} conj(f_{|x|,Q_k}(P_k)), the same field element as the product of
// the per-pair miller_loop() values.  Pairs with use[k] == false contribute 1 (their point
// arithmetic still runs so that every row of a wave follows one control path).
template <int K>
LSG_INL fp12_t miller_loop_multi(const g1a_t (&P)[K], const g2a_t (&Q)[K], const bool (&use)[K]) {
  const uint64_t xa = ((uint64_t)LSG_X_ABS_HI << 32) | LSG_X_ABS_LO;
  g2p_t T[K];
  fp12_t f = fp12_one();
  bool started = false;  // row-uniform: f still 1
#pragma unroll
  for (int k = 0; k < K; k++) {
    T[k] = proj_from_aff(Q[k]);
    line_t L = ml_dbl_step(T[k], P[k].x, P[k].y);
    fp12_t g = started ? fp12_mul_line(f, L.l00, L.l01, L.l11) : fp12_from_line(L);
    f = fp12_select(use[k], g, f);
    started = true;
  }
#pragma unroll
  for (int k = 0; k < K; k++) {  // bit 62 of |x| is 1
    line_t L = ml_add_step(T[k], Q[k], P[k].x, P[k].y);
    f = fp12_select(use[k], fp12_mul_line(f, L.l00, L.l01, L.l11), f);
  }
#pragma unroll 1
  for (int b = 61; b >= 0; b--) {
    f = fp12_sqr(f);
#pragma unroll
    for (int k = 0; k < K; k++) {
      line_t L = ml_dbl_step(T[k], P[k].x, P[k].y);
      f = fp12_select(use[k], fp12_mul_line(f, L.l00, L.l01, L.l11), f);
    }
    if ((xa >> b) & 1u) {
#pragma unroll
      for (int k = 0; k < K; k++) {
        line_t L = ml_add_step(T[k], Q[k], P[k].x, P[k].y);
        f = fp12_select(use[k], fp12_mul_line(f, L.l00, L.l01, L.l11), f);
      }
    }
  }
  return fp12_conj(f);
}

// ---- Split Miller loop (device path): the G2 side and the Fp12 side run as two kernels.
// miller_lines writes the ML_STEPS unevaluated lines of one Q in loop order (step 0: the
// first doubling, step 1: the addition for bit 62, then per bit b = 61..0 a doubling and,
// for set bits, an addition); miller_accum_multi evaluates them at the P_k and accumulates
// f with the same operation order as miller_loop_multi, so the result is the same field
// element.  Each kernel then holds only its own half of the state (T and a line, or f and a
// line) instead of f, K points and the line together.
constexpr int ML_STEPS = 68;  // 63 doublings + 5 additions for |x| = 0xd201000000010000

template <class Put>
LSG_INL void miller_lines(const g2a_t& Q, Put&& put) {
  const uint64_t xa = ((uint64_t)LSG_X_ABS_HI << 32) | LSG_X_ABS_LO;
  g2p_t T = proj_from_aff(Q);
  int s = 0;
  put(s++, ml_dbl_step_raw(T));
  put(s++, ml_add_step_raw(T, Q));
#pragma unroll 1
  for (int b = 61; b >= 0; b--) {
    put(s++, ml_dbl_step_raw(T));
    if ((xa >> b) & 1u) put(s++, ml_add_step_raw(T, Q));
  }
}

// get(k, step) -> the unevaluated line of pair k at that step
template <int K, class Get>
LSG_INL fp12_t miller_accum_multi(const g1a_t (&P)[K], const bool (&use)[K], Get&& get) {
  const uint64_t xa = ((uint64_t)LSG_X_ABS_HI << 32) | LSG_X_ABS_LO;
  fp12_t f = fp12_one();
#pragma unroll
  for (int k = 0; k < K; k++) {
    line_t L = line_eval(get(k, 0), P[k].x, P[k].y);
    fp12_t g = k > 0 ? fp12_mul_line(f, L.l00, L.l01, L.l11) : fp12_from_line(L);
    f = fp12_select(use[k], g, f);
  }
#pragma unroll
  for (int k = 0; k < K; k++) {
    line_t L = line_eval(get(k, 1), P[k].x, P[k].y);
    f = fp12_select(use[k], fp12_mul_line(f, L.l00, L.l01, L.l11), f);
  }
  int s = 2;
#pragma unroll 1
  for (int b = 61; b >= 0; b--) {
    f = fp12_sqr(f);
    const int n_steps = 1 + (int)((xa >> b) & 1u);
#pragma unroll 1
    for (int j = 0; j < n_steps; j++, s++) {
#pragma unroll
      for (int k = 0; k < K; k++) {
        line_t L = line_eval(get(k, s), P[k].x, P[k].y);
        f = fp12_select(use[k], fp12_mul_line(f, L.l00, L.l01, L.l11), f);
      }
    }
  }
  return fp12_conj(f);
}

// g^x for g in the cyclotomic subgroup
LSG_BIGFN fp12_t fp12_exp_by_x(fp12_t g) {
  const uint64_t xa = ((uint64_t)LSG_X_ABS_HI << 32) | LSG_X_ABS_LO;
  fp12_t r = g;
  for (int b = 62; b >= 0; b--) {
    r = fp12_cyclotomic_sqr(r);
    if ((xa >> b) & 1u) r = fp12_mul(r, g);
  }
  return fp12_conj(r);
}

// f^(3 (p^12 - 1)/r)   -- oracle/pairing.py:final_exp_fast
LSG_BIGFN fp12_t final_exp(fp12_t f) {
  fp12_t f1 = fp12_mul(fp12_conj(f), fp12_inv(f));
  fp12_t g = fp12_mul(fp12_frob2(f1), f1);
  fp12_t t0 = fp12_mul(fp12_exp_by_x(g), fp12_conj(g));
  t0 = fp12_mul(fp12_exp_by_x(t0), fp12_conj(t0));
  fp12_t t1 = fp12_mul(fp12_exp_by_x(t0), fp12_frob(t0));
  fp12_t t2 = fp12_mul(fp12_mul(fp12_exp_by_x(fp12_exp_by_x(t1)), fp12_frob2(t1)), fp12_conj(t1));
  return fp12_mul(t2, fp12_mul(fp12_sqr(g), g));
}
