/*
 * ORACLE / CPU BASELINE -- test infrastructure only, never linked into or called by the
 * product (lodestar_amd/).  A C restatement of the Python oracle (the oracle/ modules), i.e. of the
 * BLS12-381 verification path under Lodestar's IBlsVerifier (packages/beacon-node/src/
 * chain/bls/maybeBatch.ts:16-39, multithread/worker.ts:30-106) as the un-vendored
 * @chainsafe/blst@0.2.8 computes it.  Six 64-bit limbs with unsigned __int128 Montgomery
 * products; the same formulas as oracle/fields.py, oracle/curves.py, oracle/hash_to_curve.py
 * and oracle/pairing.py (function names follow them).  Its uses:
 *   - bench.py's cpu_baseline: the worker pool's job shape (RLC batches of 16 sets, one
 *     pthread per host core) on a bounded sample of the benchmark workload;
 *   - tests/test_oracle_c.py checks it against the Python oracle and the golden vectors.
 * Build: make -C oracle/c  (gcc -O3; bls_consts.h is generated from the Python oracle).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct {
  uint64_t l[6];
} fp;
typedef struct {
  fp c0, c1;
} fp2;
typedef struct {
  fp2 c0, c1, c2;
} fp6;
typedef struct {
  fp6 c0, c1;
} fp12;

#include "bls_consts.h"

/* ------------------------------------------------------------------ Fp (oracle/fields.py) */
static int fp_geq_p(const uint64_t* a) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] > C_P[i]) return 1;
    if (a[i] < C_P[i]) return 0;
  }
  return 1;
}
static void fp_sub_p(uint64_t* a) {
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a[i] - C_P[i] - br;
    a[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
}
static inline void fp_add(fp* r, const fp* a, const fp* b) {
  uint64_t c = 0;
  for (int i = 0; i < 6; i++) {
    u128 s = (u128)a->l[i] + b->l[i] + c;
    r->l[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (fp_geq_p(r->l)) fp_sub_p(r->l);
}
static inline void fp_sub(fp* r, const fp* a, const fp* b) {
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a->l[i] - b->l[i] - br;
    r->l[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; i++) {
      u128 s = (u128)r->l[i] + C_P[i] + c;
      r->l[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
}
static inline int fp_is_zero(const fp* a) {
  uint64_t x = 0;
  for (int i = 0; i < 6; i++) x |= a->l[i];
  return x == 0;
}
static inline int fp_eq(const fp* a, const fp* b) { return memcmp(a, b, sizeof(fp)) == 0; }
static inline void fp_neg(fp* r, const fp* a) {
  fp z;
  memset(&z, 0, sizeof z);
  fp_sub(r, &z, a);
}
/* CIOS Montgomery product */
static void fp_mul(fp* r, const fp* a, const fp* b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 6; i++) {
    uint64_t C = 0;
    for (int j = 0; j < 6; j++) {
      u128 s = (u128)a->l[j] * b->l[i] + t[j] + C;
      t[j] = (uint64_t)s;
      C = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[6] + C;
    t[6] = (uint64_t)s;
    t[7] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * C_N0;
    s = (u128)m * C_P[0] + t[0];
    C = (uint64_t)(s >> 64);
    for (int j = 1; j < 6; j++) {
      s = (u128)m * C_P[j] + t[j] + C;
      t[j - 1] = (uint64_t)s;
      C = (uint64_t)(s >> 64);
    }
    s = (u128)t[6] + C;
    t[5] = (uint64_t)s;
    t[6] = t[7] + (uint64_t)(s >> 64);
  }
  memcpy(r->l, t, 48);
  if (t[6] || fp_geq_p(r->l)) fp_sub_p(r->l);
}
static inline void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }
static void fp_pow(fp* r, const fp* a, const uint64_t* e) {
  fp acc = C_ONE, base = *a;
  int started = 0;
  for (int w = 5; w >= 0; w--)
    for (int b = 63; b >= 0; b--) {
      if (started) fp_sqr(&acc, &acc);
      if ((e[w] >> b) & 1) {
        if (started)
          fp_mul(&acc, &acc, &base);
        else
          acc = base;
        started = 1;
      }
    }
  *r = acc;
}
static inline void fp_inv(fp* r, const fp* a) { fp_pow(r, a, C_EXP_INV); }
/* canonical (non-Montgomery) value <-> 48 big-endian bytes */
static void fp_from_mont(uint64_t* out, const fp* a) {
  fp one;
  memset(&one, 0, sizeof one);
  one.l[0] = 1;
  fp t;
  fp_mul(&t, a, &one);
  memcpy(out, t.l, 48);
}
static void fp_to_be48(uint8_t* b, const fp* a) {
  uint64_t v[6];
  fp_from_mont(v, a);
  for (int i = 0; i < 6; i++)
    for (int k = 0; k < 8; k++) b[47 - 8 * i - k] = (uint8_t)(v[i] >> (8 * k));
}
static void be_to_limbs(uint64_t* v, const uint8_t* b, int nbytes) {
  memset(v, 0, 48);
  for (int i = 0; i < nbytes; i++) {
    int k = nbytes - 1 - i;
    v[k / 8] |= (uint64_t)b[i] << (8 * (k % 8));
  }
}
static int lt_p(const uint64_t* v) { return !fp_geq_p(v); }
static void fp_from_canon(fp* r, const uint64_t* v) {
  fp t;
  memcpy(t.l, v, 48);
  fp_mul(r, &t, &C_R2);
}
static int fp_sqrt(fp* r, const fp* a) {
  fp s, t;
  fp_pow(&s, a, C_EXP_SQRT);
  fp_sqr(&t, &s);
  *r = s;
  return fp_eq(&t, a);
}
static int canon_gt_half(const fp* a) {
  uint64_t v[6];
  fp_from_mont(v, a);
  for (int i = 5; i >= 0; i--) {
    if (v[i] > C_HALF_P[i]) return 1;
    if (v[i] < C_HALF_P[i]) return 0;
  }
  return 0;
}

/* ------------------------------------------------------------------ Fp2 */
static inline void f2_add(fp2* r, const fp2* a, const fp2* b) {
  fp_add(&r->c0, &a->c0, &b->c0);
  fp_add(&r->c1, &a->c1, &b->c1);
}
static inline void f2_sub(fp2* r, const fp2* a, const fp2* b) {
  fp_sub(&r->c0, &a->c0, &b->c0);
  fp_sub(&r->c1, &a->c1, &b->c1);
}
static inline void f2_neg(fp2* r, const fp2* a) {
  fp_neg(&r->c0, &a->c0);
  fp_neg(&r->c1, &a->c1);
}
static inline void f2_conj(fp2* r, const fp2* a) {
  r->c0 = a->c0;
  fp_neg(&r->c1, &a->c1);
}
static void f2_mul(fp2* r, const fp2* a, const fp2* b) {
  fp t0, t1, s0, s1, t2;
  fp_mul(&t0, &a->c0, &b->c0);
  fp_mul(&t1, &a->c1, &b->c1);
  fp_add(&s0, &a->c0, &a->c1);
  fp_add(&s1, &b->c0, &b->c1);
  fp_mul(&t2, &s0, &s1);
  fp_sub(&r->c0, &t0, &t1);
  fp_sub(&t2, &t2, &t0);
  fp_sub(&r->c1, &t2, &t1);
}
static void f2_sqr(fp2* r, const fp2* a) {
  fp s, d, p;
  fp_add(&s, &a->c0, &a->c1);
  fp_sub(&d, &a->c0, &a->c1);
  fp_mul(&p, &a->c0, &a->c1);
  fp_mul(&r->c0, &s, &d);
  fp_add(&r->c1, &p, &p);
}
static inline void f2_mul_fp(fp2* r, const fp2* a, const fp* k) {
  fp_mul(&r->c0, &a->c0, k);
  fp_mul(&r->c1, &a->c1, k);
}
static inline void f2_mul_xi(fp2* r, const fp2* a) { /* (1 + u) a */
  fp t0, t1;
  fp_sub(&t0, &a->c0, &a->c1);
  fp_add(&t1, &a->c0, &a->c1);
  r->c0 = t0;
  r->c1 = t1;
}
static inline int f2_is_zero(const fp2* a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static inline int f2_eq(const fp2* a, const fp2* b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static void f2_norm(fp* r, const fp2* a) {
  fp t0, t1;
  fp_sqr(&t0, &a->c0);
  fp_sqr(&t1, &a->c1);
  fp_add(r, &t0, &t1);
}
static void f2_inv(fp2* r, const fp2* a) {
  fp n, ni;
  f2_norm(&n, a);
  fp_inv(&ni, &n);
  fp_mul(&r->c0, &a->c0, &ni);
  fp t;
  fp_mul(&t, &a->c1, &ni);
  fp_neg(&r->c1, &t);
}
/* a square root of a (any sign; callers fix it), 0 if none -- norm method */
static int f2_sqrt(fp2* r, const fp2* a) {
  if (f2_is_zero(a)) {
    *r = *a;
    return 1;
  }
  fp n, s, half, c, t, cs;
  f2_norm(&n, a);
  if (!fp_sqrt(&s, &n)) return 0;
  fp two = C_ONE;
  fp_add(&two, &two, &two);
  fp_inv(&half, &two);
  for (int k = 0; k < 2; k++) {
    fp sg = s;
    if (k) fp_neg(&sg, &s);
    fp_add(&c, &a->c0, &sg);
    fp_mul(&c, &c, &half);
    if (fp_is_zero(&c)) continue;
    if (fp_sqrt(&t, &c)) {
      fp x1, d;
      fp_add(&d, &t, &t);
      fp_inv(&d, &d);
      fp_mul(&x1, &a->c1, &d);
      fp2 cand = {t, x1}, sq;
      f2_sqr(&sq, &cand);
      if (f2_eq(&sq, a)) {
        *r = cand;
        return 1;
      }
    }
  }
  /* a1 == 0 and a0 a non-square: root = sqrt(-a0) u */
  fp na0;
  fp_neg(&na0, &a->c0);
  if (fp_is_zero(&a->c1) && fp_sqrt(&cs, &na0)) {
    memset(&r->c0, 0, sizeof(fp));
    r->c1 = cs;
    return 1;
  }
  return 0;
}
static int f2_sgn0(const fp2* a) {
  uint64_t v0[6], v1[6];
  fp_from_mont(v0, &a->c0);
  fp_from_mont(v1, &a->c1);
  int s0 = (int)(v0[0] & 1);
  int z0 = fp_is_zero(&a->c0);
  int s1 = (int)(v1[0] & 1);
  return s0 | (z0 & s1);
}
static int f2_lexi_largest(const fp2* y) {
  return fp_is_zero(&y->c1) ? canon_gt_half(&y->c0) : canon_gt_half(&y->c1);
}

/* ------------------------------------------------------------------ Fp6 / Fp12 */
static void f6_add(fp6* r, const fp6* a, const fp6* b) {
  f2_add(&r->c0, &a->c0, &b->c0);
  f2_add(&r->c1, &a->c1, &b->c1);
  f2_add(&r->c2, &a->c2, &b->c2);
}
static void f6_sub(fp6* r, const fp6* a, const fp6* b) {
  f2_sub(&r->c0, &a->c0, &b->c0);
  f2_sub(&r->c1, &a->c1, &b->c1);
  f2_sub(&r->c2, &a->c2, &b->c2);
}
static void f6_neg(fp6* r, const fp6* a) {
  f2_neg(&r->c0, &a->c0);
  f2_neg(&r->c1, &a->c1);
  f2_neg(&r->c2, &a->c2);
}
static void f6_mul_v(fp6* r, const fp6* a) {
  fp2 t;
  f2_mul_xi(&t, &a->c2);
  fp6 o = {t, a->c0, a->c1};
  *r = o;
}
static void f6_mul(fp6* r, const fp6* a, const fp6* b) {
  fp2 v0, v1, v2, s, t, u, c0, c1, c2;
  f2_mul(&v0, &a->c0, &b->c0);
  f2_mul(&v1, &a->c1, &b->c1);
  f2_mul(&v2, &a->c2, &b->c2);
  f2_add(&s, &a->c1, &a->c2);
  f2_add(&t, &b->c1, &b->c2);
  f2_mul(&u, &s, &t);
  f2_sub(&u, &u, &v1);
  f2_sub(&u, &u, &v2);
  f2_mul_xi(&u, &u);
  f2_add(&c0, &v0, &u);
  f2_add(&s, &a->c0, &a->c1);
  f2_add(&t, &b->c0, &b->c1);
  f2_mul(&u, &s, &t);
  f2_sub(&u, &u, &v0);
  f2_sub(&u, &u, &v1);
  f2_mul_xi(&s, &v2);
  f2_add(&c1, &u, &s);
  f2_add(&s, &a->c0, &a->c2);
  f2_add(&t, &b->c0, &b->c2);
  f2_mul(&u, &s, &t);
  f2_sub(&u, &u, &v0);
  f2_sub(&u, &u, &v2);
  f2_add(&c2, &u, &v1);
  r->c0 = c0;
  r->c1 = c1;
  r->c2 = c2;
}
static void f6_inv(fp6* r, const fp6* a) {
  fp2 t0, t1, t2, x, y, den, di;
  f2_sqr(&t0, &a->c0);
  f2_mul(&x, &a->c1, &a->c2);
  f2_mul_xi(&x, &x);
  f2_sub(&t0, &t0, &x);
  f2_sqr(&t1, &a->c2);
  f2_mul_xi(&t1, &t1);
  f2_mul(&x, &a->c0, &a->c1);
  f2_sub(&t1, &t1, &x);
  f2_sqr(&t2, &a->c1);
  f2_mul(&x, &a->c0, &a->c2);
  f2_sub(&t2, &t2, &x);
  f2_mul(&den, &a->c0, &t0);
  f2_mul(&x, &a->c2, &t1);
  f2_mul(&y, &a->c1, &t2);
  f2_add(&x, &x, &y);
  f2_mul_xi(&x, &x);
  f2_add(&den, &den, &x);
  f2_inv(&di, &den);
  f2_mul(&r->c0, &t0, &di);
  f2_mul(&r->c1, &t1, &di);
  f2_mul(&r->c2, &t2, &di);
}
static void f12_mul(fp12* r, const fp12* a, const fp12* b) {
  fp6 t0, t1, s, t, u;
  f6_mul(&t0, &a->c0, &b->c0);
  f6_mul(&t1, &a->c1, &b->c1);
  f6_add(&s, &a->c0, &a->c1);
  f6_add(&t, &b->c0, &b->c1);
  f6_mul(&u, &s, &t);
  f6_sub(&u, &u, &t0);
  f6_sub(&r->c1, &u, &t1);
  f6_mul_v(&t1, &t1);
  f6_add(&r->c0, &t0, &t1);
}
static void f12_sqr(fp12* r, const fp12* a) {
  fp6 t, u, s, v;
  f6_mul(&t, &a->c0, &a->c1);
  f6_add(&s, &a->c0, &a->c1);
  f6_mul_v(&v, &a->c1);
  f6_add(&v, &a->c0, &v);
  f6_mul(&u, &s, &v);
  f6_sub(&u, &u, &t);
  f6_mul_v(&v, &t);
  f6_sub(&r->c0, &u, &v);
  f6_add(&r->c1, &t, &t);
}
static void f12_conj(fp12* r, const fp12* a) {
  r->c0 = a->c0;
  f6_neg(&r->c1, &a->c1);
}
static void f12_inv(fp12* r, const fp12* a) {
  fp6 t0, t1, ti;
  f6_mul(&t0, &a->c0, &a->c0);
  f6_mul(&t1, &a->c1, &a->c1);
  f6_mul_v(&t1, &t1);
  f6_sub(&t0, &t0, &t1);
  f6_inv(&ti, &t0);
  f6_mul(&r->c0, &a->c0, &ti);
  f6_mul(&t1, &a->c1, &ti);
  f6_neg(&r->c1, &t1);
}
static void f12_one(fp12* r) {
  memset(r, 0, sizeof *r);
  r->c0.c0.c0 = C_ONE;
}
static int f12_is_one(const fp12* a) {
  fp12 o;
  f12_one(&o);
  return memcmp(a, &o, sizeof o) == 0;
}
/* a^p: coefficient of w^j (order c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2) is conj(c_j) g1_j */
static void f12_frob(fp12* r, const fp12* a) {
  fp2 t;
  f2_conj(&r->c0.c0, &a->c0.c0);
  f2_conj(&t, &a->c1.c0);
  f2_mul(&r->c1.c0, &t, &C_GAMMA1[1]);
  f2_conj(&t, &a->c0.c1);
  f2_mul(&r->c0.c1, &t, &C_GAMMA1[2]);
  f2_conj(&t, &a->c1.c1);
  f2_mul(&r->c1.c1, &t, &C_GAMMA1[3]);
  f2_conj(&t, &a->c0.c2);
  f2_mul(&r->c0.c2, &t, &C_GAMMA1[4]);
  f2_conj(&t, &a->c1.c2);
  f2_mul(&r->c1.c2, &t, &C_GAMMA1[5]);
}
static void f12_frob2(fp12* r, const fp12* a) {
  r->c0.c0 = a->c0.c0;
  f2_mul(&r->c1.c0, &a->c1.c0, &C_GAMMA2[1]);
  f2_mul(&r->c0.c1, &a->c0.c1, &C_GAMMA2[2]);
  f2_mul(&r->c1.c1, &a->c1.c1, &C_GAMMA2[3]);
  f2_mul(&r->c0.c2, &a->c0.c2, &C_GAMMA2[4]);
  f2_mul(&r->c1.c2, &a->c1.c2, &C_GAMMA2[5]);
}
/* Granger-Scott squaring (oracle/pairing.py f12_cyclotomic_sqr) */
static void fp4_square(fp2* c0, fp2* c1, const fp2* a, const fp2* b) {
  fp2 t0, t1, s;
  f2_sqr(&t0, a);
  f2_sqr(&t1, b);
  f2_mul_xi(c0, &t1);
  f2_add(c0, c0, &t0);
  f2_add(&s, a, b);
  f2_sqr(&s, &s);
  f2_sub(&s, &s, &t0);
  f2_sub(c1, &s, &t1);
}
static void f12_cyclo_sqr(fp12* r, const fp12* f) {
  fp2 z0 = f->c0.c0, z4 = f->c0.c1, z3 = f->c0.c2, z2 = f->c1.c0, z1 = f->c1.c1, z5 = f->c1.c2;
  fp2 t0, t1, u0, u1, t2, t3, x;
  fp4_square(&t0, &t1, &z0, &z1);
  fp4_square(&u0, &u1, &z2, &z3);
  fp4_square(&t2, &t3, &z4, &z5);
  f2_sub(&z0, &t0, &z0);
  f2_add(&z0, &z0, &z0);
  f2_add(&z0, &z0, &t0);
  f2_add(&z1, &t1, &z1);
  f2_add(&z1, &z1, &z1);
  f2_add(&z1, &z1, &t1);
  f2_sub(&z4, &u0, &z4);
  f2_add(&z4, &z4, &z4);
  f2_add(&z4, &z4, &u0);
  f2_add(&z5, &u1, &z5);
  f2_add(&z5, &z5, &z5);
  f2_add(&z5, &z5, &u1);
  f2_mul_xi(&x, &t3);
  f2_add(&z2, &x, &z2);
  f2_add(&z2, &z2, &z2);
  f2_add(&z2, &z2, &x);
  f2_sub(&z3, &t2, &z3);
  f2_add(&z3, &z3, &z3);
  f2_add(&z3, &z3, &t2);
  r->c0.c0 = z0;
  r->c0.c1 = z4;
  r->c0.c2 = z3;
  r->c1.c0 = z2;
  r->c1.c1 = z1;
  r->c1.c2 = z5;
}

/* ------------------------------------------------------------------ curves: homogeneous
 * projective, Renes-Costello-Batina complete formulas (a = 0), b3 = 3b */
typedef struct {
  fp X, Y, Z;
} g1p;
typedef struct {
  fp2 X, Y, Z;
} g2p;

static void fp_mul_b3(fp* r, const fp* a) { /* 12 a */
  fp t;
  fp_add(&t, a, a);
  fp_add(&t, &t, &t);
  fp_add(r, &t, &t);
  fp_add(r, r, &t);
}
static void f2_mul_b3(fp2* r, const fp2* a) { /* 12 (1 + u) a */
  fp2 t;
  f2_mul_xi(&t, a);
  fp_mul_b3(&r->c0, &t.c0);
  fp_mul_b3(&r->c1, &t.c1);
}

#define DEFINE_CURVE(G, F, ADD, SUB, MUL, MB3, ZERO_P, FONE)                                      \
  static void G##_add(G* r, const G* p, const G* q) {                                             \
    F t0, t1, t2, t3, t4, X3, Y3, Z3, s, u;                                                       \
    MUL(&t0, &p->X, &q->X);                                                                       \
    MUL(&t1, &p->Y, &q->Y);                                                                       \
    MUL(&t2, &p->Z, &q->Z);                                                                       \
    ADD(&s, &p->X, &p->Y);                                                                        \
    ADD(&u, &q->X, &q->Y);                                                                        \
    MUL(&t3, &s, &u);                                                                             \
    ADD(&t4, &t0, &t1);                                                                           \
    SUB(&t3, &t3, &t4);                                                                           \
    ADD(&s, &p->Y, &p->Z);                                                                        \
    ADD(&u, &q->Y, &q->Z);                                                                        \
    MUL(&t4, &s, &u);                                                                             \
    ADD(&X3, &t1, &t2);                                                                           \
    SUB(&t4, &t4, &X3);                                                                           \
    ADD(&s, &p->X, &p->Z);                                                                        \
    ADD(&u, &q->X, &q->Z);                                                                        \
    MUL(&X3, &s, &u);                                                                             \
    ADD(&Y3, &t0, &t2);                                                                           \
    SUB(&Y3, &X3, &Y3);                                                                           \
    ADD(&X3, &t0, &t0);                                                                           \
    ADD(&t0, &X3, &t0);                                                                           \
    MB3(&t2, &t2);                                                                                \
    ADD(&Z3, &t1, &t2);                                                                           \
    SUB(&t1, &t1, &t2);                                                                           \
    MB3(&Y3, &Y3);                                                                                \
    MUL(&X3, &t4, &Y3);                                                                           \
    MUL(&t2, &t3, &t1);                                                                           \
    SUB(&X3, &t2, &X3);                                                                           \
    MUL(&Y3, &Y3, &t0);                                                                           \
    MUL(&t1, &t1, &Z3);                                                                           \
    ADD(&Y3, &t1, &Y3);                                                                           \
    MUL(&t0, &t0, &t3);                                                                           \
    MUL(&Z3, &Z3, &t4);                                                                           \
    ADD(&Z3, &Z3, &t0);                                                                           \
    r->X = X3;                                                                                    \
    r->Y = Y3;                                                                                    \
    r->Z = Z3;                                                                                    \
  }                                                                                               \
  static void G##_dbl(G* r, const G* p) {                                                         \
    F t0, t1, t2, X3, Y3, Z3;                                                                     \
    MUL(&t0, &p->Y, &p->Y);                                                                       \
    ADD(&Z3, &t0, &t0);                                                                           \
    ADD(&Z3, &Z3, &Z3);                                                                           \
    ADD(&Z3, &Z3, &Z3);                                                                           \
    MUL(&t1, &p->Y, &p->Z);                                                                       \
    MUL(&t2, &p->Z, &p->Z);                                                                       \
    MB3(&t2, &t2);                                                                                \
    MUL(&X3, &t2, &Z3);                                                                           \
    ADD(&Y3, &t0, &t2);                                                                           \
    MUL(&Z3, &t1, &Z3);                                                                           \
    ADD(&t1, &t2, &t2);                                                                           \
    ADD(&t2, &t1, &t2);                                                                           \
    SUB(&t0, &t0, &t2);                                                                           \
    MUL(&Y3, &t0, &Y3);                                                                           \
    ADD(&Y3, &X3, &Y3);                                                                           \
    MUL(&t1, &p->X, &p->Y);                                                                       \
    MUL(&X3, &t0, &t1);                                                                           \
    ADD(&X3, &X3, &X3);                                                                           \
    r->X = X3;                                                                                    \
    r->Y = Y3;                                                                                    \
    r->Z = Z3;                                                                                    \
  }                                                                                               \
  static void G##_mul_u64(G* r, const G* p, uint64_t k) {                                         \
    G acc;                                                                                        \
    memset(&acc, 0, sizeof acc);                                                                  \
    acc.Y = FONE;                                                                                 \
    for (int b = 63; b >= 0; b--) {                                                               \
      G##_dbl(&acc, &acc);                                                                        \
      if ((k >> b) & 1) G##_add(&acc, &acc, p);                                                   \
    }                                                                                             \
    *r = acc;                                                                                     \
  }

DEFINE_CURVE(g1p, fp, fp_add, fp_sub, fp_mul, fp_mul_b3, fp_is_zero, C_ONE)
static fp2 f2_one_v(void) {
  fp2 o;
  memset(&o, 0, sizeof o);
  o.c0 = C_ONE;
  return o;
}
#define F2ONE f2_one_v()
DEFINE_CURVE(g2p, fp2, f2_add, f2_sub, f2_mul, f2_mul_b3, f2_is_zero, F2ONE)

static int g2p_eq(const g2p* a, const g2p* b) {
  int ia = f2_is_zero(&a->Z), ib = f2_is_zero(&b->Z);
  if (ia || ib) return ia && ib;
  fp2 l, r;
  f2_mul(&l, &a->X, &b->Z);
  f2_mul(&r, &b->X, &a->Z);
  if (!f2_eq(&l, &r)) return 0;
  f2_mul(&l, &a->Y, &b->Z);
  f2_mul(&r, &b->Y, &a->Z);
  return f2_eq(&l, &r);
}
static void g2_psi(g2p* r, const g2p* p) {
  fp2 t;
  f2_conj(&t, &p->X);
  f2_mul(&r->X, &t, &C_PSI_CX);
  f2_conj(&t, &p->Y);
  f2_mul(&r->Y, &t, &C_PSI_CY);
  f2_conj(&r->Z, &p->Z);
}
static void g2_mul_xabs(g2p* r, const g2p* p) {
  g2p acc = *p;
  for (int b = 62; b >= 0; b--) {
    g2p_dbl(&acc, &acc);
    if ((C_X_ABS >> b) & 1) g2p_add(&acc, &acc, p);
  }
  *r = acc;
}
/* Scott's G2 membership test psi(P) == [x]P, x < 0 (oracle/curves.py in_g2_psi) */
static int g2_in_group(const g2p* p) {
  if (f2_is_zero(&p->Z)) return 1;
  g2p xp, ps;
  g2_mul_xabs(&xp, p);
  f2_neg(&xp.Y, &xp.Y);
  g2_psi(&ps, p);
  return g2p_eq(&ps, &xp);
}
static void g2p_to_aff(fp2* x, fp2* y, const g2p* p) {
  fp2 zi;
  f2_inv(&zi, &p->Z);
  f2_mul(x, &p->X, &zi);
  f2_mul(y, &p->Y, &zi);
}
static void g1p_to_aff(fp* x, fp* y, const g1p* p) {
  fp zi;
  fp_inv(&zi, &p->Z);
  fp_mul(x, &p->X, &zi);
  fp_mul(y, &p->Y, &zi);
}

/* ------------------------------------------------------------------ (de)serialisation (ZCash) */
enum { E_OK = 0, E_BAD_ENCODING = 1, E_NOT_ON_CURVE = 2, E_NOT_IN_GROUP = 3, E_PK_INF = 6, E_INVALID_SIZE = 10 };

static int read_fp48(fp* r, const uint8_t* b) {
  uint64_t v[6];
  be_to_limbs(v, b, 48);
  v[5] &= (1ull << 61) - 1; /* the 3 flag bits */
  if (!lt_p(v)) return E_BAD_ENCODING;
  fp_from_canon(r, v);
  return E_OK;
}
/* blst POINTonE2_Uncompress_Z + subgroup check (oracle/curves.py g2_uncompress, in_g2);
 * *inf = 1 for the point at infinity */
static int g2_decode_sig(fp2* x, fp2* y, int* inf, const uint8_t* b, size_t len) {
  *inf = 0;
  if (len != 96 && len != 192) return E_INVALID_SIZE;
  uint8_t in0 = b[0];
  if (len != 96 || !(in0 & 0x80)) return E_BAD_ENCODING; /* this baseline takes compressed signatures */
  if (in0 & 0x40) {
    if ((in0 & 0x3f) != 0) return E_BAD_ENCODING;
    for (int i = 1; i < 96; i++)
      if (b[i]) return E_BAD_ENCODING;
    *inf = 1;
    return E_OK;
  }
  int e;
  if ((e = read_fp48(&x->c1, b)) || (e = read_fp48(&x->c0, b + 48))) return e;
  fp2 rhs, t, b2;
  f2_sqr(&t, x);
  f2_mul(&rhs, &t, x);
  b2.c0 = C_ONE;
  fp_add(&b2.c0, &b2.c0, &b2.c0);
  fp_add(&b2.c0, &b2.c0, &b2.c0); /* 4 */
  b2.c1 = b2.c0;
  f2_add(&rhs, &rhs, &b2);
  if (!f2_sqrt(y, &rhs)) return E_NOT_ON_CURVE;
  if (f2_lexi_largest(y) != !!(in0 & 0x20)) f2_neg(y, y);
  if (f2_is_zero(x)) return E_NOT_IN_GROUP;
  g2p p = {*x, *y, f2_one_v()};
  if (!g2_in_group(&p)) return E_NOT_IN_GROUP;
  return E_OK;
}
/* blst_p1_deserialize of a 96-byte uncompressed key, on-curve only (worker.ts:108-114) */
static int g1_decode_pk(fp* x, fp* y, int* inf, const uint8_t* b) {
  *inf = 0;
  uint8_t in0 = b[0];
  if (in0 & 0x80) return E_BAD_ENCODING;
  if (in0 & 0x40) {
    if ((in0 & 0x3f) != 0) return E_BAD_ENCODING;
    for (int i = 1; i < 96; i++)
      if (b[i]) return E_BAD_ENCODING;
    *inf = 1;
    return E_OK;
  }
  if (in0 & 0x20) return E_BAD_ENCODING;
  int e;
  if ((e = read_fp48(x, b)) || (e = read_fp48(y, b + 48))) return e;
  fp l, r, t, four = C_ONE;
  fp_add(&four, &four, &four);
  fp_add(&four, &four, &four);
  fp_sqr(&l, y);
  fp_sqr(&t, x);
  fp_mul(&r, &t, x);
  fp_add(&r, &r, &four);
  if (!fp_eq(&l, &r)) return E_NOT_ON_CURVE;
  if (fp_is_zero(x)) return E_NOT_IN_GROUP;
  return E_OK;
}

/* ------------------------------------------------------------------ SHA-256 + hash_to_G2 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
    0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
    0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
    0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha256_block(uint32_t* h, const uint8_t* blk) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) | ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}
/* SHA-256 of the concatenation of up to 4 byte strings */
static void sha256_cat(uint8_t out[32], const uint8_t* const* parts, const size_t* lens, int np) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t blk[64];
  size_t fill = 0, total = 0;
  for (int k = 0; k < np; k++)
    for (size_t i = 0; i < lens[k]; i++) {
      blk[fill++] = parts[k][i];
      total++;
      if (fill == 64) {
        sha256_block(h, blk);
        fill = 0;
      }
    }
  blk[fill++] = 0x80;
  if (fill > 56) {
    while (fill < 64) blk[fill++] = 0;
    sha256_block(h, blk);
    fill = 0;
  }
  while (fill < 56) blk[fill++] = 0;
  uint64_t bits = (uint64_t)total * 8;
  for (int i = 0; i < 8; i++) blk[56 + i] = (uint8_t)(bits >> (56 - 8 * i));
  sha256_block(h, blk);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(h[i] >> 8);
    out[4 * i + 3] = (uint8_t)h[i];
  }
}
/* RFC 9380 5.3.1, len_in_bytes = 256 (oracle/hash_to_curve.py expand_message_xmd) */
static void expand_xmd_256(uint8_t out[256], const uint8_t* msg, size_t mlen, const uint8_t* dst, size_t dlen) {
  uint8_t zpad[64] = {0}, lib[3] = {1, 0, 0}, dprime[256], b0[32], bi[32], x[33];
  memcpy(dprime, dst, dlen);
  dprime[dlen] = (uint8_t)dlen;
  const uint8_t* p0[4] = {zpad, msg, lib, dprime};
  size_t l0[4] = {64, mlen, 3, dlen + 1};
  sha256_cat(b0, p0, l0, 4);
  for (int i = 1; i <= 8; i++) {
    for (int k = 0; k < 32; k++) x[k] = (i == 1) ? b0[k] : (uint8_t)(b0[k] ^ bi[k]);
    x[32] = (uint8_t)i;
    const uint8_t* p1[2] = {x, dprime};
    size_t l1[2] = {33, dlen + 1};
    sha256_cat(bi, p1, l1, 2);
    memcpy(out + 32 * (i - 1), bi, 32);
  }
}
/* 64 big-endian bytes -> Fp (Montgomery): hi * 2^256 + lo with hi, lo < 2^256 < p */
static void fp_from_be64_mod(fp* r, const uint8_t* b) {
  uint64_t hi[6], lo[6];
  be_to_limbs(hi, b, 32);
  be_to_limbs(lo, b + 32, 32);
  fp h, l;
  fp_from_canon(&h, hi);
  fp_from_canon(&l, lo);
  fp_mul(&h, &h, &C_2P256);
  fp_add(r, &h, &l);
}
/* RFC 9380 6.6.2 simplified SWU on E2' (oracle map_to_curve_sswu) */
static void map_to_curve_sswu(fp2* x, fp2* y, const fp2* u) {
  fp2 u2, zu2, tv1, x1, gx1, x2, gx2, t, one = f2_one_v();
  f2_sqr(&u2, u);
  f2_mul(&zu2, &C_SSWU_Z, &u2);
  f2_sqr(&tv1, &zu2);
  f2_add(&tv1, &tv1, &zu2);
  if (f2_is_zero(&tv1)) {
    f2_mul(&t, &C_SSWU_Z, &C_SSWU_A);
    f2_inv(&t, &t);
    f2_mul(&x1, &C_SSWU_B, &t);
  } else {
    fp2 nb, ai, ti;
    f2_neg(&nb, &C_SSWU_B);
    f2_inv(&ai, &C_SSWU_A);
    f2_mul(&nb, &nb, &ai);
    f2_inv(&ti, &tv1);
    f2_add(&ti, &one, &ti);
    f2_mul(&x1, &nb, &ti);
  }
  f2_sqr(&t, &x1);
  f2_mul(&gx1, &t, &x1);
  f2_mul(&t, &C_SSWU_A, &x1);
  f2_add(&gx1, &gx1, &t);
  f2_add(&gx1, &gx1, &C_SSWU_B);
  f2_mul(&x2, &zu2, &x1);
  f2_sqr(&t, &x2);
  f2_mul(&gx2, &t, &x2);
  f2_mul(&t, &C_SSWU_A, &x2);
  f2_add(&gx2, &gx2, &t);
  f2_add(&gx2, &gx2, &C_SSWU_B);
  if (f2_sqrt(y, &gx1)) {
    *x = x1;
  } else {
    (void)f2_sqrt(y, &gx2);
    *x = x2;
  }
  if (f2_sgn0(u) != f2_sgn0(y)) f2_neg(y, y);
}
static void peval(fp2* r, const fp2* c, int n, const fp2* x) {
  fp2 acc;
  memset(&acc, 0, sizeof acc);
  for (int i = n - 1; i >= 0; i--) {
    f2_mul(&acc, &acc, x);
    f2_add(&acc, &acc, &c[i]);
  }
  *r = acc;
}
#define NELEM(a) ((int)(sizeof(a) / sizeof((a)[0])))
/* 3-isogeny E2' -> E2, projective (xn yd : y yn xd : xd yd) */
static void iso_map3(g2p* r, const fp2* x, const fp2* y) {
  fp2 xn, xd, yn, yd, t;
  peval(&xn, C_ISO_XNUM, NELEM(C_ISO_XNUM), x);
  peval(&xd, C_ISO_XDEN, NELEM(C_ISO_XDEN), x);
  peval(&yn, C_ISO_YNUM, NELEM(C_ISO_YNUM), x);
  peval(&yd, C_ISO_YDEN, NELEM(C_ISO_YDEN), x);
  f2_mul(&r->X, &xn, &yd);
  f2_mul(&t, y, &yn);
  f2_mul(&r->Y, &t, &xd);
  f2_mul(&r->Z, &xd, &yd);
  if (f2_is_zero(&r->Z)) {
    memset(r, 0, sizeof *r);
    r->Y = f2_one_v();
  }
}
/* h_eff P = [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P)  (RFC 9380 G.3) */
static void clear_cofactor(g2p* r, const g2p* p) {
  g2p t1, t2, t3, u;
  g2_mul_xabs(&t1, p);
  f2_neg(&t1.Y, &t1.Y); /* [x]P */
  g2_psi(&t2, p);
  g2p_dbl(&t3, p);
  g2_psi(&t3, &t3);
  g2_psi(&t3, &t3);
  u = t2;
  f2_neg(&u.Y, &u.Y);
  g2p_add(&t3, &t3, &u);
  g2p_add(&t2, &t1, &t2);
  g2_mul_xabs(&t2, &t2);
  f2_neg(&t2.Y, &t2.Y);
  g2p_add(&t3, &t3, &t2);
  u = t1;
  f2_neg(&u.Y, &u.Y);
  g2p_add(&t3, &t3, &u);
  u = *p;
  f2_neg(&u.Y, &u.Y);
  g2p_add(r, &t3, &u);
}
static const uint8_t DST_POP[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
static void hash_to_g2(g2p* r, const uint8_t* msg, size_t mlen, const uint8_t* dst, size_t dlen) {
  uint8_t ub[256];
  expand_xmd_256(ub, msg, mlen, dst, dlen);
  fp2 u0, u1, x, y;
  fp_from_be64_mod(&u0.c0, ub);
  fp_from_be64_mod(&u0.c1, ub + 64);
  fp_from_be64_mod(&u1.c0, ub + 128);
  fp_from_be64_mod(&u1.c1, ub + 192);
  g2p q0, q1;
  map_to_curve_sswu(&x, &y, &u0);
  iso_map3(&q0, &x, &y);
  map_to_curve_sswu(&x, &y, &u1);
  iso_map3(&q1, &x, &y);
  g2p_add(&q0, &q0, &q1);
  clear_cofactor(r, &q0);
}

/* ------------------------------------------------------------------ pairing (oracle/pairing.py) */
typedef struct {
  fp2 l00, l01, l11;
} line_t;
static void dbl_step(line_t* L, g2p* T, const fp* xP, const fp* yP) {
  fp2 t0, t1, t2, XX, XX3, Z3, X3, Y3, u1, u2, s0, v1, t;
  f2_sqr(&t0, &T->Y);
  f2_mul(&t1, &T->Y, &T->Z);
  f2_sqr(&t2, &T->Z);
  f2_mul_b3(&t2, &t2);
  f2_sqr(&XX, &T->X);
  f2_sub(&L->l00, &t2, &t0);
  f2_add(&XX3, &XX, &XX);
  f2_add(&XX3, &XX3, &XX);
  f2_mul_fp(&L->l01, &XX3, xP);
  f2_add(&t, &t1, &t1);
  f2_neg(&t, &t);
  f2_mul_fp(&L->l11, &t, yP);
  f2_add(&Z3, &t0, &t0);
  f2_add(&Z3, &Z3, &Z3);
  f2_add(&Z3, &Z3, &Z3);
  f2_mul(&X3, &t2, &Z3);
  f2_add(&Y3, &t0, &t2);
  f2_mul(&Z3, &t1, &Z3);
  f2_add(&u1, &t2, &t2);
  f2_add(&u2, &u1, &t2);
  f2_sub(&s0, &t0, &u2);
  f2_mul(&Y3, &s0, &Y3);
  f2_add(&Y3, &X3, &Y3);
  f2_mul(&v1, &T->X, &T->Y);
  f2_mul(&X3, &s0, &v1);
  f2_add(&X3, &X3, &X3);
  T->X = X3;
  T->Y = Y3;
  T->Z = Z3;
}
static void add_step(line_t* L, g2p* T, const fp2* xQ, const fp2* yQ, const fp* xP, const fp* yP) {
  fp2 theta, delta, t, C, D, E, F, G, H, X3, Y3, Z3;
  f2_mul(&t, yQ, &T->Z);
  f2_sub(&theta, &T->Y, &t);
  f2_mul(&t, xQ, &T->Z);
  f2_sub(&delta, &T->X, &t);
  fp2 a, b;
  f2_mul(&a, &delta, yQ);
  f2_mul(&b, &theta, xQ);
  f2_sub(&L->l00, &a, &b);
  f2_mul_fp(&L->l01, &theta, xP);
  f2_neg(&t, &delta);
  f2_mul_fp(&L->l11, &t, yP);
  f2_sqr(&C, &theta);
  f2_sqr(&D, &delta);
  f2_mul(&E, &D, &delta);
  f2_mul(&F, &T->Z, &C);
  f2_mul(&G, &T->X, &D);
  f2_add(&H, &E, &F);
  f2_add(&t, &G, &G);
  f2_sub(&H, &H, &t);
  f2_mul(&X3, &delta, &H);
  f2_sub(&t, &G, &H);
  f2_mul(&Y3, &theta, &t);
  f2_mul(&t, &E, &T->Y);
  f2_sub(&Y3, &Y3, &t);
  f2_mul(&Z3, &E, &T->Z);
  T->X = X3;
  T->Y = Y3;
  T->Z = Z3;
}
static void f6_mul_01(fp6* r, const fp6* a, const fp2* b0, const fp2* b1) {
  fp2 t0, t1, c0, c1, c2, s, u;
  f2_mul(&t0, &a->c0, b0);
  f2_mul(&t1, &a->c1, b1);
  f2_mul(&c0, &a->c2, b1);
  f2_mul_xi(&c0, &c0);
  f2_add(&c0, &c0, &t0);
  f2_add(&s, &a->c0, &a->c1);
  f2_add(&u, b0, b1);
  f2_mul(&c1, &s, &u);
  f2_sub(&c1, &c1, &t0);
  f2_sub(&c1, &c1, &t1);
  f2_mul(&c2, &a->c2, b0);
  f2_add(&c2, &c2, &t1);
  r->c0 = c0;
  r->c1 = c1;
  r->c2 = c2;
}
static void f6_mul_1(fp6* r, const fp6* a, const fp2* b1) {
  fp2 c0, c1, c2;
  f2_mul(&c0, &a->c2, b1);
  f2_mul_xi(&c0, &c0);
  f2_mul(&c1, &a->c0, b1);
  f2_mul(&c2, &a->c1, b1);
  r->c0 = c0;
  r->c1 = c1;
  r->c2 = c2;
}
static void f12_mul_line(fp12* f, const line_t* L) {
  fp6 t0, t1, s, u;
  fp2 m;
  f6_mul_01(&t0, &f->c0, &L->l00, &L->l01);
  f6_mul_1(&t1, &f->c1, &L->l11);
  f6_add(&s, &f->c0, &f->c1);
  f2_add(&m, &L->l01, &L->l11);
  f6_mul_01(&u, &s, &L->l00, &m);
  f6_sub(&u, &u, &t0);
  f6_sub(&f->c1, &u, &t1);
  f6_mul_v(&t1, &t1);
  f6_add(&f->c0, &t0, &t1);
}
/* prod_k conj(f_{|x|,Q_k}(P_k)): one f, shared squarings (blst miller_loop_n) */
static void miller_loop_n(fp12* out, const fp* xP, const fp* yP, const fp2* xQ, const fp2* yQ, int n) {
  g2p T[17];
  fp12 f;
  f12_one(&f);
  int first = 1;
  for (int k = 0; k < n; k++) {
    T[k].X = xQ[k];
    T[k].Y = yQ[k];
    T[k].Z = f2_one_v();
  }
  for (int b = 62; b >= 0; b--) {
    if (!first) f12_sqr(&f, &f);
    for (int k = 0; k < n; k++) {
      line_t L;
      dbl_step(&L, &T[k], &xP[k], &yP[k]);
      f12_mul_line(&f, &L);
    }
    first = 0;
    if ((C_X_ABS >> b) & 1)
      for (int k = 0; k < n; k++) {
        line_t L;
        add_step(&L, &T[k], &xQ[k], &yQ[k], &xP[k], &yP[k]);
        f12_mul_line(&f, &L);
      }
  }
  f12_conj(out, &f);
}
static void f12_exp_by_x(fp12* r, const fp12* g) {
  fp12 res = *g;
  for (int b = 62; b >= 0; b--) {
    f12_cyclo_sqr(&res, &res);
    if ((C_X_ABS >> b) & 1) f12_mul(&res, &res, g);
  }
  f12_conj(r, &res);
}
/* f^(3 (p^12 - 1)/r)  (oracle final_exp_fast) */
static void final_exp(fp12* r, const fp12* f) {
  fp12 f1, fi, g, t0, t1, t2, u, v;
  f12_conj(&f1, f);
  f12_inv(&fi, f);
  f12_mul(&f1, &f1, &fi);
  f12_frob2(&g, &f1);
  f12_mul(&g, &g, &f1);
  f12_exp_by_x(&t0, &g);
  f12_conj(&u, &g);
  f12_mul(&t0, &t0, &u);
  f12_exp_by_x(&v, &t0);
  f12_conj(&u, &t0);
  f12_mul(&t0, &v, &u);
  f12_exp_by_x(&t1, &t0);
  f12_frob(&u, &t0);
  f12_mul(&t1, &t1, &u);
  f12_exp_by_x(&t2, &t1);
  f12_exp_by_x(&t2, &t2);
  f12_frob2(&u, &t1);
  f12_mul(&t2, &t2, &u);
  f12_conj(&u, &t1);
  f12_mul(&t2, &t2, &u);
  f12_sqr(&u, &g);
  f12_mul(&u, &u, &g);
  f12_mul(r, &t2, &u);
}

/* ------------------------------------------------------------------ verification */
static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

/* verifySignatureSetsMaybeBatch (maybeBatch.ts:16-39) over n <= 16 single-pubkey sets:
 * n >= 2 -> RLC batch, n == 1 -> verify.  Returns 1 valid, 0 invalid, -code on error. */
static int verify_sets(const uint8_t* pks96, const uint8_t* msgs32, const uint8_t* sigs96, int n, uint64_t seed) {
  if (n <= 0 || n > 16) return -100;
  fp xP[17], yP[17];
  fp2 xQ[17], yQ[17];
  g2p S;
  memset(&S, 0, sizeof S);
  S.Y = f2_one_v();
  int m = 0;
  for (int i = 0; i < n; i++) {
    fp2 sx, sy;
    int sinf, pinf, e;
    if ((e = g2_decode_sig(&sx, &sy, &sinf, sigs96 + 96 * i, 96))) return -e;
    fp px, py;
    if ((e = g1_decode_pk(&px, &py, &pinf, pks96 + 96 * i))) return -e;
    if (pinf) return -E_PK_INF;
    uint64_t r = 1;
    if (n >= 2) do r = splitmix(&seed); while (r == 0);
    g2p h;
    hash_to_g2(&h, msgs32 + 32 * i, 32, DST_POP, sizeof(DST_POP) - 1);
    if (!sinf) {
      g2p sp = {sx, sy, f2_one_v()}, rs;
      g2p_mul_u64(&rs, &sp, r);
      g2p_add(&S, &S, &rs);
    }
    g1p pp = {px, py, C_ONE}, rp;
    g1p_mul_u64(&rp, &pp, r);
    g1p_to_aff(&xP[m], &yP[m], &rp);
    g2p_to_aff(&xQ[m], &yQ[m], &h);
    m++;
  }
  if (!f2_is_zero(&S.Z)) {
    xP[m] = C_G1_X;
    yP[m] = C_G1_NEG_Y;
    g2p_to_aff(&xQ[m], &yQ[m], &S);
    m++;
  }
  fp12 f, e;
  miller_loop_n(&f, xP, yP, xQ, yQ, m);
  final_exp(&e, &f);
  return f12_is_one(&e);
}

typedef struct {
  const uint8_t *pks, *msgs, *sigs;
  size_t n;
  int chunk;
  int* verdicts;
  size_t next;
  pthread_mutex_t mu;
  uint64_t seed;
} job_t;

static void* worker(void* arg) {
  job_t* J = (job_t*)arg;
  for (;;) {
    pthread_mutex_lock(&J->mu);
    size_t c = J->next++;
    pthread_mutex_unlock(&J->mu);
    size_t first = c * (size_t)J->chunk;
    if (first >= J->n) break;
    int cnt = (int)((J->n - first < (size_t)J->chunk) ? J->n - first : (size_t)J->chunk);
    J->verdicts[c] = verify_sets(J->pks + 96 * first, J->msgs + 32 * first, J->sigs + 96 * first, cnt,
                                 J->seed ^ (0x1234567ull * (c + 1)));
  }
  return NULL;
}

/* ------------------------------------------------------------------ exported (ctypes) */
/* n sets (96-byte uncompressed pubkeys, 32-byte messages, 96-byte compressed signatures),
 * verified in RLC chunks of `chunk` sets (worker.ts batches of >= 16 jobs) on `threads`
 * pthreads; verdicts[c] per chunk (1 valid, 0 invalid, <0 error).  Returns #valid chunks. */
int cpu_verify_chunks(const uint8_t* pks96, const uint8_t* msgs32, const uint8_t* sigs96, size_t n, int chunk,
                      int threads, uint64_t seed, int* verdicts) {
  if (chunk < 1 || chunk > 16 || threads < 1) return -1;
  job_t J = {pks96, msgs32, sigs96, n, chunk, verdicts, 0, PTHREAD_MUTEX_INITIALIZER, seed};
  pthread_t th[512];
  if (threads > 512) threads = 512;
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, &J);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  size_t nc = (n + chunk - 1) / chunk;
  int ok = 0;
  for (size_t c = 0; c < nc; c++) ok += verdicts[c] == 1;
  return ok;
}

static void g2_aff_to_bytes(uint8_t out[192], const g2p* p) {
  if (f2_is_zero(&p->Z)) {
    memset(out, 0, 192);
    out[0] = 0x40;
    return;
  }
  fp2 x, y;
  g2p_to_aff(&x, &y, p);
  fp_to_be48(out, &x.c1);
  fp_to_be48(out + 48, &x.c0);
  fp_to_be48(out + 96, &y.c1);
  fp_to_be48(out + 144, &y.c0);
}
/* hash_to_G2 -> 192-byte uncompressed (parity with tests/golden/hash_to_g2.json) */
void cpu_hash_to_g2(const uint8_t* msg, size_t mlen, const uint8_t* dst, size_t dlen, uint8_t out[192]) {
  g2p h;
  hash_to_g2(&h, msg, mlen, dst, dlen);
  g2_aff_to_bytes(out, &h);
}
/* Signature.fromBytes(sig, affine, validate) -> error code; out192 uncompressed if ok */
int cpu_sig_decode(const uint8_t* sig, size_t len, uint8_t out[192]) {
  fp2 x, y;
  int inf;
  int e = g2_decode_sig(&x, &y, &inf, sig, len);
  if (e) return e;
  g2p p = {x, y, f2_one_v()};
  if (inf) memset(&p, 0, sizeof p);
  g2_aff_to_bytes(out, &p);
  return 0;
}
/* maybeBatch over n <= 16 sets with a fixed seed: 1 / 0 / -code */
int cpu_verify_sets(const uint8_t* pks96, const uint8_t* msgs32, const uint8_t* sigs96, int n, uint64_t seed) {
  return verify_sets(pks96, msgs32, sigs96, n, seed);
}
