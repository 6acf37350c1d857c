// G1 (over Fp) and G2 (over Fp2) group law for gfx950, homogeneous projective coordinates
// with the Renes-Costello-Batina complete formulas (a = 0).  Replaces blst's POINTonE1/E2
// code reached through @chainsafe/bls PublicKey.aggregate (packages/beacon-node/src/chain/
// bls/utils.ts:11), Signature.fromBytes(..., validate) (maybeBatch.ts:23,36) and the
// Pairing.mul_n_aggregate randomizer multiplications.
#pragma once
#include "lsg_tower.hpp"

// ---- overload set so one template serves G1 and G2
LSG_INL fp_t fadd(const fp_t& a, const fp_t& b) { return fp_add(a, b); }
LSG_INL fp2_t fadd(const fp2_t& a, const fp2_t& b) { return fp2_add(a, b); }
LSG_INL fp_t fsub(const fp_t& a, const fp_t& b) { return fp_sub(a, b); }
LSG_INL fp2_t fsub(const fp2_t& a, const fp2_t& b) { return fp2_sub(a, b); }
LSG_INL fp_t fmul(const fp_t& a, const fp_t& b) { return fp_mul(a, b); }
LSG_INL fp2_t fmul(const fp2_t& a, const fp2_t& b) { return fp2_mul(a, b); }
LSG_INL fp_t fsqr(const fp_t& a) { return fp_sqr(a); }
LSG_INL fp2_t fsqr(const fp2_t& a) { return fp2_sqr(a); }
LSG_INL fp_t fneg(const fp_t& a) { return fp_neg(a); }
LSG_INL fp2_t fneg(const fp2_t& a) { return fp2_neg(a); }
LSG_INL fp_t fmul_b3(const fp_t& a) { return fp_mul12(a); }
LSG_INL fp2_t fmul_b3(const fp2_t& a) { return fp2_mul_b3(a); }
LSG_INL bool fis_zero(const fp_t& a) { return fp_is_zero(a); }
LSG_INL bool fis_zero(const fp2_t& a) { return fp2_is_zero(a); }
LSG_INL bool feq(const fp_t& a, const fp_t& b) { return fp_eq(a, b); }
LSG_INL bool feq(const fp2_t& a, const fp2_t& b) { return fp2_eq(a, b); }
LSG_INL fp_t fselect(bool c, const fp_t& a, const fp_t& b) { return fp_select(c, a, b); }
LSG_INL fp2_t fselect(bool c, const fp2_t& a, const fp2_t& b) { return fp2_select(c, a, b); }
LSG_INL fp_t finv(const fp_t& a) { return fp_inv(a); }
LSG_INL fp2_t finv(const fp2_t& a) { return fp2_inv(a); }
template <class F> LSG_INL F fzero();
template <> LSG_INL fp_t fzero<fp_t>() { return fp_zero(); }
template <> LSG_INL fp2_t fzero<fp2_t>() { return fp2_zero(); }
template <class F> LSG_INL F fone();
template <> LSG_INL fp_t fone<fp_t>() { return FP_ONE; }
template <> LSG_INL fp2_t fone<fp2_t>() { return fp2_one(); }

template <class F>
struct aff_t {
  F x, y;
};
template <class F>
struct proj_t {
  F X, Y, Z;
};
typedef aff_t<fp_t> g1a_t;
typedef aff_t<fp2_t> g2a_t;
typedef proj_t<fp_t> g1p_t;
typedef proj_t<fp2_t> g2p_t;

template <class F>
LSG_INL proj_t<F> proj_inf() {
  proj_t<F> r;
  r.X = fzero<F>();
  r.Y = fone<F>();
  r.Z = fzero<F>();
  return r;
}

template <class F>
LSG_INL proj_t<F> proj_from_aff(const aff_t<F>& a) {
  proj_t<F> r;
  r.X = a.x;
  r.Y = a.y;
  r.Z = fone<F>();
  return r;
}

template <class F>
LSG_INL bool proj_is_inf(const proj_t<F>& a) {
  return fis_zero(a.Z);
}

template <class F>
LSG_INL proj_t<F> proj_neg(const proj_t<F>& a) {
  proj_t<F> r = a;
  r.Y = fneg(a.Y);
  return r;
}

// RCB 2016 algorithm 7 (complete addition, a = 0)
template <class F>
LSG_INL proj_t<F> proj_add(const proj_t<F>& p, const proj_t<F>& q) {
  F t0 = fmul(p.X, q.X);
  F t1 = fmul(p.Y, q.Y);
  F t2 = fmul(p.Z, q.Z);
  F t3 = fmul(fadd(p.X, p.Y), fadd(q.X, q.Y));
  F t4 = fadd(t0, t1);
  t3 = fsub(t3, t4);
  t4 = fmul(fadd(p.Y, p.Z), fadd(q.Y, q.Z));
  F X3 = fadd(t1, t2);
  t4 = fsub(t4, X3);
  X3 = fmul(fadd(p.X, p.Z), fadd(q.X, q.Z));
  F Y3 = fadd(t0, t2);
  Y3 = fsub(X3, Y3);
  X3 = fadd(t0, t0);
  t0 = fadd(X3, t0);
  t2 = fmul_b3(t2);
  F Z3 = fadd(t1, t2);
  t1 = fsub(t1, t2);
  Y3 = fmul_b3(Y3);
  X3 = fmul(t4, Y3);
  t2 = fmul(t3, t1);
  X3 = fsub(t2, X3);
  Y3 = fmul(Y3, t0);
  t1 = fmul(t1, Z3);
  Y3 = fadd(t1, Y3);
  t0 = fmul(t0, t3);
  Z3 = fmul(Z3, t4);
  Z3 = fadd(Z3, t0);
  proj_t<F> r;
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
  return r;
}

// RCB 2016 algorithm 8 (mixed addition, q affine and finite, a = 0)
template <class F>
LSG_INL proj_t<F> proj_add_mixed(const proj_t<F>& p, const aff_t<F>& q) {
  F t0 = fmul(p.X, q.x);
  F t1 = fmul(p.Y, q.y);
  F t3 = fmul(fadd(q.x, q.y), fadd(p.X, p.Y));
  F t4 = fadd(t0, t1);
  t3 = fsub(t3, t4);
  t4 = fadd(fmul(q.y, p.Z), p.Y);
  F Y3 = fadd(fmul(q.x, p.Z), p.X);
  F X3 = fadd(t0, t0);
  t0 = fadd(X3, t0);
  F t2 = fmul_b3(p.Z);
  F Z3 = fadd(t1, t2);
  t1 = fsub(t1, t2);
  Y3 = fmul_b3(Y3);
  X3 = fmul(t4, Y3);
  t2 = fmul(t3, t1);
  X3 = fsub(t2, X3);
  Y3 = fmul(Y3, t0);
  t1 = fmul(t1, Z3);
  Y3 = fadd(t1, Y3);
  t0 = fmul(t0, t3);
  Z3 = fmul(Z3, t4);
  Z3 = fadd(Z3, t0);
  proj_t<F> r;
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
  return r;
}

// RCB 2016 algorithm 9 (doubling, a = 0)
template <class F>
LSG_INL proj_t<F> proj_dbl(const proj_t<F>& p) {
  F t0 = fsqr(p.Y);
  F Z3 = fadd(t0, t0);
  Z3 = fadd(Z3, Z3);
  Z3 = fadd(Z3, Z3);
  F t1 = fmul(p.Y, p.Z);
  F t2 = fmul_b3(fsqr(p.Z));
  F X3 = fmul(t2, Z3);
  F Y3 = fadd(t0, t2);
  Z3 = fmul(t1, Z3);
  t1 = fadd(t2, t2);
  t2 = fadd(t1, t2);
  t0 = fsub(t0, t2);
  Y3 = fmul(t0, Y3);
  Y3 = fadd(X3, Y3);
  t1 = fmul(p.X, p.Y);
  X3 = fmul(t0, t1);
  X3 = fadd(X3, X3);
  proj_t<F> r;
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
  return r;
}

// Non-inlined wrappers (keep call sites small: one G2 op expands to ~12 Fp2 muls)
LSG_BIGFN g1p_t g1_add(g1p_t p, g1p_t q) { return proj_add(p, q); }
LSG_BIGFN g1p_t g1_add_mixed(g1p_t p, g1a_t q) { return proj_add_mixed(p, q); }
LSG_BIGFN g1p_t g1_dbl(g1p_t p) { return proj_dbl(p); }
#ifdef LSG_ROW_SPLIT
// Row backend with the rows of a wave sharing one item (lsg_fp_lane.hpp): the same RCB
// formulas with their independent Fp2 products issued as batches (two rounds each), so the
// four rows split them.  Values are fully reduced there: the results are identical.
// Karatsuba operands of the Fp2 product a b at x/y[k..k+2], and its combination
LSG_INL void kar_prep(fp_t* x, fp_t* y, int k, const fp2_t& a, const fp2_t& b) {
  x[k] = a.c0;
  y[k] = b.c0;
  x[k + 1] = a.c1;
  y[k + 1] = b.c1;
  x[k + 2] = fp_add(a.c0, a.c1);
  y[k + 2] = fp_add(b.c0, b.c1);
}
LSG_INL fp2_t kar_fin(const fp_t* z, int k) {
  return fp2_t(fp_sub(z[k], z[k + 1]), fp_sub(fp_sub(z[k + 2], z[k]), z[k + 1]));
}
// RCB 2016 algorithm 7 (a = 0): round 1 the six cross products, round 2 the six outputs
LSG_INL g2p_t g2_add_rows(const g2p_t& p, const g2p_t& q) {
  fp_t x[18], y[18], z[18];
  kar_prep(x, y, 0, p.X, q.X);
  kar_prep(x, y, 3, p.Y, q.Y);
  kar_prep(x, y, 6, p.Z, q.Z);
  kar_prep(x, y, 9, fp2_add(p.X, p.Y), fp2_add(q.X, q.Y));
  kar_prep(x, y, 12, fp2_add(p.Y, p.Z), fp2_add(q.Y, q.Z));
  kar_prep(x, y, 15, fp2_add(p.X, p.Z), fp2_add(q.X, q.Z));
  fp_mul_list<18>(z, x, y);
  fp2_t t0 = kar_fin(z, 0), t1 = kar_fin(z, 3), t2 = kar_fin(z, 6);
  const fp2_t t3 = fp2_sub(kar_fin(z, 9), fp2_add(t0, t1));
  const fp2_t t4 = fp2_sub(kar_fin(z, 12), fp2_add(t1, t2));
  fp2_t Y3 = fp2_sub(kar_fin(z, 15), fp2_add(t0, t2));
  t0 = fp2_add(fp2_add(t0, t0), t0);
  t2 = fp2_mul_b3(t2);
  const fp2_t Z3 = fp2_add(t1, t2);
  t1 = fp2_sub(t1, t2);
  Y3 = fp2_mul_b3(Y3);
  kar_prep(x, y, 0, t4, Y3);
  kar_prep(x, y, 3, t3, t1);
  kar_prep(x, y, 6, Y3, t0);
  kar_prep(x, y, 9, t1, Z3);
  kar_prep(x, y, 12, t0, t3);
  kar_prep(x, y, 15, Z3, t4);
  fp_mul_list<18>(z, x, y);
  g2p_t r;
  r.X = fp2_sub(kar_fin(z, 3), kar_fin(z, 0));
  r.Y = fp2_add(kar_fin(z, 9), kar_fin(z, 6));
  r.Z = fp2_add(kar_fin(z, 15), kar_fin(z, 12));
  return r;
}
// RCB 2016 algorithm 9 (a = 0): round 1 Y^2, YZ, Z^2, XY; round 2 the four outputs
LSG_INL g2p_t g2_dbl_rows(const g2p_t& p) {
  fp_t x[12], y[12], z[12];
  kar_prep(x, y, 0, p.Y, p.Y);
  kar_prep(x, y, 3, p.Y, p.Z);
  kar_prep(x, y, 6, p.Z, p.Z);
  kar_prep(x, y, 9, p.X, p.Y);
  fp_mul_list<12>(z, x, y);
  const fp2_t t0 = kar_fin(z, 0), t1 = kar_fin(z, 3), t2 = fp2_mul_b3(kar_fin(z, 6)), xy = kar_fin(z, 9);
  const fp2_t z8 = fp2_dbl(fp2_dbl(fp2_dbl(t0)));
  const fp2_t y3 = fp2_add(t0, t2);
  const fp2_t s0 = fp2_sub(t0, fp2_add(fp2_add(t2, t2), t2));
  kar_prep(x, y, 0, t2, z8);
  kar_prep(x, y, 3, t1, z8);
  kar_prep(x, y, 6, s0, y3);
  kar_prep(x, y, 9, s0, xy);
  fp_mul_list<12>(z, x, y);
  g2p_t r;
  r.X = fp2_dbl(kar_fin(z, 9));
  r.Y = fp2_add(kar_fin(z, 0), kar_fin(z, 6));
  r.Z = kar_fin(z, 3);
  return r;
}
LSG_BIGFN g2p_t g2_add(g2p_t p, g2p_t q) { return g2_add_rows(p, q); }
LSG_BIGFN g2p_t g2_dbl(g2p_t p) { return g2_dbl_rows(p); }
#else
LSG_BIGFN g2p_t g2_add(g2p_t p, g2p_t q) { return proj_add(p, q); }
LSG_BIGFN g2p_t g2_dbl(g2p_t p) { return proj_dbl(p); }
#endif
LSG_BIGFN g2p_t g2_add_mixed(g2p_t p, g2a_t q) { return proj_add_mixed(p, q); }

LSG_INL g1p_t gadd(const g1p_t& p, const g1p_t& q) { return g1_add(p, q); }
LSG_INL g2p_t gadd(const g2p_t& p, const g2p_t& q) { return g2_add(p, q); }
LSG_INL g1p_t gdbl(const g1p_t& p) { return g1_dbl(p); }
LSG_INL g2p_t gdbl(const g2p_t& p) { return g2_dbl(p); }

// ---- Jacobian doubling chains.  A doubling in Jacobian coordinates (x = X/Z^2, y = Y/Z^3;
// dbl-2009-l, a = 0: 1M + 5S) costs 13 Fp multiplications over Fp2 against 22 for the
// complete RCB doubling, and it is exact for every input of these curves: the point at
// infinity (Z = 0) stays at infinity, and a finite point with Y = 0 would have order 2,
// which neither E1 nor E2 has (both group orders are odd).  Additions stay on the complete
// RCB formula (homogeneous coordinates), with conversions around them, so scalar products
// are exact for every input, including adversarial non-subgroup points.
template <class F>
struct jac_t {
  F X, Y, Z;
};

// homogeneous (X:Y:Z) -> Jacobian (XZ : YZ^2 : Z); infinity -> (1 : 1 : 0)
template <class F>
LSG_INL jac_t<F> jac_from_proj(const proj_t<F>& p) {
  F zz = fsqr(p.Z);
  jac_t<F> r;
  bool inf = fis_zero(p.Z);
  r.X = fselect(inf, fone<F>(), fmul(p.X, p.Z));
  r.Y = fselect(inf, fone<F>(), fmul(p.Y, zz));
  r.Z = p.Z;
  return r;
}

// Jacobian -> homogeneous (XZ : Y : Z^3); infinity -> (0 : 1 : 0)
template <class F>
LSG_INL proj_t<F> jac_to_proj(const jac_t<F>& p) {
  F zz = fsqr(p.Z);
  proj_t<F> r;
  bool inf = fis_zero(p.Z);
  r.X = fmul(p.X, p.Z);
  r.Y = fselect(inf, fone<F>(), p.Y);
  r.Z = fmul(zz, p.Z);
  return r;
}

template <class F>
LSG_INL jac_t<F> jac_dbl_t(const jac_t<F>& p) {
  F A = fsqr(p.X);
  F B = fsqr(p.Y);
  F C = fsqr(B);
  F D = fsub(fsqr(fadd(p.X, B)), fadd(A, C));
  D = fadd(D, D);
  F E = fadd(fadd(A, A), A);
  F Fq = fsqr(E);
  jac_t<F> r;
  r.X = fsub(Fq, fadd(D, D));
  F C8 = fadd(C, C);
  C8 = fadd(C8, C8);
  C8 = fadd(C8, C8);
  r.Y = fsub(fmul(E, fsub(D, r.X)), C8);
  F yz = fmul(p.Y, p.Z);
  r.Z = fadd(yz, yz);
  return r;
}
LSG_BIGFN jac_t<fp_t> jac_dbl(jac_t<fp_t> p) { return jac_dbl_t(p); }
LSG_BIGFN jac_t<fp2_t> jac_dbl(jac_t<fp2_t> p) { return jac_dbl_t(p); }

// acc (Jacobian) + q (homogeneous) through the complete RCB addition
template <class F>
LSG_INL jac_t<F> jac_add_proj(const jac_t<F>& acc, const proj_t<F>& q) {
  return jac_from_proj(gadd(jac_to_proj(acc), q));
}

// [k]P for a 64-bit scalar k (per lane), 4-bit fixed windows: 60 Jacobian doublings and 16
// complete additions of a table entry T[d] = [d]P (T[0] = O), selected per row.
template <class F>
LSG_INL proj_t<F> proj_mul_u64(const proj_t<F>& p, uint64_t k) {
  proj_t<F> T[16];
  T[0] = proj_inf<F>();
  T[1] = p;
  T[2] = gdbl(p);
#pragma unroll 1
  for (int d = 3; d < 16; d++) T[d] = gadd(T[d - 1], p);
  // the digit is uniform over the lanes of one element: a per-lane indexed read of the table
  auto pick = [&](uint32_t d) { return T[d]; };
  jac_t<F> acc = jac_from_proj(pick((uint32_t)(k >> 60) & 15u));
#pragma unroll 1
  for (int w = 14; w >= 0; w--) {
    acc = jac_dbl(acc);
    acc = jac_dbl(acc);
    acc = jac_dbl(acc);
    acc = jac_dbl(acc);
    acc = jac_add_proj(acc, pick((uint32_t)(k >> (4 * w)) & 15u));
  }
  return jac_to_proj(acc);
}

// [k]P for a 64-bit scalar k, signed 3-bit windows: k = sum_{i<22} d_i 8^i with d_i in
// [-4, 3] (d_21 in [0, 2]), table T[1..4] = [1..4]P held in registers and picked with selects
// (a per-lane indexed table lives in scratch).  63 Jacobian doublings and 21 complete
// additions, plus 2 doublings and 1 addition for the table (the 4-bit form: 61 + 29).
template <class F>
LSG_INL proj_t<F> proj_pick_signed(const proj_t<F>& T1, const proj_t<F>& T2, const proj_t<F>& T3,
                                   const proj_t<F>& T4, int d) {
  const int a = d < 0 ? -d : d;
  proj_t<F> r = proj_inf<F>();
  auto take = [&](bool s, const proj_t<F>& t) {
    r.X = fselect(s, t.X, r.X);
    r.Y = fselect(s, t.Y, r.Y);
    r.Z = fselect(s, t.Z, r.Z);
  };
  take(a == 1, T1);
  take(a == 2, T2);
  take(a == 3, T3);
  take(a == 4, T4);
  r.Y = fselect(d < 0, fneg(r.Y), r.Y);
  return r;
}
template <class F>
LSG_INL proj_t<F> proj_mul_u64_s3(const proj_t<F>& p, uint64_t k) {
  const proj_t<F> T2 = gdbl(p);
  const proj_t<F> T3 = gadd(T2, p);
  const proj_t<F> T4 = gdbl(T2);
  // carry into window i (bit i): windows of value >= 4 borrow 8 from the next one
  uint32_t cm = 0;
#pragma unroll
  for (int i = 0; i < 21; i++) {
    const uint32_t v = (uint32_t)((k >> (3 * i)) & 7u) + ((cm >> i) & 1u);
    cm |= (v >= 4u ? 1u : 0u) << (i + 1);
  }
  auto digit = [&](int i) {
    return (int)((k >> (3 * i)) & 7u) + (int)((cm >> i) & 1u) - (i < 21 ? 8 * (int)((cm >> (i + 1)) & 1u) : 0);
  };
  jac_t<F> acc = jac_from_proj(proj_pick_signed(p, T2, T3, T4, digit(21)));
#pragma unroll 1
  for (int i = 20; i >= 0; i--) {
    acc = jac_dbl(acc);
    acc = jac_dbl(acc);
    acc = jac_dbl(acc);
    acc = jac_add_proj(acc, proj_pick_signed(p, T2, T3, T4, digit(i)));
  }
  return jac_to_proj(acc);
}

// [|x|]P for the BLS parameter |x| = 0xd201000000010000 (public, uniform branch):
// 63 Jacobian doublings, 5 complete additions
// The base point comes from get() at each addition: a per-set kernel keeps it in LDS
// (lsg_kcommon.hpp lds_park) so that the doubling chain holds one point in registers.
template <class F, class G>
LSG_INL proj_t<F> proj_mul_xabs_get(const G& get) {
  const uint64_t xa = ((uint64_t)LSG_X_ABS_HI << 32) | LSG_X_ABS_LO;
  jac_t<F> acc = jac_from_proj(get());
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    acc = jac_dbl(acc);
    if ((xa >> b) & 1u) acc = jac_add_proj(acc, get());
  }
  return jac_to_proj(acc);
}
template <class F>
LSG_INL proj_t<F> proj_mul_xabs(const proj_t<F>& p) {
  return proj_mul_xabs_get<F>([&]() { return p; });
}

template <class F>
LSG_INL bool proj_eq(const proj_t<F>& a, const proj_t<F>& b) {
  bool ia = proj_is_inf(a), ib = proj_is_inf(b);
  if (ia || ib) return ia && ib;
  return feq(fmul(a.X, b.Z), fmul(b.X, a.Z)) && feq(fmul(a.Y, b.Z), fmul(b.Y, a.Z));
}

template <class F>
LSG_INL aff_t<F> proj_to_aff(const proj_t<F>& p) {
  F zi = finv(p.Z);
  aff_t<F> r;
  r.x = fmul(p.X, zi);
  r.y = fmul(p.Y, zi);
  return r;
}

// ---- psi endomorphism of E2 (untwist-Frobenius-twist), valid on projective points
LSG_INL g2p_t g2_psi(const g2p_t& p) {
  g2p_t r;
  r.X = fp2_mul(fp2_conj(p.X), PSI_CX);
  r.Y = fp2_mul(fp2_conj(p.Y), PSI_CY);
  r.Z = fp2_conj(p.Z);
  return r;
}
LSG_INL g2p_t g2_psi2(const g2p_t& p) {
  g2p_t r;
  r.X = fp2_mul_fp(p.X, PSI2_CX);
  r.Y = fp2_mul_fp(p.Y, PSI2_CY);
  r.Z = p.Z;
  return r;
}

// Scott's G2 membership test: psi(P) == [x]P (x < 0)
template <class G>
LSG_INL bool g2_in_group_get(const G& get) {
  if (proj_is_inf(get())) return true;
  g2p_t xp = proj_neg(proj_mul_xabs_get<fp2_t>(get));
  return proj_eq(g2_psi(get()), xp);
}
LSG_BIGFN bool g2_in_group(g2p_t p) {
  return g2_in_group_get([&]() { return p; });
}

// G1 membership by definition, [r]P == O: double-and-add over the 255-bit group order
// (KeyValidate of batched pubkey validation; not on the verify path, where keys are trusted)
LSG_BIGFN bool g1_in_group(g1p_t p) {
  const uint32_t rw[8] = {0x73eda753u, 0x299d7d48u, 0x3339d808u, 0x09a1d805u,
                          0x53bda402u, 0xfffe5bfeu, 0xffffffffu, 0x00000001u};
  g1p_t acc = proj_inf<fp_t>();
#pragma unroll 1
  for (int w = 0; w < 8; w++) {
#pragma unroll 1
    for (int b = 31; b >= 0; b--) {
      acc = g1_dbl(acc);
      if ((rw[w] >> b) & 1u) acc = g1_add(acc, p);
    }
  }
  return proj_is_inf(acc);
}

LSG_INL bool g1_on_curve_aff(const g1a_t& a) {
  fp_t rhs = fp_add(fp_mul(fp_sqr(a.x), a.x), FP_B_G1);
  return fp_eq(fp_sqr(a.y), rhs);
}
LSG_INL bool g2_on_curve_aff(const g2a_t& a) {
  fp2_t rhs = fp2_add(fp2_mul(fp2_sqr(a.x), a.x), FP2_B_G2);
  return fp2_eq(fp2_sqr(a.y), rhs);
}

// Status codes, numerically equal to blst's BLST_ERROR (+ wrapper's size error); the
// same values as include/lodestar_bls.h.
#ifndef LSG_BLST_SUCCESS
#define LSG_BLST_SUCCESS 0
#define LSG_BLST_BAD_ENCODING 1
#define LSG_BLST_POINT_NOT_ON_CURVE 2
#define LSG_BLST_POINT_NOT_IN_GROUP 3
#define LSG_BLST_AGGR_TYPE_MISMATCH 4
#define LSG_BLST_VERIFY_FAIL 5
#define LSG_BLST_PK_IS_INFINITY 6
#define LSG_BLST_BAD_SCALAR 7
#define LSG_BLST_INVALID_SIZE 10
#endif

// blst POINTonE2_Uncompress_Z (96 bytes).  Sets *inf for the infinity encoding.
LSG_INL int g2_uncompress(g2a_t& out, bool& inf, const uint8_t* in) {
  uint8_t in0 = in[0];
  inf = false;
  if (!(in0 & 0x80)) return LSG_BLST_BAD_ENCODING;
  if (in0 & 0x40) {
    uint32_t acc = in0 & 0x3f;
    for (int i = 1; i < 96; i++) acc |= in[i];
    if (acc == 0) {
      inf = true;
      out.x = fp2_zero();
      out.y = fp2_zero();
      return LSG_BLST_SUCCESS;
    }
    return LSG_BLST_BAD_ENCODING;
  }
  fp_t x1 = fp_from_be48(in);
  x1 = fp_mask_flags(x1);
  fp_t x0 = fp_from_be48(in + 48);
  if (!fp_canon_lt_p(x1) || !fp_canon_lt_p(x0)) return LSG_BLST_BAD_ENCODING;
  fp2_t x = fp2_make(fp_to_mont(x0), fp_to_mont(x1));
  fp2_t rhs = fp2_add(fp2_mul(fp2_sqr(x), x), FP2_B_G2);
  fp2_t y;
  if (!fp2_sqrt(y, rhs)) return LSG_BLST_POINT_NOT_ON_CURVE;
  bool want = (in0 & 0x20) != 0;
  if (fp2_lexi_largest(y) != want) y = fp2_neg(y);
  out.x = x;
  out.y = y;
  if (fp2_is_zero(x)) return LSG_BLST_POINT_NOT_IN_GROUP;
  return LSG_BLST_SUCCESS;
}

// blst POINTonE2_Deserialize_Z for 192-byte uncompressed input
LSG_INL int g2_deserialize_uncompressed(g2a_t& out, bool& inf, const uint8_t* in) {
  uint8_t in0 = in[0];
  inf = false;
  if (in0 & 0x80) return LSG_BLST_BAD_ENCODING;
  if (in0 & 0x40) {
    uint32_t acc = in0 & 0x3f;
    for (int i = 1; i < 192; i++) acc |= in[i];
    if (acc == 0) {
      inf = true;
      out.x = fp2_zero();
      out.y = fp2_zero();
      return LSG_BLST_SUCCESS;
    }
    return LSG_BLST_BAD_ENCODING;
  }
  if (in0 & 0x20) return LSG_BLST_BAD_ENCODING;
  fp_t v[4];
  for (int k = 0; k < 4; k++) {
    v[k] = fp_from_be48(in + 48 * k);
    if (k == 0) v[k] = fp_mask_flags(v[k]);
    if (!fp_canon_lt_p(v[k])) return LSG_BLST_BAD_ENCODING;
  }
  out.x = fp2_make(fp_to_mont(v[1]), fp_to_mont(v[0]));
  out.y = fp2_make(fp_to_mont(v[3]), fp_to_mont(v[2]));
  if (!g2_on_curve_aff(out)) return LSG_BLST_POINT_NOT_ON_CURVE;
  if (fp2_is_zero(out.x)) return LSG_BLST_POINT_NOT_IN_GROUP;
  return LSG_BLST_SUCCESS;
}

// blst_p1_deserialize: 96-byte uncompressed or 48-byte compressed
LSG_INL int g1_deserialize(g1a_t& out, bool& inf, const uint8_t* in, int len) {
  uint8_t in0 = in[0];
  inf = false;
  bool compressed = (in0 & 0x80) != 0;
  if (compressed != (len == 48)) return LSG_BLST_BAD_ENCODING;
  if (in0 & 0x40) {
    uint32_t acc = in0 & 0x3f;
    for (int i = 1; i < len; i++) acc |= in[i];
    if (acc == 0) {
      inf = true;
      out.x = fp_zero();
      out.y = fp_zero();
      return LSG_BLST_SUCCESS;
    }
    return LSG_BLST_BAD_ENCODING;
  }
  if (!compressed && (in0 & 0x20)) return LSG_BLST_BAD_ENCODING;
  fp_t x = fp_from_be48(in);
  x = fp_mask_flags(x);
  if (!fp_canon_lt_p(x)) return LSG_BLST_BAD_ENCODING;
  out.x = fp_to_mont(x);
  if (compressed) {
    fp_t rhs = fp_add(fp_mul(fp_sqr(out.x), out.x), FP_B_G1);
    fp_t y = fp_pow_id(rhs, LSG_POW_SQRT);
    if (!fp_eq(fp_sqr(y), rhs)) return LSG_BLST_POINT_NOT_ON_CURVE;
    bool want = (in0 & 0x20) != 0;
    if (fp_canon_gt_half(fp_from_mont(y)) != want) y = fp_neg(y);
    out.y = y;
  } else {
    fp_t y = fp_from_be48(in + 48);
    if (!fp_canon_lt_p(y)) return LSG_BLST_BAD_ENCODING;
    out.y = fp_to_mont(y);
    if (!g1_on_curve_aff(out)) return LSG_BLST_POINT_NOT_ON_CURVE;
  }
  if (fp_is_zero(out.x)) return LSG_BLST_POINT_NOT_IN_GROUP;
  return LSG_BLST_SUCCESS;
}

// affine G1 -> 96-byte uncompressed (blst_p1_affine_serialize)
LSG_INL void g1_serialize(uint8_t* out, const g1a_t& a, bool inf) {
  if (inf) {
    out[0] = 0x40;
    for (int i = 1; i < 96; i++) out[i] = 0;
    return;
  }
  fp_to_be48(out, fp_from_mont(a.x));
  fp_to_be48(out + 48, fp_from_mont(a.y));
}

// affine G2 -> 192-byte uncompressed
LSG_INL void g2_serialize(uint8_t* out, const g2a_t& a, bool inf) {
  if (inf) {
    out[0] = 0x40;
    for (int i = 1; i < 192; i++) out[i] = 0;
    return;
  }
  fp_to_be48(out, fp_from_mont(a.x.c1));
  fp_to_be48(out + 48, fp_from_mont(a.x.c0));
  fp_to_be48(out + 96, fp_from_mont(a.y.c1));
  fp_to_be48(out + 144, fp_from_mont(a.y.c0));
}

// affine G2 -> 96-byte ZCash-compressed (blst_p2_affine_compress)
LSG_INL void g2_compress(uint8_t* out, const g2a_t& a, bool inf) {
  if (inf) {
    out[0] = 0xc0;
    for (int i = 1; i < 96; i++) out[i] = 0;
    return;
  }
  uint32_t flags = 0x80u | (fp2_lexi_largest(a.y) ? 0x20u : 0u);
  fp_to_be48(out, fp_or_flags(fp_from_mont(a.x.c1), flags));
  fp_to_be48(out + 48, fp_from_mont(a.x.c0));
}
