// TEST INFRASTRUCTURE ONLY -- host (x86) build of the kernel math headers.
//
// Compiles lodestar_amd/csrc/lsg_*.hpp (all functions are __host__ __device__) for the
// CPU so tests/test_hostcheck_math.py can compare every stage of the device arithmetic
// with the oracle inside the build container, where no GPU exists.  It is never linked
// into, loaded by or reachable from the product library (lodestar_amd/liblodestar_bls.so);
// the product path runs only on the GPU.
#include <hip/hip_runtime.h>
#include <string.h>

#define LSG_COUNT_MULS 1
#ifdef LSG_HOSTCHECK_PAIR
// the pair backend's arithmetic (lazy signed radix-2^29 limbs) with all 14 limbs in one
// "lane": same representation, bounds and byte conversions as the gfx950 build
#define LSG_PAIR_G 1
#include "lsg_fp_pair.hpp"
#else
#include "lsg_fp_elem.hpp"
#endif
#include "lsg_h2c.hpp"
#include "lsg_pairing.hpp"

static fp_t rd(const uint8_t* b) { return fp_to_mont(fp_from_be48(b)); }
static void wr(uint8_t* b, const fp_t& a) { fp_to_be48(b, fp_from_mont(a)); }
static fp2_t rd2(const uint8_t* b) { return fp2_make(rd(b), rd(b + 48)); }  // (c0, c1)
static void wr2(uint8_t* b, const fp2_t& a) {
  wr(b, a.c0);
  wr(b + 48, a.c1);
}
static void wr12(uint8_t* b, const fp12_t& f) {
  const fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; i++) wr2(b + 96 * i, *c[i]);
}
static fp12_t rd12(const uint8_t* b) {
  fp12_t f;
  fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; i++) *c[i] = rd2(b + 96 * i);
  return f;
}

unsigned long long lsg_mul_count = 0;

extern "C" {

void hc_fp_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { wr(out, fp_mul(rd(a), rd(b))); }
void hc_fp_inv(const uint8_t* a, uint8_t* out) { wr(out, fp_inv(rd(a))); }
void hc_fp_from_be64(const uint8_t* a, uint8_t* out) { wr(out, fp_from_be64_mod(a)); }
void hc_fp2_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { wr2(out, fp2_mul(rd2(a), rd2(b))); }
void hc_fp2_sqr(const uint8_t* a, uint8_t* out) { wr2(out, fp2_sqr(rd2(a))); }
void hc_fp2_inv(const uint8_t* a, uint8_t* out) { wr2(out, fp2_inv(rd2(a))); }
int hc_fp2_sqrt(const uint8_t* a, uint8_t* out) {
  fp2_t r;
  bool ok = fp2_sqrt(r, rd2(a));
  wr2(out, r);
  return ok;
}
void hc_fp12_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { wr12(out, fp12_mul(rd12(a), rd12(b))); }
void hc_fp12_sqr(const uint8_t* a, uint8_t* out) { wr12(out, fp12_sqr(rd12(a))); }
void hc_fp12_inv(const uint8_t* a, uint8_t* out) { wr12(out, fp12_inv(rd12(a))); }
void hc_fp12_frob(const uint8_t* a, uint8_t* out) { wr12(out, fp12_frob(rd12(a))); }
void hc_fp12_frob2(const uint8_t* a, uint8_t* out) { wr12(out, fp12_frob2(rd12(a))); }
void hc_final_exp(const uint8_t* a, uint8_t* out) { wr12(out, final_exp(rd12(a))); }

int hc_g2_uncompress(const uint8_t* in, uint8_t* out192) {
  g2a_t p;
  bool inf;
  int e = g2_uncompress(p, inf, in);
  if (e == 0) g2_serialize(out192, p, inf);
  return e;
}
int hc_g2_in_group(const uint8_t* in192) {
  g2a_t p;
  bool inf;
  int e = g2_deserialize_uncompressed(p, inf, in192);
  if (e != 0 && e != LSG_BLST_POINT_NOT_IN_GROUP) return -e;
  if (inf) return 1;
  return g2_in_group(proj_from_aff(p)) ? 1 : 0;
}
int hc_g1_deserialize(const uint8_t* in, int len, uint8_t* out96) {
  g1a_t p;
  bool inf;
  int e = g1_deserialize(p, inf, in, len);
  if (e == 0) g1_serialize(out96, p, inf);
  return e;
}
void hc_expand_xmd(const uint8_t* msg, int mlen, const uint8_t* dst, int dlen, uint8_t* out256) {
  expand_message_xmd_256(out256, msg, mlen, dst, dlen);
}
void hc_sswu(const uint8_t* u96, uint8_t* out192) {
  g2a_t p = map_to_curve_sswu(rd2(u96));
  g2_serialize(out192, p, false);
}
void hc_hash_to_g2(const uint8_t* msg, int mlen, const uint8_t* dst, int dlen, uint8_t* out192) {
  uint8_t ub[256];
  expand_message_xmd_256(ub, msg, mlen, dst, dlen);
  fp2_t u0 = fp2_make(fp_from_be64_mod(ub), fp_from_be64_mod(ub + 64));
  fp2_t u1 = fp2_make(fp_from_be64_mod(ub + 128), fp_from_be64_mod(ub + 192));
  g2p_t q0 = iso_map3(map_to_curve_sswu(u0));
  g2p_t q1 = iso_map3(map_to_curve_sswu(u1));
  g2p_t r = clear_cofactor_g2(g2_add(q0, q1));
  bool inf = proj_is_inf(r);
  g2a_t a = inf ? g2a_t{fp2_zero(), fp2_zero()} : proj_to_aff(r);
  g2_serialize(out192, a, inf);
}
void hc_g1_mul_u64(const uint8_t* in96, uint64_t k, uint8_t* out96) {
  g1a_t p;
  bool inf;
  g1_deserialize(p, inf, in96, 96);
  g1p_t r = proj_mul_u64_s3(proj_from_aff(p), k);
  bool rinf = proj_is_inf(r);
  g1a_t a = rinf ? g1a_t{fp_zero(), fp_zero()} : proj_to_aff(r);
  g1_serialize(out96, a, rinf);
}
void hc_g2_mul_u64(const uint8_t* in192, uint64_t k, uint8_t* out192) {
  g2a_t p;
  bool inf;
  g2_deserialize_uncompressed(p, inf, in192);
  g2p_t r = proj_mul_u64(proj_from_aff(p), k);
  bool rinf = proj_is_inf(r);
  g2a_t a = rinf ? g2a_t{fp2_zero(), fp2_zero()} : proj_to_aff(r);
  g2_serialize(out192, a, rinf);
}
void hc_miller(const uint8_t* p96, const uint8_t* q192, uint8_t* out576) {
  g1a_t p;
  g2a_t q;
  bool inf;
  g1_deserialize(p, inf, p96, 96);
  g2_deserialize_uncompressed(q, inf, q192);
  wr12(out576, miller_loop(p, q));
}

// Fp-multiplication counts of each device stage for one representative set (bench/opcount.json).
// counts[]: sig_decode, sig_subgroup, pk_decode, pk_scale, hash_map, sig_scale, miller,
//           g2_add, fp12_mul, final_exp, g1_add
// multi-Miller loop over 4 pairs (use[k] = 0 drops pair k) -- lsg_pairing.hpp:miller_loop_multi
void hc_miller_multi4(const uint8_t* p96x4, const uint8_t* q192x4, const int32_t* use4, uint8_t* out576) {
  g1a_t P[4];
  g2a_t Q[4];
  bool use[4];
  for (int k = 0; k < 4; k++) {
    bool inf;
    g1_deserialize(P[k], inf, p96x4 + 96 * k, 96);
    g2_deserialize_uncompressed(Q[k], inf, q192x4 + 192 * k);
    use[k] = use4[k] != 0;
  }
  wr12(out576, miller_loop_multi<4>(P, Q, use));
}

// the split multi-Miller loop over 4 pairs: miller_lines per Q, then miller_accum_multi
// (lsg_pairing.hpp; the device kernels k_miller_lines / k_miller_accum)
void hc_miller_split4(const uint8_t* p96x4, const uint8_t* q192x4, const int32_t* use4, uint8_t* out576) {
  g1a_t P[4];
  bool use[4];
  static line_t lines[4][ML_STEPS];
  for (int k = 0; k < 4; k++) {
    bool inf;
    g2a_t Q;
    g1_deserialize(P[k], inf, p96x4 + 96 * k, 96);
    g2_deserialize_uncompressed(Q, inf, q192x4 + 192 * k);
    use[k] = use4[k] != 0;
    int cnt = 0;
    miller_lines(Q, [&](int st, const line_t& L) {
      lines[k][st] = L;
      cnt++;
    });
    if (cnt != ML_STEPS) abort();
  }
  wr12(out576, miller_accum_multi<4>(P, use, [&](int k, int st) { return lines[k][st]; }));
}

// The fused kernel's schedule (lsg_k_miller.hip k_miller_fused) restated on the host with
// the same formulas: per step the four lines, multiplied in pairs (P phase), then f^2 on
// doublings after the first two steps (S phase) and f * M01 * M23 (M phase).
struct pair_m_t {
  fp2_t m0, m1, m2, m4, m5;  // (m0 + m1 v + m2 v^2) + (m4 v + m5 v^2) w
};
static pair_m_t hc_pair_lines(const line_t& a, const line_t& b) {
  const fp2_t P0 = fp2_mul(a.l00, b.l00), P1 = fp2_mul(a.l11, b.l11), P2 = fp2_mul(a.l01, b.l01);
  const fp2_t P3 = fp2_mul(fp2_add(a.l00, a.l01), fp2_add(b.l00, b.l01));
  const fp2_t P4 = fp2_mul(fp2_add(a.l00, a.l11), fp2_add(b.l00, b.l11));
  const fp2_t P5 = fp2_mul(fp2_add(a.l01, a.l11), fp2_add(b.l01, b.l11));
  pair_m_t m;
  m.m0 = fp2_add(P0, fp2_mul_xi(P1));
  m.m1 = fp2_sub(fp2_sub(P3, P0), P2);
  m.m2 = P2;
  m.m4 = fp2_sub(fp2_sub(P4, P0), P1);
  m.m5 = fp2_sub(fp2_sub(P5, P2), P1);
  return m;
}
static fp12_t hc_mul_pair(const fp12_t& f, const pair_m_t& M) {
  const fp6_t& a = f.c0;
  const fp6_t& b = f.c1;
  const fp2_t V0 = fp2_mul(a.c0, M.m0), V1 = fp2_mul(a.c1, M.m1), V2 = fp2_mul(a.c2, M.m2);
  const fp2_t V3 = fp2_mul(fp2_add(a.c0, a.c1), fp2_add(M.m0, M.m1));
  const fp2_t V4 = fp2_mul(fp2_add(a.c1, a.c2), fp2_add(M.m1, M.m2));
  const fp2_t V5 = fp2_mul(fp2_add(a.c0, a.c2), fp2_add(M.m0, M.m2));
  const fp2_t V6 = fp2_mul(b.c0, M.m4), V7 = fp2_mul(b.c1, M.m5), V8 = fp2_mul(fp2_add(b.c0, b.c1), fp2_add(M.m4, M.m5));
  const fp2_t V9 = fp2_mul(b.c2, M.m4), V10 = fp2_mul(b.c2, M.m5);
  const fp6_t sv = fp6_add(a, b);
  const fp2_t q0 = M.m0, q1 = fp2_add(M.m1, M.m4), q2 = fp2_add(M.m2, M.m5);
  const fp2_t V11 = fp2_mul(sv.c0, q0), V12 = fp2_mul(sv.c1, q1), V13 = fp2_mul(sv.c2, q2);
  const fp2_t V14 = fp2_mul(fp2_add(sv.c0, sv.c1), fp2_add(q0, q1));
  const fp2_t V15 = fp2_mul(fp2_add(sv.c1, sv.c2), fp2_add(q1, q2));
  const fp2_t V16 = fp2_mul(fp2_add(sv.c0, sv.c2), fp2_add(q0, q2));
  const fp2_t t0[3] = {fp2_add(V0, fp2_mul_xi(fp2_sub(fp2_sub(V4, V1), V2))),
                       fp2_add(fp2_sub(fp2_sub(V3, V0), V1), fp2_mul_xi(V2)), fp2_add(fp2_sub(fp2_sub(V5, V0), V2), V1)};
  const fp2_t t2[3] = {fp2_add(V11, fp2_mul_xi(fp2_sub(fp2_sub(V15, V12), V13))),
                       fp2_add(fp2_sub(fp2_sub(V14, V11), V12), fp2_mul_xi(V13)),
                       fp2_add(fp2_sub(fp2_sub(V16, V11), V13), V12)};
  const fp2_t n[3] = {fp2_add(V6, fp2_mul_xi(V10)), fp2_sub(fp2_sub(V8, V6), V7), fp2_add(V7, V9)};
  fp12_t r;
  r.c0 = fp6_make(fp2_add(t0[0], fp2_mul_xi(n[1])), fp2_add(t0[1], fp2_mul_xi(n[2])), fp2_add(t0[2], n[0]));
  r.c1 = fp6_make(fp2_sub(fp2_sub(t2[0], t0[0]), fp2_mul_xi(n[2])), fp2_sub(fp2_sub(t2[1], t0[1]), n[0]),
                  fp2_sub(fp2_sub(t2[2], t0[2]), n[1]));
  return r;
}
void hc_miller_paired4(const uint8_t* p96x4, const uint8_t* q192x4, const int32_t* use4, uint8_t* out576) {
  g1a_t P[4];
  g2a_t Q[4];
  g2p_t T[4];
  bool use[4];
  for (int k = 0; k < 4; k++) {
    bool inf;
    g1_deserialize(P[k], inf, p96x4 + 96 * k, 96);
    g2_deserialize_uncompressed(Q[k], inf, q192x4 + 192 * k);
    use[k] = use4[k] != 0;
    T[k] = proj_from_aff(Q[k]);
  }
  fp12_t f = fp12_one();
  auto step = [&](bool add, bool sqr) {
    line_t L[4];
    for (int k = 0; k < 4; k++) {
      line_t l = line_eval(add ? ml_add_step_raw(T[k], Q[k]) : ml_dbl_step_raw(T[k]), P[k].x, P[k].y);
      L[k] = use[k] ? l : line_t{fp2_one(), fp2_zero(), fp2_zero()};
    }
    const pair_m_t M01 = hc_pair_lines(L[0], L[1]), M23 = hc_pair_lines(L[2], L[3]);
    if (sqr) f = fp12_sqr(f);
    f = hc_mul_pair(hc_mul_pair(f, M01), M23);
  };
  const uint64_t xa = ((uint64_t)LSG_X_ABS_HI << 32) | LSG_X_ABS_LO;
  step(false, false);
  step(true, false);
  for (int b = 61; b >= 0; b--) {
    step(false, true);
    if ((xa >> b) & 1u) step(true, false);
  }
  wr12(out576, fp12_conj(f));
}

// KeyValidate's subgroup test (lsg_curve.hpp:g1_in_group) on a 96-byte uncompressed point
int hc_g1_in_group(const uint8_t* p96) {
  g1a_t a;
  bool inf;
  if (g1_deserialize(a, inf, p96, 96) != 0) return -1;
  return g1_in_group(inf ? proj_inf<fp_t>() : proj_from_aff(a)) ? 1 : 0;
}

void hc_opcount(const uint8_t* sig96, const uint8_t* pk96, const uint8_t* msg32, uint64_t r, unsigned long long* counts) {
  g2a_t s;
  g1a_t pk;
  bool inf;
  lsg_mul_count = 0;
  g2_uncompress(s, inf, sig96);
  counts[0] = lsg_mul_count;
  lsg_mul_count = 0;
  (void)g2_in_group(proj_from_aff(s));
  counts[1] = lsg_mul_count;
  lsg_mul_count = 0;
  g1_deserialize(pk, inf, pk96, 96);
  counts[2] = lsg_mul_count;
  g1a_t P = proj_to_aff(proj_mul_u64_s3(proj_from_aff(pk), r));  // value (inversion not counted:)
  lsg_mul_count = 0;
  {  // device: projective [r]PK, 1/Z from the batched inversion (3 M per element), 2 M to affine
    g1p_t Pp = proj_mul_u64_s3(proj_from_aff(pk), r);
    fp_t zi = fp_one();
    (void)fp_mul(Pp.X, zi);
    (void)fp_mul(Pp.Y, zi);
  }
  counts[3] = lsg_mul_count + 3;
  uint8_t ub[256];
  expand_message_xmd_256(ub, msg32, 32, (const uint8_t*)"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_", 43);
  fp2_t u0 = fp2_make(fp_from_be64_mod(ub), fp_from_be64_mod(ub + 64));
  fp2_t u1 = fp2_make(fp_from_be64_mod(ub + 128), fp_from_be64_mod(ub + 192));
  g2a_t H = proj_to_aff(clear_cofactor_g2(g2_add(iso_map3(map_to_curve_sswu(u0)), iso_map3(map_to_curve_sswu(u1)))));
  lsg_mul_count = 0;
  {  // device stages k_h2c_prep / k_h2c_map / k_h2c_affine; the three inversions per set are
     // batched (3 M per inverted element)
    fp2_t v0 = fp2_make(fp_from_be64_mod(ub), fp_from_be64_mod(ub + 64));
    fp2_t v1 = fp2_make(fp_from_be64_mod(ub + 128), fp_from_be64_mod(ub + 192));
    fp_t n0 = fp2_norm(sswu_tv1(v0)), n1 = fp2_norm(sswu_tv1(v1));
    g2p_t q = clear_cofactor_g2(g2_add(iso_map3(map_to_curve_sswu_ni(v0, n0)), iso_map3(map_to_curve_sswu_ni(v1, n1))));
    fp_t zn = fp2_norm(q.Z);
    fp2_t zi = fp2_inv_with_norm_inv(q.Z, zn);
    (void)fp2_mul(q.X, zi);
    (void)fp2_mul(q.Y, zi);
  }
  counts[4] = lsg_mul_count + 9;
  lsg_mul_count = 0;
  g2p_t rs = proj_mul_u64(proj_from_aff(s), r);
  counts[5] = lsg_mul_count;
  lsg_mul_count = 0;
  fp12_t f = miller_loop(P, H);
  counts[6] = lsg_mul_count;
  {  // the device runs the multi-Miller loop with K = 2 pairs per item: cost per set
    g1a_t P2[2] = {P, P};
    g2a_t H2[2] = {H, H};
    bool use2[2] = {true, true};
    lsg_mul_count = 0;
    (void)miller_loop_multi<2>(P2, H2, use2);
    counts[11] = lsg_mul_count / 2;
  }
  {  // split device path: line schedule per set, then the accumulation over K = 2 pairs
    line_t lines[ML_STEPS];
    lsg_mul_count = 0;
    miller_lines(H, [&](int st, const line_t& L) { lines[st] = L; });
    counts[12] = lsg_mul_count;
    g1a_t P2[2] = {P, P};
    bool use2[2] = {true, true};
    lsg_mul_count = 0;
    (void)miller_accum_multi<2>(P2, use2, [&](int, int st) { return lines[st]; });
    counts[13] = lsg_mul_count / 2;
    g1a_t P4[4] = {P, P, P, P};
    bool use4[4] = {true, true, true, true};
    lsg_mul_count = 0;
    (void)miller_accum_multi<4>(P4, use4, [&](int, int st) { return lines[st]; });
    counts[14] = lsg_mul_count / 4;  // K = 4 pairs per item (the default, LSG_MILLER_K)
  }
  lsg_mul_count = 0;
  (void)g2_add(rs, rs);
  counts[7] = lsg_mul_count;
  lsg_mul_count = 0;
  (void)fp12_mul(f, f);
  counts[8] = lsg_mul_count;
  lsg_mul_count = 0;
  (void)final_exp(f);
  counts[9] = lsg_mul_count;
  lsg_mul_count = 0;
  (void)g1_add(proj_from_aff(pk), proj_from_aff(pk));
  counts[10] = lsg_mul_count;
}
}

#ifdef LSG_HOSTCHECK_PAIR
// ---- the straight-line programs of the serial stages (tools/gen_slp.py), executed op by op
// with the gfx950 interpreter's own operation code (lsg_slp_exec.hpp) on the host
#include <vector>
#include "lsg_slp_exec.hpp"
#include "lsg_slp_progs.h"
struct HcProg {
  const uint32_t *ops, *steps, *consts;
  const uint16_t *in, *out;
  int n_steps, n_slots, n_consts, n_in, n_out;
};
#define HC_PROG(NAME, UP)                                                                                  \
  HcProg{lsg_slp_##NAME##_w1_ops, lsg_slp_##NAME##_w1_steps, lsg_slp_##NAME##_w1_consts, lsg_slp_##NAME##_w1_in,  \
         lsg_slp_##NAME##_w1_out, LSG_SLP_##UP##_W1_N_STEPS, LSG_SLP_##UP##_W1_N_SLOTS,                           \
         LSG_SLP_##UP##_W1_N_CONSTS, LSG_SLP_##UP##_W1_N_IN, LSG_SLP_##UP##_W1_N_OUT},                           \
  HcProg{lsg_slp_##NAME##_w2_ops, lsg_slp_##NAME##_w2_steps, lsg_slp_##NAME##_w2_consts, lsg_slp_##NAME##_w2_in,  \
         lsg_slp_##NAME##_w2_out, LSG_SLP_##UP##_W2_N_STEPS, LSG_SLP_##UP##_W2_N_SLOTS,                           \
         LSG_SLP_##UP##_W2_N_CONSTS, LSG_SLP_##UP##_W2_N_IN, LSG_SLP_##UP##_W2_N_OUT}
extern "C" {
// prog: 2 k + (W - 1) for k = 0 final_exp, 1 miller_neg_g1, 2 horner_miller, 3 miller_item1,
// 4 h2c_clear, 5 g2_subgroup, 6 g2_scale (the last four with lane-form
// Montgomery inputs/outputs are converted here); in: the item's inputs as canonical 48-byte
// values; out: the canonical outputs (48 bytes each).  Returns the output count.
int hc_slp_run(int prog, const uint8_t* in, uint8_t* out) {
  const HcProg P[14] = {HC_PROG(final_exp, FINAL_EXP), HC_PROG(miller_neg_g1, MILLER_NEG_G1),
                        HC_PROG(horner_miller, HORNER_MILLER), HC_PROG(miller_item1, MILLER_ITEM1),
                        HC_PROG(h2c_clear, H2C_CLEAR), HC_PROG(g2_subgroup, G2_SUBGROUP),
                        HC_PROG(g2_scale, G2_SCALE)};
  const bool mont = prog / 2 >= 3;  // Montgomery-form inputs and outputs (lane-form programs)
  const fp_t r2 = fp_t(FP_R2), one = fp_t(FP_ONE_CANON);
  const HcProg& p = P[prog];
  std::vector<uint32_t> lds((size_t)p.n_slots * 16, 0xdeadbeefu);
  for (int j = 0; j < p.n_consts; j++) {
    fp_t v;
    for (int k = 0; k < 14; k++) v.l[k] = p.consts[14 * j + k];
    slot_store(lds.data(), j, 0, v);
  }
  for (int j = 0; j < p.n_in; j++) {
    fp_t x = fp_from_be_bytes(in + 48 * j, 12);
    if (mont) {
      fp_t m;
      pair_mont_mul_n<1>(&m, &x, &r2);
      x = m;
    }
    slot_store(lds.data(), p.in[j], 0, x);
  }
  for (int s = 0; s < p.n_steps; s++) {
    const uint32_t d = p.steps[s];
    for (uint32_t q = 0; q < (d & 255u); q++) slp_exec(lds.data(), p.ops + 8 * ((d >> 16) + q), in, 0, d);
  }
  for (int j = 0; j < p.n_out; j++) {
    if (mont) {
      fp_t c, v = slot_load(lds.data(), p.out[j], 0);
      pair_mont_mul_n<1>(&c, &v, &one);
      fp_to_be48(out + 48 * j, pair_canon_small(c));
    } else {
      fp_to_be48(out + 48 * j, slp_output(lds.data(), p.out[j], 0));
    }
  }
  return p.n_out;
}
}
#endif

#ifdef LSG_HOSTCHECK_PAIR
#include "lsg_inv.hpp"
extern "C" {
// x^-1 mod p by the divstep GCD of the INV operation (lsg_inv.hpp), canonical in and out
void hc_inv_gcd(const uint8_t* a48, uint8_t* out48) {
  const fp_t d = pair_inv_gcd(fp_from_be_bytes(a48, 12));
  fp_t m, c;
  const fp_t r2 = fp_t(FP_R2), one = fp_t(FP_ONE_CANON);
  pair_mont_mul_n<1>(&m, &d, &r2);  // d R mod p
  pair_mont_mul_n<1>(&c, &m, &one);  // d mod p, in (-p, 2p)
  fp_to_be48(out48, pair_canon_small(c));
}
}
#endif

#ifdef LSG_HOSTCHECK_PAIR
extern "C" {
// the Fp2 product leaf on raw lazy limbs (14 signed words per component, the pair layout with
// all limbs in one lane): a0, a1, b0, b1 in, (c0, c1) out -- for tests at the lazy bounds
void hc_pair_fp2_mul_raw(const int32_t* a, const int32_t* b, int32_t* out) {
  fp_t a0, a1, b0, b1, c0, c1;
  for (int k = 0; k < 14; k++) {
    a0.l[k] = (uint32_t)a[k];
    a1.l[k] = (uint32_t)a[14 + k];
    b0.l[k] = (uint32_t)b[k];
    b1.l[k] = (uint32_t)b[14 + k];
  }
  pair_fp2_mul_sop(c0, c1, a0, a1, b0, b1);
  for (int k = 0; k < 14; k++) {
    out[k] = (int32_t)c0.l[k];
    out[14 + k] = (int32_t)c1.l[k];
  }
}
}
#endif
