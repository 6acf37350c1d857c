// lsg_bls.hip -- gfx950 kernels and the C ABI (include/lodestar_bls.h) of the MI355X
// BLS12-381 signature-set verifier.
//
// Reference path replaced (file:line under /root/reference):
//   packages/beacon-node/src/chain/bls/multithread/worker.ts:30-114  (verifyManySignatureSets,
//       deserializeSet: batch-of-jobs verification with the per-job retry fallback)
//   packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39         (RLC batch vs single verify)
//   packages/beacon-node/src/chain/bls/utils.ts:5-26               (pubkey aggregation)
//   + the un-vendored @chainsafe/blst@0.2.8 arithmetic underneath.
//
// Execution model: every field element is limb-parallel over a lane pair (lsg_fp_pair.hpp,
// the default build; lsg_fp_quad.hpp / lsg_fp_lane.hpp are alternative builds), so one work
// item (a set, a pubkey, a group) is one pair and a wave64 carries 32 items.  Per package:
//   k_expand_msg      expand_message_xmd (SHA-256), one thread per set          [M3]
//   k_sig_decode      96/192-byte signature -> affine G2                         [M2]
//   k_sig_subgroup    psi(P) == [x]P                                             [M2]
//   k_pk_decode       48/96-byte pubkey -> projective G1 (on-curve only)         [H8]
//   tree(G1 add)      per-set pubkey aggregation, pairwise over levels           [M1]
//   k_pk_scale        P_i = [r_i] agg_i; batched 1/Z; k_pk_affine               [M4]
//   k_h2c_prep/map/affine  hash_to_field -> SSWU x2 -> 3-isogeny -> add ->
//                     clear_cofactor -> affine, inversions batched per stage       [M3]
//   k_sig_proj        sig_i for the bucket MSM (k_sig_scale [r_i] sig_i for small groups) [M4]
//   k_miller_multi    f_item = prod of ML(P_i, H(m_i)) over <= K sets            [M5]
// then per group (an RLC batch = a chunk of batchable jobs, or one job):
//   msm_buckets/msm_bits   per-bit sums C_{g,k} of sum r_i sig_i (8-bit windows)
//   k_row_horner_miller    S_g = sum_k 2^k C_{g,k}, f_g = ML(-G1, S_g)   (row backend, lsg_serial.hip)
//   tree(Fp12 mul)    F_g = f_g prod f_item
//   k_row_final_exp   FE(F_g) == 1                                               [M6]
// Per-set values stay resident between the batch attempt and the per-job retry.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/lodestar_bls.h"
#include "lsg_serial.h"

// The math headers go into an anonymous namespace: lsg_serial.hip instantiates the same
// generic code over the row backend, and the two fp_t must never be merged at link time.
namespace {
#if defined(LSG_BACKEND_ROW)
#include "lsg_fp_lane.hpp"  // one element per 16-lane DPP row
#elif defined(LSG_BACKEND_QUAD)
#include "lsg_fp_quad.hpp"  // one element per 4-lane quad, fully reduced 32-bit limbs
#else
#include "lsg_fp_pair.hpp"  // one element per lane pair, lazy radix-2^29 limbs (default)
#endif
#include "lsg_h2c.hpp"
#include "lsg_io.hpp"
}  // namespace

#define LSG_TPB 256  // threads per block
// Register budget of the lane kernels: waves per SIMD the compiler must leave room for
// (it spills beyond that).  See DESIGN.md section 4 for the measured trade-off.
#ifndef LSG_WAVES_PER_EU
#ifdef LSG_PAIR_MODE
#define LSG_WAVES_PER_EU 2  // pair: 256 VGPRs (1.32M vs 1.15M sets/s at 3, 1.06M at 4)
#else
#define LSG_WAVES_PER_EU 4
#endif
#endif
#define LSG_KERNEL_ATTR __launch_bounds__(LSG_TPB) __attribute__((amdgpu_waves_per_eu(LSG_WAVES_PER_EU)))
// per-kernel register budget (waves per SIMD) for the kernels whose live state does not fit
// 256 registers: at 1 wave per SIMD a wave owns 512 (VGPRs + AGPRs) instead of spilling
#define LSG_KERNEL_ATTR_W(w) __launch_bounds__(LSG_TPB) __attribute__((amdgpu_waves_per_eu(w)))
#ifndef LSG_H2C_WAVES
#define LSG_H2C_WAVES LSG_WAVES_PER_EU
#endif
#ifndef LSG_H2C_SPLIT
#define LSG_H2C_SPLIT 1
#endif
#ifndef LSG_SUBGROUP_WAVES
#define LSG_SUBGROUP_WAVES LSG_WAVES_PER_EU
#endif
#define LSG_ITEMS_PER_BLOCK (LSG_TPB / LSG_GROUP)

static __device__ __forceinline__ size_t gtid() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }
#define LANE_ITEM(n)                        \
  lsg_lane_setup();                         \
  const size_t item = gtid() / LSG_GROUP;   \
  if (item >= (size_t)(n)) return;          \
  const bool lead = (threadIdx.x % LSG_GROUP) == 0

// ---------------------------------------------------------------------------- kernels
// expand_message_xmd(msg_i, DST, 256): one thread per set (byte-serial SHA-256)
__global__ void __launch_bounds__(64) k_expand_msg(int n, const uint8_t* __restrict__ msg,
                                                    const uint32_t* __restrict__ msg_off,
                                                    const uint32_t* __restrict__ msg_len,
                                                    const uint8_t* __restrict__ dst, uint32_t dst_len,
                                                    uint8_t* __restrict__ ub) {
  size_t i = gtid();
  if (i >= (size_t)n) return;
  uint8_t out[256];
  expand_message_xmd_256(out, msg + msg_off[i], msg_len[i], dst, dst_len);
  uint32_t* o = (uint32_t*)(ub + 256 * i);
  for (int k = 0; k < 64; k++) {
    uint32_t w;
    __builtin_memcpy(&w, out + 4 * k, 4);
    o[k] = w;
  }
}

__global__ void LSG_KERNEL_ATTR k_sig_decode(int n, const uint8_t* __restrict__ sig,
                                                         const uint32_t* __restrict__ sig_len,
                                                         uint32_t* __restrict__ sig_aff, uint8_t* __restrict__ inf,
                                                         int32_t* __restrict__ err) {
  LANE_ITEM(n);
  uint32_t len = sig_len[item];
  g2a_t p;
  p.x = fp2_zero();
  p.y = fp2_zero();
  bool is_inf = false;
  int e;
  if (len == 96)
    e = g2_uncompress(p, is_inf, sig + 192 * item);
  else if (len == 192)
    e = g2_deserialize_uncompressed(p, is_inf, sig + 192 * item);
  else
    e = LSG_BLST_INVALID_SIZE;
  lane_store(sig_aff, item, p);
  if (lead) {
    inf[item] = is_inf ? 1 : 0;
    err[item] = e;
  }
}

__global__ void LSG_KERNEL_ATTR_W(LSG_SUBGROUP_WAVES) k_sig_subgroup(int n, const uint32_t* __restrict__ sig_aff,
                                                           const uint8_t* __restrict__ inf, int32_t* __restrict__ err) {
  LANE_ITEM(n);
  if (err[item] != 0 || inf[item]) return;
  bool ok = g2_in_group(proj_from_aff(lane_load<g2a_t>(sig_aff, item)));
  if (lead && !ok) err[item] = LSG_BLST_POINT_NOT_IN_GROUP;
}

// pubkey -> projective G1 (infinity and undecodable keys become (0:1:0)).  A key given by
// index (len == LSG_PK_INDEX: the slot's first 4 bytes) is gathered from the resident table
// (tab, tab_ok: decoded keys of lsg_pubkey_table_set; tab_n indices).
__global__ void LSG_KERNEL_ATTR k_pk_decode(int n, const uint8_t* __restrict__ pk,
                                                        const uint32_t* __restrict__ pk_len, uint32_t* __restrict__ pkp,
                                                        int32_t* __restrict__ err, const uint32_t* __restrict__ tab,
                                                        const uint8_t* __restrict__ tab_ok, uint32_t tab_n) {
  LANE_ITEM(n);
  uint32_t len = pk_len[item];
  g1p_t p = proj_inf<fp_t>();
  int e;
  if (len == LSG_PK_INDEX) {
    const uint8_t* b = pk + 96 * item;
    const uint32_t idx = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    const bool ok = idx < tab_n && tab_ok[idx];
    e = ok ? 0 : LSG_ERR_BAD_INDEX;
    if (ok) p = lane_load<g1p_t>(tab, idx);
  } else {
    g1a_t a;
    a.x = fp_zero();
    a.y = fp_zero();
    bool is_inf = false;
    e = (len == 48 || len == 96) ? g1_deserialize(a, is_inf, pk + 96 * item, (int)len) : LSG_BLST_INVALID_SIZE;
    if (e == 0 && !is_inf) p = proj_from_aff(a);
  }
  lane_store(pkp, item, p);
  if (lead) err[item] = e;
}

// KeyValidate (lsg_pubkey_validate): decode, reject infinity and points outside G1; pts
// receives the key as a projective point (the identity for rejected keys); keys sit in the
// staging arena's 96-byte slots
__global__ void LSG_KERNEL_ATTR k_pk_validate(int n, const uint8_t* __restrict__ pk, uint32_t len,
                                              uint32_t* __restrict__ pts, int32_t* __restrict__ err) {
  LANE_ITEM(n);
  g1a_t a;
  a.x = fp_zero();
  a.y = fp_zero();
  bool is_inf = false;
  int e = g1_deserialize(a, is_inf, pk + 96 * item, (int)len);
  if (e == 0 && is_inf) e = LSG_BLST_PK_IS_INFINITY;
  const g1p_t p = e == 0 ? proj_from_aff(a) : proj_inf<fp_t>();
  if (e == 0 && !g1_in_group(p)) e = LSG_BLST_POINT_NOT_IN_GROUP;
  lane_store(pts, item, e == 0 ? p : proj_inf<fp_t>());
  if (lead) err[item] = e;
}

// ---- batched field inversion (Montgomery's trick as a product tree over the batch): every
// field inversion of a stage -- 1/Z of the scaled pubkeys, 1/N(tv1) of the SSWU maps, 1/N(Z)
// of the hashed points -- shares one exponentiation per batch instead of one per set.
// Zero inputs (points at infinity, the SSWU exceptional case) are carried as 1 through the
// tree and come out as 0, the value fp_inv(0) gives.
// level up: out[i] = in[2i] * in[2i+1] (a missing right child is 1)
__global__ void LSG_KERNEL_ATTR k_binv_up(int n_out, int n_in, int zero_to_one,
                                                      const uint32_t* __restrict__ in, uint32_t* __restrict__ out) {
  LANE_ITEM(n_out);
  const fp_t one = fp_one();
  fp_t a = lane_load<fp_t>(in, 2 * item);
  fp_t b = (2 * (int)item + 1 < n_in) ? lane_load<fp_t>(in, 2 * item + 1) : one;
  if (zero_to_one) {
    a = fp_select(fp_is_zero(a), one, a);
    b = fp_select(fp_is_zero(b), one, b);
  }
  lane_store(out, item, fp_mul(a, b));
}
__global__ void LSG_KERNEL_ATTR k_binv_root(const uint32_t* __restrict__ top, uint32_t* __restrict__ inv) {
  LANE_ITEM(1);
  lane_store(inv, 0, fp_inv(lane_load<fp_t>(top, 0)));
}
// level down: inv(child c) = inv(parent c/2) * value(sibling c^1); at level 0 (zero_to_one)
// zero children get 0
__global__ void LSG_KERNEL_ATTR k_binv_down(int n_child, int zero_to_one, const uint32_t* __restrict__ vals,
                                                        const uint32_t* __restrict__ pinv, uint32_t* __restrict__ cinv) {
  LANE_ITEM(n_child);
  const fp_t one = fp_one();
  const int sib = (int)item ^ 1;
  fp_t s = sib < n_child ? lane_load<fp_t>(vals, sib) : one;
  if (zero_to_one) s = fp_select(fp_is_zero(s), one, s);
  fp_t r = fp_mul(lane_load<fp_t>(pinv, item >> 1), s);
  if (zero_to_one) r = fp_select(fp_is_zero(lane_load<fp_t>(vals, item)), fp_zero(), r);
  lane_store(cinv, item, r);
}

// P_i = [r_i] agg_i, projective (r_i == 0: no scaling); zP_i = its Z (0 at infinity) for the
// batched inversion; pinf = aggregate is infinity
__global__ void LSG_KERNEL_ATTR k_pk_scale(int n, const uint32_t* __restrict__ agg,
                                                       const uint64_t* __restrict__ rnd, uint32_t* __restrict__ Pp,
                                                       uint32_t* __restrict__ zP, uint8_t* __restrict__ pinf) {
  LANE_ITEM(n);
  g1p_t acc = lane_load<g1p_t>(agg, item);
  uint64_t r = rnd[item];
  bool is_inf = proj_is_inf(acc);
  if (r != 0 && !is_inf) acc = proj_mul_u64(acc, r);
  lane_store(Pp, item, acc);
  lane_store(zP, item, is_inf ? fp_zero() : acc.Z);
  if (lead) pinf[item] = is_inf ? 1 : 0;
}
// P_i affine = (X / Z, Y / Z) with 1/Z from the batched inversion
__global__ void LSG_KERNEL_ATTR k_pk_affine(int n, const uint32_t* __restrict__ Pp,
                                                        const uint32_t* __restrict__ zinv, uint32_t* __restrict__ P) {
  LANE_ITEM(n);
  g1p_t p = lane_load<g1p_t>(Pp, item);
  fp_t zi = lane_load<fp_t>(zinv, item);
  g1a_t a;
  fp_mul2(a.x, a.y, p.X, zi, p.Y, zi);
  lane_store(P, item, a);
}

// hash_to_G2, stage 1: u0, u1 = hash_to_field(expand_message_xmd); norms N(tv1(u0)),
// N(tv1(u1)) at slots 2i, 2i+1 for the batched inversion
struct h2c_u_t {
  fp2_t u0, u1;
};
__global__ void LSG_KERNEL_ATTR k_h2c_prep(int n, const uint8_t* __restrict__ ub, uint32_t* __restrict__ U,
                                                       uint32_t* __restrict__ norms) {
  LANE_ITEM(n);
  const uint8_t* b = ub + 256 * item;
  h2c_u_t u;
  u.u0 = fp2_make(fp_from_be64_mod(b), fp_from_be64_mod(b + 64));
  u.u1 = fp2_make(fp_from_be64_mod(b + 128), fp_from_be64_mod(b + 192));
  lane_store(U, item, u);
  lane_store(norms, 2 * item, fp2_norm(sswu_tv1(u.u0)));
  lane_store(norms, 2 * item + 1, fp2_norm(sswu_tv1(u.u1)));
}
// stage 2: SSWU x2 (with the batched 1/N(tv1)) -> 3-isogeny -> add -> clear_cofactor,
// projective; zN_i = N(Z) (0 at infinity) for the second batched inversion
__global__ void LSG_KERNEL_ATTR_W(LSG_H2C_WAVES) k_h2c_map(int n, const uint32_t* __restrict__ U,
                                                      const uint32_t* __restrict__ ninv, uint32_t* __restrict__ Hp,
                                                      uint32_t* __restrict__ zN, uint8_t* __restrict__ hinf) {
  LANE_ITEM(n);
  h2c_u_t u = lane_load<h2c_u_t>(U, item);
  g2p_t q0 = iso_map3(map_to_curve_sswu_ni(u.u0, lane_load<fp_t>(ninv, 2 * item)));
  g2p_t q1 = iso_map3(map_to_curve_sswu_ni(u.u1, lane_load<fp_t>(ninv, 2 * item + 1)));
#if LSG_H2C_SPLIT
  lane_store(Hp, item, g2_add(q0, q1));  // k_h2c_clear finishes the point
#else
  g2p_t q = clear_cofactor_g2(g2_add(q0, q1));
  bool is_inf = proj_is_inf(q);
  lane_store(Hp, item, q);
  lane_store(zN, item, is_inf ? fp_zero() : fp2_norm(q.Z));
  if (lead) hinf[item] = is_inf ? 1 : 0;
#endif
}
// stage 2b (LSG_H2C_SPLIT): clear_cofactor in place.  Split from the map so that neither
// kernel holds the other's live state: the fused kernel spilled 757 registers.
__global__ void LSG_KERNEL_ATTR_W(LSG_H2C_WAVES) k_h2c_clear(int n, uint32_t* __restrict__ Hp,
                                                            uint32_t* __restrict__ zN, uint8_t* __restrict__ hinf) {
  LANE_ITEM(n);
  g2p_t q = clear_cofactor_g2(lane_load<g2p_t>(Hp, item));
  bool is_inf = proj_is_inf(q);
  lane_store(Hp, item, q);
  lane_store(zN, item, is_inf ? fp_zero() : fp2_norm(q.Z));
  if (lead) hinf[item] = is_inf ? 1 : 0;
}
// stage 3: H affine = (X, Y) * conj(Z) / N(Z)   (= proj_to_aff, 1/Z = conj(Z) / N(Z))
__global__ void LSG_KERNEL_ATTR k_h2c_affine(int n, const uint32_t* __restrict__ Hp,
                                                         const uint32_t* __restrict__ ninv, const uint8_t* __restrict__ hinf,
                                                         uint32_t* __restrict__ H) {
  LANE_ITEM(n);
  g2p_t q = lane_load<g2p_t>(Hp, item);
  g2a_t a;
  if (hinf[item]) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    fp2_t zi = fp2_inv_with_norm_inv(q.Z, lane_load<fp_t>(ninv, item));
    a.x = fp2_mul(q.X, zi);
    a.y = fp2_mul(q.Y, zi);
  }
  lane_store(H, item, a);
}

__global__ void LSG_KERNEL_ATTR k_sig_scale(int n, const uint32_t* __restrict__ sig_aff,
                                                        const uint8_t* __restrict__ inf, const int32_t* __restrict__ err,
                                                        const uint64_t* __restrict__ rnd, uint32_t* __restrict__ rs) {
  LANE_ITEM(n);
  g2p_t r = proj_inf<fp2_t>();
  if (err[item] == 0 && !inf[item]) r = proj_mul_u64(proj_from_aff(lane_load<g2a_t>(sig_aff, item)), rnd[item]);
  lane_store(rs, item, r);
}

// f_item = prod over the item's sets (<= K consecutive sets of one job) of ML(P_i, H(m_i)):
// one shared f and one squaring per loop step for all K pairs.  Sets with errors or an
// infinite point contribute 1.
template <int K>
__global__ void LSG_KERNEL_ATTR k_miller_multi(int n_items, const int32_t* __restrict__ item_first,
                                                           const int32_t* __restrict__ item_cnt,
                                                           const uint32_t* __restrict__ P,
                                                           const uint8_t* __restrict__ pinf, const uint32_t* __restrict__ H,
                                                           const uint8_t* __restrict__ hinf,
                                                           const int32_t* __restrict__ err, uint32_t* __restrict__ f) {
  LANE_ITEM(n_items);
  const int first = item_first[item], cnt = item_cnt[item];
  g1a_t Pk[K];
  g2a_t Qk[K];
  bool use[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int i = first + (k < cnt ? k : cnt - 1);
    use[k] = k < cnt && err[i] == 0 && !pinf[i] && !hinf[i];
    Pk[k] = lane_load<g1a_t>(P, i);
    Qk[k] = lane_load<g2a_t>(H, i);
  }
  lane_store(f, item, miller_loop_multi<K>(Pk, Qk, use));
}

// ---- split Miller loop (lsg_pairing.hpp: miller_lines / miller_accum_multi)
// Line storage is word-major over sets: word k (of the W per lane of a line_t) of step st of
// set i lives at lines[((st * W + k) * n + i) * G + h], so one store or load instruction of a
// wave touches one contiguous 256-byte run.  ML_STEPS lines = 68 x 6 Fp per set (~22.8 KB).
constexpr int W_LINE = (int)(sizeof(line_t) / 4);
LSG_DEVI void line_store(uint32_t* __restrict__ lines, size_t n, size_t i, int st, const line_t& L) {
  uint32_t w[W_LINE];
  __builtin_memcpy(w, &L, sizeof(line_t));
  uint32_t* p = lines + (((size_t)st * W_LINE) * n + i) * LSG_GROUP + (threadIdx.x % LSG_GROUP);
#pragma unroll
  for (int k = 0; k < W_LINE; k++) p[(size_t)k * n * LSG_GROUP] = w[k];
}
LSG_DEVI line_t line_load(const uint32_t* __restrict__ lines, size_t n, size_t i, int st) {
  uint32_t w[W_LINE];
  const uint32_t* p = lines + (((size_t)st * W_LINE) * n + i) * LSG_GROUP + (threadIdx.x % LSG_GROUP);
#pragma unroll
  for (int k = 0; k < W_LINE; k++) w[k] = p[(size_t)k * n * LSG_GROUP];
  line_t L;
  __builtin_memcpy(&L, w, sizeof(line_t));
  return L;
}

// the G2 half: the 68 unevaluated lines of Q_i = H(m_i) for every set (no dependency on the
// pubkey side, so it runs as soon as hash_to_G2 is done).  Sets whose point is unusable still
// run the chain on whatever Q holds: every lane pair follows one control path.
__global__ void LSG_KERNEL_ATTR k_miller_lines(int n, const uint32_t* __restrict__ H, uint32_t* __restrict__ lines) {
  LANE_ITEM(n);
  const g2a_t Q = lane_load<g2a_t>(H, item);
  miller_lines(Q, [&](int st, const line_t& L) { line_store(lines, (size_t)n, item, st, L); });
}

// the Fp12 half: f_item = prod over the item's <= K sets of their lines evaluated at P_i,
// with shared squarings -- the value k_miller_multi computes
#ifndef LSG_ACCUM_WAVES
#define LSG_ACCUM_WAVES 1  // 512 registers: f, the line and the products stay out of scratch (1.33M -> 1.43M sets/s)
#endif
template <int K>
__global__ void LSG_KERNEL_ATTR_W(LSG_ACCUM_WAVES) k_miller_accum(int n_items, const int32_t* __restrict__ item_first,
                                               const int32_t* __restrict__ item_cnt, const uint32_t* __restrict__ P,
                                               const uint8_t* __restrict__ pinf, const uint8_t* __restrict__ hinf,
                                               const int32_t* __restrict__ err, int n_sets,
                                               const uint32_t* __restrict__ lines, uint32_t* __restrict__ f) {
  LANE_ITEM(n_items);
  const int first = item_first[item], cnt = item_cnt[item];
  g1a_t Pk[K];
  bool use[K];
  int idx[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int i = first + (k < cnt ? k : cnt - 1);
    idx[k] = i;
    use[k] = k < cnt && err[i] == 0 && !pinf[i] && !hinf[i];
    Pk[k] = lane_load<g1a_t>(P, i);
  }
  lane_store(f, item, miller_accum_multi<K>(Pk, use, [&](int k, int st) {
               return line_load(lines, (size_t)n_sets, (size_t)idx[k], st);
             }));
}

// one level of a segmented pairwise reduction: dst[k] = src[ia[k]] (+) src[ib[k]]  (ib < 0: copy;
// ia < 0: the identity, for an empty group)
template <int OP>  // OP 2 (Fp12 products) gets 1 wave per SIMD: its operands do not fit 256 registers
__global__ void LSG_KERNEL_ATTR_W(OP == 2 ? 1 : LSG_WAVES_PER_EU) k_tree_level(int n, const int32_t* __restrict__ ia,
                                                         const int32_t* __restrict__ ib, const uint32_t* __restrict__ src,
                                                         uint32_t* __restrict__ dst) {
  LANE_ITEM(n);
  int32_t a = ia[item], b = ib[item];
  if (OP == 0) {
    g1p_t x = a >= 0 ? lane_load<g1p_t>(src, a) : proj_inf<fp_t>();
    if (b >= 0) x = g1_add(x, lane_load<g1p_t>(src, b));
    lane_store(dst, item, x);
  } else if (OP == 1) {
    g2p_t x = a >= 0 ? lane_load<g2p_t>(src, a) : proj_inf<fp2_t>();
    if (b >= 0) x = g2_add(x, lane_load<g2p_t>(src, b));
    lane_store(dst, item, x);
  } else {
    fp12_t x = a >= 0 ? lane_load<fp12_t>(src, a) : fp12_one();
    if (b >= 0) x = fp12_mul(x, lane_load<fp12_t>(src, b));
    lane_store(dst, item, x);
  }
}

// Signature points for the bucket MSM: projective sig_i, or the identity for a set whose
// signature did not decode or is the point at infinity (same contribution as k_sig_scale's)
__global__ void LSG_KERNEL_ATTR k_sig_proj(int n, const uint32_t* __restrict__ sig_aff,
                                                       const uint8_t* __restrict__ inf, const int32_t* __restrict__ err,
                                                       uint32_t* __restrict__ out) {
  LANE_ITEM(n);
  g2p_t r = proj_inf<fp2_t>();
  if (err[item] == 0 && !inf[item]) r = proj_from_aff(lane_load<g2a_t>(sig_aff, item));
  lane_store(out, item, r);
}


// partials: canonical big-endian 576-byte Fp12 blobs -> lane form (one item each)
__global__ void LSG_KERNEL_ATTR k_blobs_to_fp12(int n, const uint8_t* __restrict__ blobs,
                                                            uint32_t* __restrict__ out) {
  LANE_ITEM(n);
  lane_store(out, item, fp12_from_canon_bytes(blobs + 576 * item));
}

__global__ void LSG_KERNEL_ATTR k_fp12_to_canon(int n, const uint32_t* __restrict__ in,
                                                            uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  fp12_to_canon_bytes(out + 576 * item, lane_load<fp12_t>(in, item));
}

// group signature sums S_g (lane form) -> canonical 288-byte projective points for the row stage
__global__ void LSG_KERNEL_ATTR k_g2p_to_canon(int n, const uint32_t* __restrict__ in,
                                                           uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  g2p_to_canon_bytes(out + 288 * item, lane_load<g2p_t>(in, item));
}

__global__ void LSG_KERNEL_ATTR k_g1p_to_bytes(int n, const uint32_t* __restrict__ pts,
                                                           uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  g1p_t p = lane_load<g1p_t>(pts, item);
  bool inf = proj_is_inf(p);
  g1a_t a;
  if (inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    a = proj_to_aff(p);
  }
  g1_serialize(out + 96 * item, a, inf);
}

__global__ void LSG_KERNEL_ATTR k_g2a_to_bytes(int n, const uint32_t* __restrict__ pts,
                                                           const uint8_t* __restrict__ inf, uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  g2_serialize(out + 192 * item, lane_load<g2a_t>(pts, item), inf[item] != 0);
}

// [k]P for a 256-bit big-endian scalar (test-data utilities only: signing, keygen)
template <class F>
__device__ proj_t<F> proj_mul_be256(const proj_t<F>& p, const uint8_t* k) {
  proj_t<F> acc = proj_inf<F>();
  for (int byte = 0; byte < 32; byte++) {
    uint32_t v = k[byte];
    for (int b = 7; b >= 0; b--) {
      acc = gdbl(acc);
      proj_t<F> s = gadd(acc, p);
      bool bit = (v >> b) & 1u;
      acc.X = fselect(bit, s.X, acc.X);
      acc.Y = fselect(bit, s.Y, acc.Y);
      acc.Z = fselect(bit, s.Z, acc.Z);
    }
  }
  return acc;
}

// sig_i = [sk_i] H(m_i), ZCash-compressed (bench/test input generation; not on the verify path)
__global__ void LSG_KERNEL_ATTR k_sign(int n, const uint8_t* __restrict__ sks, const uint32_t* __restrict__ H,
                                                   uint8_t* __restrict__ out96) {
  LANE_ITEM(n);
  g2p_t s = proj_mul_be256(proj_from_aff(lane_load<g2a_t>(H, item)), sks + 32 * item);
  bool inf = proj_is_inf(s);
  g2a_t a;
  if (inf) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    a = proj_to_aff(s);
  }
  g2_compress(out96 + 96 * item, a, inf);
}

// op-pool aggregates (lsg_aggregate_signatures): projective G2 sums -> ZCash-compressed
// 96 bytes, Signature.toBytes() of the aggregate (the identity -> 0xc0 || 0^95)
__global__ void LSG_KERNEL_ATTR k_g2p_compress(int n, const uint32_t* __restrict__ pts,
                                               uint8_t* __restrict__ out96) {
  LANE_ITEM(n);
  g2p_t p = lane_load<g2p_t>(pts, item);
  bool inf = proj_is_inf(p);
  g2a_t a;
  if (inf) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    a = proj_to_aff(p);
  }
  g2_compress(out96 + 96 * item, a, inf);
}

// ---- SSZ signing roots, one thread per object.  Chunks are 8 big-endian
// SHA-256 words; every node is SHA-256 of exactly 64 bytes, so its second block is the
// constant padding block of a 512-bit message.
LSG_INL void ssz_hash2(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint32_t blk[16];
  for (int k = 0; k < 8; k++) {
    blk[k] = a[k];
    blk[8 + k] = b[k];
  }
  sha256_compress(st, blk);
  for (int k = 0; k < 16; k++) blk[k] = 0;
  blk[0] = 0x80000000u;
  blk[15] = 512;
  sha256_compress(st, blk);
  for (int k = 0; k < 8; k++) out[k] = st[k];
}

// `len` (<= 32) bytes at p as a zero-padded SSZ chunk
LSG_INL void ssz_chunk(uint32_t* w, const uint8_t* p, int len) {
  for (int k = 0; k < 8; k++) {
    uint32_t v = 0;
    for (int j = 0; j < 4; j++) v = (v << 8) | (4 * k + j < len ? p[4 * k + j] : 0u);
    w[k] = v;
  }
}

LSG_INL void ssz_store(uint8_t* out, const uint32_t* w) { be_words_to_bytes(out, w, 8); }

// hash_tree_root(SigningData{objectRoot, domain}) (util/signingRoot.ts:7-13)
__global__ void __launch_bounds__(64) k_signing_root(int n, const uint8_t* __restrict__ roots,
                                                     const uint8_t* __restrict__ domains, uint32_t dstride,
                                                     uint8_t* __restrict__ out32) {
  size_t i = gtid();
  if (i >= (size_t)n) return;
  uint32_t r[8], d[8], o[8];
  ssz_chunk(r, roots + 32 * i, 32);
  ssz_chunk(d, domains + dstride * i, 32);
  ssz_hash2(r, d, o);
  ssz_store(out32 + 32 * i, o);
}

// getAttestationDataSigningRoot (signatureSets/indexedAttestation.ts:11-19) from the SSZ
// serialization of phase0.AttestationData (128 bytes: slot u64, index u64, beaconBlockRoot,
// source {epoch u64, root}, target {epoch u64, root}): 5 fields -> 8 leaves, 3 levels, then
// SigningData -- 10 node hashes per object
__global__ void __launch_bounds__(64) k_attestation_signing_root(int n, const uint8_t* __restrict__ data,
                                                                 const uint8_t* __restrict__ domains,
                                                                 uint32_t dstride, uint8_t* __restrict__ out32) {
  size_t i = gtid();
  if (i >= (size_t)n) return;
  const uint8_t* a = data + 128 * i;
  uint32_t l0[8], l1[8], l2[8], l3[8], l4[8], t[8], z[8], z1[8], h01[8], h23[8], h45[8];
  for (int k = 0; k < 8; k++) z[k] = 0;
  ssz_chunk(l0, a, 8);       // slot
  ssz_chunk(l1, a + 8, 8);   // index
  ssz_chunk(l2, a + 16, 32); // beaconBlockRoot
  ssz_chunk(t, a + 48, 8);   // source = Checkpoint{epoch, root}
  ssz_chunk(l3, a + 56, 32);
  ssz_hash2(t, l3, l3);
  ssz_chunk(t, a + 88, 8);   // target
  ssz_chunk(l4, a + 96, 32);
  ssz_hash2(t, l4, l4);
  ssz_hash2(z, z, z1);       // leaves 5..7 are zero chunks
  ssz_hash2(l0, l1, h01);
  ssz_hash2(l2, l3, h23);
  ssz_hash2(l4, z, h45);
  ssz_hash2(h01, h23, h01);
  ssz_hash2(h45, z1, h45);
  ssz_hash2(h01, h45, t);    // AttestationData.hashTreeRoot
  ssz_chunk(z, domains + dstride * i, 32);
  ssz_hash2(t, z, t);
  ssz_store(out32 + 32 * i, t);
}

// pk_i = [sk_i] G1, uncompressed 96 bytes (bench/test input generation)
__global__ void LSG_KERNEL_ATTR k_sk_to_pk(int n, const uint8_t* __restrict__ sks,
                                                       uint8_t* __restrict__ out96) {
  LANE_ITEM(n);
  g1a_t g;
  g.x = fp_t(G1_GEN_X);
  g.y = fp_t(G1_GEN_Y);
  g1p_t s = proj_mul_be256(proj_from_aff(g), sks + 32 * item);
  bool inf = proj_is_inf(s);
  g1a_t a;
  if (inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    a = proj_to_aff(s);
  }
  g1_serialize(out96 + 96 * item, a, inf);
}

// roofline probe: 4 independent limb-parallel Montgomery chains per row
__global__ void LSG_KERNEL_ATTR k_probe_fp_mul(int n, int iters, uint32_t* __restrict__ io) {
  LANE_ITEM(n);
  fp_t a = lane_load<fp_t>(io, item), b = fp_t(FP_R2), c = fp_t(FP_R3), d = fp_t(FP_HALF);
  for (int k = 0; k < iters; k++) {
    a = fp_mul(a, b);
    b = fp_mul(b, c);
    c = fp_mul(c, d);
    d = fp_mul(d, a);
  }
  lane_store(io, item, fp_add(fp_add(a, b), fp_add(c, d)));
}

// roofline probe: raw v_mad_u64_u32 issue rate, 16 independent 64-bit accumulators per lane
__global__ void __launch_bounds__(256) k_probe_mad(int iters, uint32_t seed, uint64_t* __restrict__ io) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc[16];
  uint32_t x[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    acc[k] = t + k;
    x[k] = (t * 2654435761u) ^ (seed + 977u * k);
  }
  const uint32_t y = seed | 1u;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 16; k++) acc[k] = (uint64_t)x[k] * y + acc[k];
  }
  uint64_t r = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) r ^= acc[k];
  io[t] = r;
}

// ---------------------------------------------------------------------------- host side
//
// Pipelining.  A context owns LSG_SLOTS pipeline slots; each slot has two streams (main:
// hash_to_G2 -> Miller loops -> products -> FE; side: pubkeys -> signatures -> RLC sums ->
// signature Miller loop), its own device state and pinned host mirrors.  A submit call
// launches one package on a free slot and returns a ticket without waiting; the matching
// wait call synchronises on the slot's completion event and applies the reference's verdict
// rules.  Final exponentiations of all-gathered partials run on a dedicated stream, so the
// serial FE of batch k overlaps the per-set stages of batch k+1.
namespace {

const uint8_t DST_POP[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
const uint32_t DST_POP_LEN = 43;
constexpr int LSG_SLOTS = 16;  // batch / job slots in flight
constexpr int LSG_FINALS = 64;  // final-exponentiation entries in flight
constexpr int LSG_FE_STREAMS = 8;  // streams the final exponentiations run on

// u32 words per item for each lane-form type
constexpr size_t W_G1A = lane_words<g1a_t>();
constexpr size_t W_G1P = lane_words<g1p_t>();
constexpr size_t W_G2A = lane_words<g2a_t>();
constexpr size_t W_G2P = lane_words<g2p_t>();
constexpr size_t W_F12 = lane_words<fp12_t>();

uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

struct HostBuf {  // pinned host memory (async copies)
  void* p = nullptr;
  size_t cap = 0;
};

struct Timer {
  const char* name;
  hipEvent_t a, b;
};

struct TreeSlot {
  DevBuf idx, tA, tB;
  std::vector<int32_t> host;  // index pairs of the last reduction (alive until the slot completes)
};

// Index plan of a segmented pairwise reduction (see tree_reduce): per level, the pairs
// (ia[k], ib[k]) of the level's inputs; the last level gathers one value per group.
struct TreePlan {
  std::vector<int32_t> idx;                       // per level: ia[cnt] then ib[cnt]
  std::vector<std::pair<size_t, size_t>> levels;  // (offset into idx, cnt)
  size_t max_level = 0;
};

TreePlan plan_tree(const std::vector<std::vector<int32_t>>& groups) {
  TreePlan P;
  size_t ng = groups.size();
  std::vector<std::vector<int32_t>> cur = groups;
  for (;;) {
    bool done = true;
    for (auto& g : cur)
      if (g.size() > 1) done = false;
    size_t cnt = 0;
    std::vector<int32_t> ia, ib;
    std::vector<std::vector<int32_t>> nxt(ng);
    if (done) {  // final gather into out[g] (an empty group gets the identity)
      for (size_t g = 0; g < ng; g++) {
        ia.push_back(!cur[g].empty() ? cur[g][0] : -1);
        ib.push_back(-1);
      }
      cnt = ng;
    } else {
      for (size_t g = 0; g < ng; g++) {
        for (size_t k = 0; k < cur[g].size(); k += 2) {
          ia.push_back(cur[g][k]);
          ib.push_back(k + 1 < cur[g].size() ? cur[g][k + 1] : -1);
          nxt[g].push_back((int32_t)cnt++);
        }
      }
    }
    // a level that leaves group g's single value in slot g is the last one: it writes out[]
    // directly and the gather launch is skipped (one launch less per tree on the chain)
    bool placed = !done;
    for (size_t g = 0; placed && g < ng; g++)
      if (nxt[g].size() != 1 || nxt[g][0] != (int32_t)g) placed = false;
    P.levels.push_back({P.idx.size(), cnt});
    P.idx.insert(P.idx.end(), ia.begin(), ia.end());
    P.idx.insert(P.idx.end(), ib.begin(), ib.end());
    P.max_level = std::max(P.max_level, cnt);
    if (done || placed) break;
    cur.swap(nxt);
  }
  return P;
}

// Bucket MSM plan of the RLC signature sums of one staged package split into groups of
// group_size consecutive sets (Pippenger, 8-bit windows, planned on the host from the
// known randomizers r_i):
//   bucket (g, w, d), d = 1..255: the sets i of group g whose w-th byte of r_i is d
//   bit (g, k = 8w + j): the buckets (g, w, d) whose digit d has bit j set
// so that sum_i r_i sig_i = sum_k 2^k bit(g, k) (Horner in k_row_horner_miller).  Device copies of the index
// plans are kept with the package and shared by every ticket that submits it.
struct MsmPlan {
  size_t group_size = 0, ng = 0;
  bool valid = false;
  TreePlan buckets, bits;
  DevBuf d_buckets, d_bits;
};
constexpr int MSM_WINDOWS = 8, MSM_DIGITS = 255, MSM_BITS = 64;

// chunkifyMaximizeChunkSize (multithread/utils.ts:4-19)
std::vector<std::pair<size_t, size_t>> chunkify(size_t len, size_t min_per_chunk) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t chunk_count = len / min_per_chunk;
  if (chunk_count <= 1) {
    out.push_back({0, len});
    return out;
  }
  size_t per = (len + chunk_count - 1) / chunk_count;
  for (size_t i = 0; i < len; i += per) out.push_back({i, std::min(len, i + per)});
  return out;
}

}  // namespace

// A device-resident package of signature sets (inputs + randomizers), read-only to kernels.
struct lsg_staged {
  DevBuf d_sig, d_siglen, d_msg, d_msgoff, d_msglen, d_pk, d_pklen, d_rnd;
  HostBuf h_arena;  // pinned staging copy
  size_t n_sets = 0, n_pks = 0;
  std::vector<uint32_t> pk_cnt;
  std::vector<std::vector<int32_t>> sets_pks;  // per set: indices of its pubkeys
  std::vector<uint64_t> rnd;                   // per set: the RLC randomizer r_i
  mutable MsmPlan msm;                         // bucket plan of the last grouping submitted
  // pubkey-aggregation tree plan of sets_pks, built and uploaded by the first submission
  mutable TreePlan pk_plan;
  mutable DevBuf d_pk_plan;
  mutable bool pk_plan_valid = false;
};

namespace {

enum SlotKind { SLOT_FREE = 0, SLOT_JOBS = 1, SLOT_BATCH = 2, SLOT_FINAL = 3, SLOT_UTIL = 4 };

struct JobsPlan {
  std::vector<size_t> jfirst, jcount;
  std::vector<std::vector<int32_t>> groups;
  std::vector<std::vector<size_t>> group_jobs;
  std::vector<bool> group_is_chunk;
  std::vector<std::vector<size_t>> empty_chunks;
  std::vector<lsg_job_result> results;
  lsg_stats stats;
};

struct Slot {
  lsg_ctx* c = nullptr;
  int index = 0;
  hipStream_t st[2] = {nullptr, nullptr};  // [0] main, [1] side
  bool own_streams = true;
  int cur = 0;
  hipEvent_t ev_in = nullptr, ev_sig = nullptr, ev_grp = nullptr, ev_done = nullptr;
  lsg_staged own;                  // inputs staged by submit calls
  const lsg_staged* in = nullptr;  // inputs of the running package
  DevBuf d_dst;
  // per-set / per-pk state
  DevBuf d_ub, d_sigaff, d_siginf, d_seterr, d_pkp, d_pkerr, d_agg, d_P, d_pinf, d_H, d_hinf, d_rs, d_fall;
  // groups, reductions, outputs
  DevBuf d_S, d_F, d_verdict, d_blob, d_aux;
  DevBuf d_Sb, d_fgb, d_Fb;  // canonical blobs handed to / from the row-backend group stages
  // batched inversions: projective pubkeys and their Z; hash_to_field elements, SSWU norms,
  // projective hashes and their norms; inverses; product-tree scratch per stream
  DevBuf d_Pp, d_zP, d_zPi, d_U, d_nrm, d_nrmi, d_Hp, d_zN, d_zNi;
  DevBuf binv_lv[2], binv_iv[2];
  // tree scratch: [0] Fp12 products (main stream), [1] pubkey aggregation, [2] signature sums,
  // [3] [4] MSM buckets and bit sums (side stream)
  TreeSlot tree[5];
  DevBuf d_lines;        // split Miller loop: ML_STEPS unevaluated lines per set
  DevBuf d_bkt, d_bits;  // MSM buckets and per-bit partial sums (lane-form G2, projective)
  bool msm = false;      // signature sums of this package by bucket MSM (else per-set [r_i] sig_i)
  // Miller items: <= LSG_MILLER_K consecutive sets of one job share one multi-Miller loop
  std::vector<int32_t> item_host;  // [first..., count...]
  std::vector<int32_t> set_item;   // set -> item
  size_t n_items = 0;
  DevBuf d_items;
  HostBuf h_err, h_pinf, h_pkerr, h_verdict, h_blob;  // pinned result mirrors
  size_t n_verdicts = 0;
  size_t n_partials = 1;  // batch tickets: Miller partials produced
  std::vector<Timer> timers;
  size_t ntimers = 0;
  // ticket state
  int kind = SLOT_FREE;
  uint64_t serial = 0;
  JobsPlan plan;
};

}  // namespace

struct lsg_ctx {
  int device = 0;
  std::mutex mu;
  std::string err;
  hipStream_t s_final = nullptr;  // utility calls
  hipStream_t s_fe[LSG_FE_STREAMS] = {};  // final exponentiations (entries share these round-robin)
  Slot slots[LSG_SLOTS];
  Slot finals[LSG_FINALS];
  Slot util;
  uint64_t next_serial = 1;
  const Slot* last = nullptr;  // slot whose timers lsg_last_kernel_times reports
  // validator pubkey table (lsg_pubkey_table_set): projective lane-form keys + validity bytes
  DevBuf d_pktab, d_pktab_ok;
  size_t pktab_n = 0, pktab_cap = 0;
};

namespace {

int fail(Slot* s, const char* what, hipError_t e) {
  s->c->err = std::string(what) + ": " + hipGetErrorString(e);
  return LSG_ERR_DEVICE;
}
int fail_c(lsg_ctx* c, const char* what, hipError_t e) {
  c->err = std::string(what) + ": " + hipGetErrorString(e);
  return LSG_ERR_DEVICE;
}

#define LSG_HIP(s, call)                               \
  do {                                                 \
    hipError_t _e = (call);                            \
    if (_e != hipSuccess) return fail((s), #call, _e); \
  } while (0)
#define LSG_HIPC(c, call)                                \
  do {                                                   \
    hipError_t _e = (call);                              \
    if (_e != hipSuccess) return fail_c((c), #call, _e); \
  } while (0)

int ensure(Slot* s, DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 64;
  if (b.cap >= bytes) return LSG_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t cap = std::max(bytes + bytes / 4, (size_t)4096);
  hipError_t e = hipMalloc(&b.p, cap);
  if (e != hipSuccess) return fail(s, "hipMalloc", e);
  b.cap = cap;
  return LSG_OK;
}

int ensure_host(Slot* s, HostBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 64;
  if (b.cap >= bytes) return LSG_OK;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t cap = std::max(bytes + bytes / 4, (size_t)4096);
  hipError_t e = hipHostMalloc(&b.p, cap, hipHostMallocDefault);
  if (e != hipSuccess) return fail(s, "hipHostMalloc", e);
  b.cap = cap;
  return LSG_OK;
}

template <class T>
T* P_(const DevBuf& b) {
  return (T*)b.p;
}
template <class T>
T* H_(const HostBuf& b) {
  return (T*)b.p;
}

int lane_blocks(size_t items) { return (int)((items + LSG_ITEMS_PER_BLOCK - 1) / LSG_ITEMS_PER_BLOCK); }

inline hipStream_t S_(Slot* s) { return s->st[s->cur]; }

void timer_reset(Slot* s) {
  s->ntimers = 0;
  s->cur = 0;
}

void timer_begin(Slot* s, const char* name) {
  if (s->ntimers >= s->timers.size()) {
    Timer t;
    (void)hipEventCreate(&t.a);
    (void)hipEventCreate(&t.b);
    s->timers.push_back(t);
  }
  Timer& t = s->timers[s->ntimers];
  t.name = name;
  (void)hipEventRecord(t.a, S_(s));
}

void timer_end(Slot* s) {
  (void)hipEventRecord(s->timers[s->ntimers].b, S_(s));
  s->ntimers++;
}

#define LAUNCH_T(s, name, kern, grid, tpb, ...)                             \
  do {                                                                      \
    timer_begin((s), name);                                                 \
    hipLaunchKernelGGL(kern, dim3(grid), dim3(tpb), 0, S_(s), __VA_ARGS__); \
    timer_end((s));                                                         \
    hipError_t _le = hipGetLastError();                                     \
    if (_le != hipSuccess) return fail((s), name, _le);                     \
  } while (0)
#define LAUNCH(s, kern, items, ...) LAUNCH_T(s, #kern, kern, lane_blocks(items), LSG_TPB, __VA_ARGS__)

// a row-backend stage (lsg_serial.hip) on the slot's current stream, timed like LAUNCH_T
#define LAUNCH_ROW(s, name, call)                     \
  do {                                                \
    timer_begin((s), name);                           \
    hipError_t _le = (call);                          \
    timer_end((s));                                   \
    if (_le != hipSuccess) return fail((s), name, _le); \
  } while (0)

int slot_create(lsg_ctx* c, Slot* s, int index, hipStream_t shared) {
  s->c = c;
  s->index = index;
  if (shared) {
    s->st[0] = s->st[1] = shared;
    s->own_streams = false;
  } else {
    for (int k = 0; k < 2; k++) LSG_HIP(s, hipStreamCreateWithFlags(&s->st[k], hipStreamNonBlocking));
  }
  hipEvent_t* evs[] = {&s->ev_in, &s->ev_sig, &s->ev_grp, &s->ev_done};
  for (hipEvent_t* e : evs) LSG_HIP(s, hipEventCreateWithFlags(e, hipEventDisableTiming));
  int rc = ensure(s, s->d_dst, 256);
  if (rc) return rc;
  LSG_HIP(s, hipMemcpy(s->d_dst.p, DST_POP, DST_POP_LEN, hipMemcpyHostToDevice));
  return LSG_OK;
}

void free_dev(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}
void free_host(HostBuf& b) {
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}

void staged_free(lsg_staged* in) {
  DevBuf* bufs[] = {&in->d_sig, &in->d_siglen, &in->d_msg, &in->d_msgoff, &in->d_msglen, &in->d_pk, &in->d_pklen, &in->d_rnd};
  for (DevBuf* b : bufs) free_dev(*b);
  free_dev(in->d_pk_plan);
  in->pk_plan_valid = false;
  free_dev(in->msm.d_buckets);
  free_dev(in->msm.d_bits);
  in->msm.valid = false;
  free_host(in->h_arena);
}

void slot_destroy(Slot* s) {
  if (!s->c) return;
  for (int k = 0; k < 2; k++)
    if (s->st[k]) (void)hipStreamSynchronize(s->st[k]);
  staged_free(&s->own);
  DevBuf* bufs[] = {&s->d_dst, &s->d_ub, &s->d_sigaff, &s->d_siginf, &s->d_seterr, &s->d_pkp, &s->d_pkerr,
                    &s->d_agg, &s->d_P,  &s->d_pinf,   &s->d_H,      &s->d_hinf,   &s->d_rs,  &s->d_fall,
                    &s->d_S,   &s->d_F,  &s->d_verdict, &s->d_blob,  &s->d_aux, &s->d_Sb, &s->d_fgb, &s->d_Fb,
                    &s->d_Pp,  &s->d_zP, &s->d_zPi, &s->d_U, &s->d_nrm, &s->d_nrmi, &s->d_Hp, &s->d_zN, &s->d_zNi,
                    &s->binv_lv[0], &s->binv_lv[1], &s->binv_iv[0], &s->binv_iv[1], &s->d_bkt, &s->d_bits, &s->d_lines};
  for (DevBuf* b : bufs) free_dev(*b);
  free_dev(s->d_items);
  for (TreeSlot& t : s->tree) {
    free_dev(t.idx);
    free_dev(t.tA);
    free_dev(t.tB);
  }
  HostBuf* hb[] = {&s->h_err, &s->h_pinf, &s->h_pkerr, &s->h_verdict, &s->h_blob};
  for (HostBuf* b : hb) free_host(*b);
  for (Timer& t : s->timers) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  hipEvent_t evs[] = {s->ev_in, s->ev_sig, s->ev_grp, s->ev_done};
  for (hipEvent_t e : evs)
    if (e) (void)hipEventDestroy(e);
  if (s->own_streams)
    for (int k = 0; k < 2; k++)
      if (s->st[k]) (void)hipStreamDestroy(s->st[k]);
  s->c = nullptr;
}

// ---- stage a package of sets: host layout in a pinned arena, async copies on `stream`
int stage_sets(Slot* s, lsg_staged* in, const lsg_set* const* sets, size_t n, uint64_t seed, bool scale,
               hipStream_t stream) {
  size_t npk = 0, msg_total = 0;
  for (size_t i = 0; i < n; i++) {
    npk += sets[i]->n_pks;
    msg_total += sets[i]->msg_len;
  }
  in->n_sets = n;
  in->n_pks = npk;
  size_t nn = std::max(n, (size_t)1), np = std::max(npk, (size_t)1);
  // arena layout (all offsets 8-byte aligned)
  auto al = [](size_t x) { return (x + 7) & ~(size_t)7; };
  size_t o_sig = 0, o_siglen = al(o_sig + 192 * nn), o_msgoff = al(o_siglen + 4 * nn), o_msglen = al(o_msgoff + 4 * nn),
         o_pklen = al(o_msglen + 4 * nn), o_rnd = al(o_pklen + 4 * np), o_pk = al(o_rnd + 8 * nn),
         o_msg = al(o_pk + 96 * np), total = al(o_msg + std::max(msg_total, (size_t)1));
  int rc;
  if ((rc = ensure_host(s, in->h_arena, total))) return rc;
  uint8_t* A = H_<uint8_t>(in->h_arena);
  memset(A + o_sig, 0, 192 * nn);
  memset(A + o_pk, 0, 96 * np);
  uint32_t* siglen = (uint32_t*)(A + o_siglen);
  uint32_t* msgoff = (uint32_t*)(A + o_msgoff);
  uint32_t* msglen = (uint32_t*)(A + o_msglen);
  uint32_t* pklen = (uint32_t*)(A + o_pklen);
  uint64_t* rnd = (uint64_t*)(A + o_rnd);
  siglen[0] = msgoff[0] = msglen[0] = pklen[0] = 0;
  rnd[0] = 0;
  in->pk_cnt.assign(n, 0);
  in->sets_pks.assign(n, {});
  in->rnd.assign(n, 0);
  in->msm.valid = false;
  in->pk_plan_valid = false;
  size_t mo = 0, po = 0;
  uint64_t sd = seed;
  FILE* ur = nullptr;
  if (scale && seed == 0) ur = fopen("/dev/urandom", "rb");
  for (size_t i = 0; i < n; i++) {
    const lsg_set* q = sets[i];
    siglen[i] = q->sig_len;
    if ((q->sig_len == 96 || q->sig_len == 192) && q->sig) memcpy(A + o_sig + 192 * i, q->sig, q->sig_len);
    msgoff[i] = (uint32_t)mo;
    msglen[i] = q->msg_len;
    if (q->msg_len) memcpy(A + o_msg + mo, q->msg, q->msg_len);
    mo += q->msg_len;
    in->pk_cnt[i] = q->n_pks;
    // a set without keys points at pk 0 and is reported as an empty aggregate
    for (uint32_t k = 0; k < q->n_pks; k++) {
      pklen[po] = q->pk_len;
      if (q->pk_len == 48 || q->pk_len == 96 || q->pk_len == LSG_PK_INDEX)
        memcpy(A + o_pk + 96 * po, q->pks + (size_t)q->pk_len * k, q->pk_len);
      in->sets_pks[i].push_back((int32_t)po);
      po++;
    }
    if (in->sets_pks[i].empty()) in->sets_pks[i].push_back(0);
    uint64_t r = 0;
    if (scale) {
      do {
        if (ur) {
          if (fread(&r, 8, 1, ur) != 1) r = splitmix64(sd) ^ now_ns();
        } else {
          r = splitmix64(sd);
        }
      } while (r == 0);
    }
    rnd[i] = r;
    in->rnd[i] = r;
  }
  if (ur) fclose(ur);
  if ((rc = ensure(s, in->d_sig, 192 * nn)) || (rc = ensure(s, in->d_siglen, 4 * nn)) ||
      (rc = ensure(s, in->d_msg, std::max(msg_total, (size_t)1))) || (rc = ensure(s, in->d_msgoff, 4 * nn)) ||
      (rc = ensure(s, in->d_msglen, 4 * nn)) || (rc = ensure(s, in->d_pk, 96 * np)) ||
      (rc = ensure(s, in->d_pklen, 4 * np)) || (rc = ensure(s, in->d_rnd, 8 * nn)))
    return rc;
  struct {
    DevBuf* d;
    size_t off, len;
  } cp[] = {{&in->d_sig, o_sig, 192 * nn},      {&in->d_siglen, o_siglen, 4 * nn}, {&in->d_msg, o_msg, std::max(msg_total, (size_t)1)},
            {&in->d_msgoff, o_msgoff, 4 * nn}, {&in->d_msglen, o_msglen, 4 * nn}, {&in->d_pk, o_pk, 96 * np},
            {&in->d_pklen, o_pklen, 4 * np},   {&in->d_rnd, o_rnd, 8 * nn}};
  for (auto& x : cp) LSG_HIP(s, hipMemcpyAsync(x.d->p, A + x.off, x.len, hipMemcpyHostToDevice, stream));
  return LSG_OK;
}

// per-set device state for the slot's current package
int size_state(Slot* s, size_t groups) {
  const lsg_staged* in = s->in;
  size_t nn = std::max(in->n_sets, (size_t)1), np = std::max(in->n_pks, (size_t)1);
  int rc;
  if ((rc = ensure(s, s->d_ub, 256 * nn)) || (rc = ensure(s, s->d_sigaff, 4 * W_G2A * nn)) ||
      (rc = ensure(s, s->d_siginf, nn)) || (rc = ensure(s, s->d_seterr, 4 * nn)) ||
      (rc = ensure(s, s->d_pkp, 4 * W_G1P * np)) || (rc = ensure(s, s->d_pkerr, 4 * np)) ||
      (rc = ensure(s, s->d_agg, 4 * W_G1P * nn)) || (rc = ensure(s, s->d_P, 4 * W_G1A * nn)) ||
      (rc = ensure(s, s->d_pinf, nn)) || (rc = ensure(s, s->d_H, 4 * W_G2A * nn)) || (rc = ensure(s, s->d_hinf, nn)) ||
      (rc = ensure(s, s->d_rs, 4 * W_G2P * nn)) || (rc = ensure(s, s->d_fall, 4 * W_F12 * (nn + groups))) ||
      (rc = ensure(s, s->d_S, 4 * W_G2P * std::max(groups, (size_t)1))) ||
      (rc = ensure(s, s->d_F, 4 * W_F12 * std::max(groups, (size_t)1))) ||
      (rc = ensure(s, s->d_verdict, 4 * std::max(groups, (size_t)1))) || (rc = ensure(s, s->d_blob, 576)) ||
      (rc = ensure_host(s, s->h_err, 4 * nn)) || (rc = ensure_host(s, s->h_pinf, nn)) ||
      (rc = ensure_host(s, s->h_pkerr, 4 * np)) || (rc = ensure_host(s, s->h_verdict, 4 * std::max(groups, (size_t)1))) ||
      (rc = ensure_host(s, s->h_blob, 576)))
    return rc;
  const size_t WF = lane_words<fp_t>();
  if ((rc = ensure(s, s->d_Pp, 4 * W_G1P * nn)) || (rc = ensure(s, s->d_zP, 4 * WF * nn)) ||
      (rc = ensure(s, s->d_zPi, 4 * WF * nn)) || (rc = ensure(s, s->d_U, 4 * lane_words<h2c_u_t>() * nn)) ||
      (rc = ensure(s, s->d_nrm, 4 * WF * 2 * nn)) || (rc = ensure(s, s->d_nrmi, 4 * WF * 2 * nn)) ||
      (rc = ensure(s, s->d_Hp, 4 * W_G2P * nn)) || (rc = ensure(s, s->d_zN, 4 * WF * nn)) ||
      (rc = ensure(s, s->d_zNi, 4 * WF * nn)))
    return rc;
  return LSG_OK;
}

// out[i] = 1 / v[i] (0 for v[i] = 0) for n lane-form Fp values, on the slot's current stream:
// a product tree up, one inversion at the root, products back down (Montgomery's trick).
// ws selects the per-stream tree scratch.
int batch_inv(Slot* s, int ws, const char* name, const uint32_t* v, size_t n, uint32_t* out) {
  if (n == 0) return LSG_OK;
  const size_t WF = lane_words<fp_t>();
  std::vector<size_t> sz{n}, off{0};
  size_t total = 0;
  do {
    size_t m = (sz.back() + 1) / 2;
    off.push_back(total);
    sz.push_back(m);
    total += m;
  } while (sz.back() > 1);
  int rc;
  if ((rc = ensure(s, s->binv_lv[ws], 4 * WF * total)) || (rc = ensure(s, s->binv_iv[ws], 4 * WF * total))) return rc;
  uint32_t* lv = P_<uint32_t>(s->binv_lv[ws]);
  uint32_t* iv = P_<uint32_t>(s->binv_iv[ws]);
  const size_t L = sz.size() - 1;  // levels above the inputs
  auto lvl = [&](size_t k) { return k == 0 ? (uint32_t*)v : lv + WF * off[k]; };
  for (size_t k = 1; k <= L; k++)
    LAUNCH_T(s, name, k_binv_up, lane_blocks(sz[k]), LSG_TPB, (int)sz[k], (int)sz[k - 1], k == 1 ? 1 : 0, lvl(k - 1),
             lvl(k));
  LAUNCH_T(s, name, k_binv_root, 1, LSG_TPB, lvl(L), iv + WF * off[L]);
  for (size_t k = L; k >= 1; k--)
    LAUNCH_T(s, name, k_binv_down, lane_blocks(sz[k - 1]), LSG_TPB, (int)sz[k - 1], k == 1 ? 1 : 0, lvl(k - 1),
             iv + WF * off[k], k == 1 ? out : iv + WF * off[k - 1]);
  return LSG_OK;
}

// hash_to_G2 of the slot's n expanded messages (d_ub) into d_H / d_hinf, on the current
// stream, with the field inversions batched over the n sets
int launch_hash(Slot* s, int n) {
  int rc;
  LAUNCH(s, k_h2c_prep, n, n, P_<uint8_t>(s->d_ub), P_<uint32_t>(s->d_U), P_<uint32_t>(s->d_nrm));
  if ((rc = batch_inv(s, 0, "binv_sswu", P_<uint32_t>(s->d_nrm), 2 * (size_t)n, P_<uint32_t>(s->d_nrmi)))) return rc;
  LAUNCH(s, k_h2c_map, n, n, P_<uint32_t>(s->d_U), P_<uint32_t>(s->d_nrmi), P_<uint32_t>(s->d_Hp),
         P_<uint32_t>(s->d_zN), P_<uint8_t>(s->d_hinf));
#if LSG_H2C_SPLIT
  LAUNCH(s, k_h2c_clear, n, n, P_<uint32_t>(s->d_Hp), P_<uint32_t>(s->d_zN), P_<uint8_t>(s->d_hinf));
#endif
  if ((rc = batch_inv(s, 0, "binv_hash", P_<uint32_t>(s->d_zN), (size_t)n, P_<uint32_t>(s->d_zNi)))) return rc;
  LAUNCH(s, k_h2c_affine, n, n, P_<uint32_t>(s->d_Hp), P_<uint32_t>(s->d_zNi), P_<uint8_t>(s->d_hinf),
         P_<uint32_t>(s->d_H));
  return LSG_OK;
}

// Segmented pairwise reduction of lane-form values on the current stream: for each group,
// combine the slots groups[g] of `src` (OP 0: G1 add, 1: G2 add, 2: Fp12 mul) into dense
// out[g].  All levels' index pairs are built on the host and uploaded once; each level is
// one launch over all pairs of all groups.  `ts` selects private scratch so that trees on
// different streams can run concurrently.
// Runs a planned reduction (plan_tree) on the current stream: each level is one launch over
// all pairs of all groups; d_idx holds the plan's index pairs on the device.
template <int OP>
int run_tree(Slot* s, int ts, const char* name, const TreePlan& P, const int32_t* d_idx, const uint32_t* src,
             uint32_t* out) {
  TreeSlot& T = s->tree[ts];
  size_t W = OP == 0 ? W_G1P : (OP == 1 ? W_G2P : W_F12);
  int rc;
  if ((rc = ensure(s, T.tA, 4 * W * P.max_level)) || (rc = ensure(s, T.tB, 4 * W * P.max_level))) return rc;
  const uint32_t* in = src;
  uint32_t* bufs[2] = {P_<uint32_t>(T.tA), P_<uint32_t>(T.tB)};
  for (size_t L = 0; L < P.levels.size(); L++) {
    size_t off = P.levels[L].first, cnt = P.levels[L].second;
    bool last = L + 1 == P.levels.size();
    uint32_t* dst = last ? out : bufs[L & 1];
    const int32_t* ia = d_idx + off;
    LAUNCH_T(s, name, k_tree_level<OP>, lane_blocks(cnt), LSG_TPB, (int)cnt, ia, ia + cnt, in, dst);
    in = dst;
  }
  return LSG_OK;
}

// Segmented pairwise reduction of lane-form values on the current stream: for each group,
// combine the slots groups[g] of `src` (OP 0: G1 add, 1: G2 add, 2: Fp12 mul) into dense
// out[g].  All levels' index pairs are built on the host and uploaded once; each level is
// one launch over all pairs of all groups.  `ts` selects private scratch so that trees on
// different streams can run concurrently.
template <int OP>
int tree_reduce(Slot* s, int ts, const char* name, const uint32_t* src,
                const std::vector<std::vector<int32_t>>& groups, uint32_t* out) {
  if (groups.empty()) return LSG_OK;
  TreeSlot& T = s->tree[ts];
  TreePlan P = plan_tree(groups);
  T.host.swap(P.idx);  // the async upload reads it; kept until the slot's next reduction
  int rc;
  if ((rc = ensure(s, T.idx, 4 * T.host.size()))) return rc;
  LSG_HIP(s, hipMemcpyAsync(T.idx.p, T.host.data(), 4 * T.host.size(), hipMemcpyHostToDevice, S_(s)));
  return run_tree<OP>(s, ts, name, P, P_<int32_t>(T.idx), src, out);
}

// Minimum RLC group size for the bucket MSM (env LSG_MSM_MIN_GROUP, read per submission):
// below ~150 sets the fixed cost of 2040 buckets and 64 bit sums per group exceeds the
// per-set scalar multiplications it replaces.
size_t msm_min_group() {
  const char* e = getenv("LSG_MSM_MIN_GROUP");
  long v = e ? atol(e) : 256;
  return v < 1 ? 1 : (size_t)v;
}

// The staged package's MSM plan for groups of group_size consecutive sets (built once per
// package and grouping; the device index copies are shared by every ticket that uses it)
int msm_plan(Slot* s, const lsg_staged* in, size_t group_size, size_t ng) {
  MsmPlan& M = in->msm;
  if (M.valid && M.group_size == group_size && M.ng == ng) return LSG_OK;
  M.valid = false;
  const size_t n = in->n_sets;
  const size_t nb = (size_t)MSM_WINDOWS * MSM_DIGITS;
  std::vector<std::vector<int32_t>> buckets(ng * nb), bits(ng * MSM_BITS);
  for (size_t i = 0; i < n; i++) {
    size_t g = i / group_size;
    uint64_t r = in->rnd[i];
    for (int w = 0; w < MSM_WINDOWS; w++) {
      uint32_t d = (uint32_t)(r >> (8 * w)) & 255u;
      if (d) buckets[g * nb + (size_t)w * MSM_DIGITS + d - 1].push_back((int32_t)i);
    }
  }
  for (size_t g = 0; g < ng; g++)
    for (int w = 0; w < MSM_WINDOWS; w++)
      for (int j = 0; j < 8; j++)
        for (uint32_t d = 1; d <= 255; d++)
          if ((d >> j) & 1u) bits[g * MSM_BITS + 8 * w + j].push_back((int32_t)(g * nb + (size_t)w * MSM_DIGITS + d - 1));
  M.buckets = plan_tree(buckets);
  M.bits = plan_tree(bits);
  int rc;
  if ((rc = ensure(s, M.d_buckets, 4 * M.buckets.idx.size())) || (rc = ensure(s, M.d_bits, 4 * M.bits.idx.size())))
    return rc;
  LSG_HIP(s, hipMemcpy(M.d_buckets.p, M.buckets.idx.data(), 4 * M.buckets.idx.size(), hipMemcpyHostToDevice));
  LSG_HIP(s, hipMemcpy(M.d_bits.p, M.bits.idx.data(), 4 * M.bits.idx.size(), hipMemcpyHostToDevice));
  M.group_size = group_size;
  M.ng = ng;
  M.valid = true;
  return LSG_OK;
}

// Per-bit sums C_{g,k} (d_bits) of S_g = sum_{i in g} r_i sig_i for the planned groups, from
// the projective sig_i in d_rs (k_sig_proj), on the current stream: bucket tree, bit tree
// (the Horner pass runs on a row, k_row_horner_miller).  About 8 point additions per set (one
// per nonzero window digit) plus ~8.2k per group, against ~60 doublings and 16 additions per
// set for [r_i] sig_i.
int msm_bit_sums(Slot* s, const MsmPlan& M) {
  const size_t ng = M.ng;
  int rc;
  if ((rc = ensure(s, s->d_bkt, 4 * W_G2P * ng * MSM_WINDOWS * MSM_DIGITS)) ||
      (rc = ensure(s, s->d_bits, 4 * W_G2P * ng * MSM_BITS)))
    return rc;
  if ((rc = run_tree<1>(s, 3, "msm_buckets", M.buckets, P_<int32_t>(M.d_buckets), P_<uint32_t>(s->d_rs),
                        P_<uint32_t>(s->d_bkt))))
    return rc;
  return run_tree<1>(s, 4, "msm_bits", M.bits, P_<int32_t>(M.d_bits), P_<uint32_t>(s->d_bkt), P_<uint32_t>(s->d_bits));
}

constexpr int LSG_MILLER_KMAX = 4;  // pairs per multi-Miller item: 1, 2 or 4 (env LSG_MILLER_K)
int miller_k() {
  static int k = [] {
    const char* e = getenv("LSG_MILLER_K");
    // K=4 since the tower is inlined: 2.45M vs 2.35M sets/s at 12x3 (profiles/r01_inline_ab.txt);
    // before, with Fp12 stack frames, K=2 was best (profiles/r01_bench_sweeps.txt)
    int v = e ? atoi(e) : 4;
    return (v == 1 || v == 2 || v == 4) ? v : 4;
  }();
  return k;
}

// Miller loop as two kernels (k_miller_lines + k_miller_accum, default) or one
// (k_miller_multi): env LSG_MILLER_SPLIT=0 selects the fused kernel (A/B)
bool miller_split() {
  static bool v = [] {
    const char* e = getenv("LSG_MILLER_SPLIT");
    return !(e && atoi(e) == 0);
  }();
  return v;
}

// Items of <= LSG_MILLER_K consecutive sets that never cross a range (a job): per-job Miller
// products, needed by the per-job retry, stay products of whole items.
void plan_items(Slot* s, const std::vector<std::pair<size_t, size_t>>& ranges) {
  std::vector<int32_t> first, cnt;
  s->set_item.assign(s->in->n_sets, 0);
  for (auto& r : ranges)
    for (size_t i = r.first; i < r.second; i += (size_t)miller_k()) {
      size_t c = std::min((size_t)miller_k(), r.second - i);
      for (size_t k = 0; k < c; k++) s->set_item[i + k] = (int32_t)first.size();
      first.push_back((int32_t)i);
      cnt.push_back((int32_t)c);
    }
  s->n_items = first.size();
  s->item_host = first;
  s->item_host.insert(s->item_host.end(), cnt.begin(), cnt.end());
}

// set-index groups -> item-index groups (every group is a union of whole jobs)
std::vector<std::vector<int32_t>> item_groups(const Slot* s, const std::vector<std::vector<int32_t>>& groups) {
  std::vector<std::vector<int32_t>> out(groups.size());
  for (size_t g = 0; g < groups.size(); g++) {
    int32_t last = -1;
    for (int32_t i : groups[g]) {
      int32_t it = s->set_item[(size_t)i];
      if (it != last) out[g].push_back(it);
      last = it;
    }
  }
  return out;
}

// Per-set stages (no host synchronisation):
//   side: pubkeys -> aggregation tree -> [r_i] scaling -> signature decode -> subgroup
//         check (event ev_sig) -> [r_i] sig_i
//   main: expand_message -> hash_to_G2 -> wait ev_sig -> Miller loops f_i
// f_i is written to d_fall[0..n); size_state reserved n + groups slots.
int launch_set_stages(Slot* s) {
  const lsg_staged* in = s->in;
  int n = (int)in->n_sets, np = (int)in->n_pks;
  if (n == 0) return LSG_OK;
  LSG_HIP(s, hipEventRecord(s->ev_in, s->st[0]));
  s->cur = 1;
  LSG_HIP(s, hipStreamWaitEvent(s->st[1], s->ev_in, 0));
  if (np > 0) {
    LAUNCH(s, k_pk_decode, np, np, P_<uint8_t>(in->d_pk), P_<uint32_t>(in->d_pklen), P_<uint32_t>(s->d_pkp),
           P_<int32_t>(s->d_pkerr), P_<uint32_t>(s->c->d_pktab), P_<uint8_t>(s->c->d_pktab_ok),
           (uint32_t)s->c->pktab_n);
    // the package's aggregation plan is built once (an aggregate-heavy package has ~450 keys
    // per set) and reused by every ticket that submits it
    if (!in->pk_plan_valid) {
      in->pk_plan = plan_tree(in->sets_pks);
      int rc = ensure(s, in->d_pk_plan, 4 * in->pk_plan.idx.size());
      if (rc) return rc;
      // synchronous: other slots may submit the same package before this stream runs
      LSG_HIP(s, hipMemcpy(in->d_pk_plan.p, in->pk_plan.idx.data(), 4 * in->pk_plan.idx.size(),
                           hipMemcpyHostToDevice));
      in->pk_plan_valid = true;
    }
    int rc = run_tree<0>(s, 1, "tree_g1_aggregate", in->pk_plan, P_<int32_t>(in->d_pk_plan), P_<uint32_t>(s->d_pkp),
                         P_<uint32_t>(s->d_agg));
    if (rc) return rc;
  }
  LAUNCH(s, k_pk_scale, n, n, P_<uint32_t>(s->d_agg), P_<uint64_t>(in->d_rnd), P_<uint32_t>(s->d_Pp),
         P_<uint32_t>(s->d_zP), P_<uint8_t>(s->d_pinf));
  {
    int rc = batch_inv(s, 1, "binv_pk", P_<uint32_t>(s->d_zP), (size_t)n, P_<uint32_t>(s->d_zPi));
    if (rc) return rc;
  }
  LAUNCH(s, k_pk_affine, n, n, P_<uint32_t>(s->d_Pp), P_<uint32_t>(s->d_zPi), P_<uint32_t>(s->d_P));
  LAUNCH(s, k_sig_decode, n, n, P_<uint8_t>(in->d_sig), P_<uint32_t>(in->d_siglen), P_<uint32_t>(s->d_sigaff),
         P_<uint8_t>(s->d_siginf), P_<int32_t>(s->d_seterr));
  LAUNCH(s, k_sig_subgroup, n, n, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf), P_<int32_t>(s->d_seterr));
  LSG_HIP(s, hipEventRecord(s->ev_sig, s->st[1]));  // pubkeys scaled, signature errors known
  if (s->msm)  // the groups' sums come from the bucket MSM over the unscaled points
    LAUNCH(s, k_sig_proj, n, n, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf), P_<int32_t>(s->d_seterr),
           P_<uint32_t>(s->d_rs));
  else
    LAUNCH(s, k_sig_scale, n, n, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf), P_<int32_t>(s->d_seterr),
           P_<uint64_t>(in->d_rnd), P_<uint32_t>(s->d_rs));
  s->cur = 0;
  LAUNCH_T(s, "k_expand_msg", k_expand_msg, (n + 63) / 64, 64, n, P_<uint8_t>(in->d_msg), P_<uint32_t>(in->d_msgoff),
           P_<uint32_t>(in->d_msglen), P_<uint8_t>(s->d_dst), DST_POP_LEN, P_<uint8_t>(s->d_ub));
  {
    int rc = launch_hash(s, n);
    if (rc) return rc;
  }
  const bool split = miller_split();
  if (split) {  // the G2 half needs only the hashes
    int rc = ensure(s, s->d_lines, 4 * (size_t)ML_STEPS * W_LINE * LSG_GROUP * (size_t)n);
    if (rc) return rc;
    LAUNCH(s, k_miller_lines, n, n, P_<uint32_t>(s->d_H), P_<uint32_t>(s->d_lines));
  }
  LSG_HIP(s, hipStreamWaitEvent(s->st[0], s->ev_sig, 0));
  int ni = (int)s->n_items;
  if (ni <= 0 || s->item_host.size() != 2 * (size_t)ni) {
    s->c->err = "internal: Miller items not planned";
    return LSG_ERR_INVALID_ARG;
  }
  int rc2;
  if ((rc2 = ensure(s, s->d_items, 4 * s->item_host.size()))) return rc2;
  LSG_HIP(s, hipMemcpyAsync(s->d_items.p, s->item_host.data(), 4 * s->item_host.size(), hipMemcpyHostToDevice,
                            s->st[0]));
  const int32_t* items = P_<int32_t>(s->d_items);
  const uint32_t* mP = P_<uint32_t>(s->d_P);
  const uint32_t* mH = P_<uint32_t>(s->d_H);
  const uint8_t* mpi = P_<uint8_t>(s->d_pinf);
  const uint8_t* mhi = P_<uint8_t>(s->d_hinf);
  const int32_t* merr = P_<int32_t>(s->d_seterr);
  uint32_t* mf = P_<uint32_t>(s->d_fall);
  if (split) {
    const uint32_t* ml = P_<uint32_t>(s->d_lines);
    if (miller_k() == 1)
      LAUNCH_T(s, "k_miller_accum", k_miller_accum<1>, lane_blocks(ni), LSG_TPB, ni, items, items + ni, mP, mpi, mhi,
               merr, n, ml, mf);
    else if (miller_k() == 2)
      LAUNCH_T(s, "k_miller_accum", k_miller_accum<2>, lane_blocks(ni), LSG_TPB, ni, items, items + ni, mP, mpi, mhi,
               merr, n, ml, mf);
    else
      LAUNCH_T(s, "k_miller_accum", k_miller_accum<4>, lane_blocks(ni), LSG_TPB, ni, items, items + ni, mP, mpi, mhi,
               merr, n, ml, mf);
    return LSG_OK;
  }
  if (miller_k() == 1)
    LAUNCH_T(s, "k_miller_multi", k_miller_multi<1>, lane_blocks(ni), LSG_TPB, ni, items, items + ni, mP, mpi, mH, mhi,
             merr, mf);
  else if (miller_k() == 2)
    LAUNCH_T(s, "k_miller_multi", k_miller_multi<2>, lane_blocks(ni), LSG_TPB, ni, items, items + ni, mP, mpi, mH, mhi,
             merr, mf);
  else
    LAUNCH_T(s, "k_miller_multi", k_miller_multi<4>, lane_blocks(ni), LSG_TPB, ni, items, items + ni, mP, mpi, mH, mhi,
             merr, mf);
  return LSG_OK;
}

// Group stages (no host synchronisation): the side stream sums [r_i] sig_i per group and
// runs the signature Miller loop; the main stream multiplies each group's f_i with it and,
// if fe, runs the final exponentiation into d_verdict (else leaves the products in d_F).
// Sets with errors contribute identities (f_i = 1, [r_i] sig_i = O), so groups may contain
// them; the host discards such groups' verdicts.
int launch_groups(Slot* s, const std::vector<std::vector<int32_t>>& groups, bool fe) {
  size_t ng = groups.size();
  if (ng == 0) return LSG_OK;
  size_t n = s->n_items;  // Miller items occupy d_fall[0..n_items)
  if (s->d_fall.cap < 4 * W_F12 * (n + ng) || s->d_S.cap < 4 * W_G2P * ng || s->d_F.cap < 4 * W_F12 * ng ||
      s->d_verdict.cap < 4 * ng) {
    s->c->err = "internal: group buffers too small";
    return LSG_ERR_INVALID_ARG;
  }
  int rc;
  if ((rc = ensure(s, s->d_Sb, 288 * ng)) || (rc = ensure(s, s->d_fgb, 576 * ng)) || (rc = ensure(s, s->d_Fb, 576 * ng)))
    return rc;
  s->cur = 1;
  if (s->msm) {  // planned by submit_batch for exactly these groups
    // buckets and per-bit sums on the pair backend, then Horner + ML(-G1, S_g) in one row
    // chain per group (k_row_horner_miller), written at d_fall slot n_items + g
    if ((rc = msm_bit_sums(s, s->in->msm))) return rc;
    if ((rc = ensure(s, s->d_Sb, (size_t)288 * MSM_BITS * ng))) return rc;
    LAUNCH(s, k_g2p_to_canon, (size_t)MSM_BITS * ng, (int)(MSM_BITS * ng), P_<uint32_t>(s->d_bits),
           P_<uint8_t>(s->d_Sb));
    LAUNCH_ROW(s, "k_row_horner_miller",
               lsg_row_horner_miller(S_(s), (int)ng, P_<uint8_t>(s->d_Sb), P_<uint8_t>(s->d_fgb)));
  } else {
    if ((rc = tree_reduce<1>(s, 2, "tree_g2_sigsum", P_<uint32_t>(s->d_rs), groups, P_<uint32_t>(s->d_S))))
      return rc;
    // f_g = ML(-G1, S_g) on the row backend, written at d_fall slot n_items + g
    LAUNCH(s, k_g2p_to_canon, ng, (int)ng, P_<uint32_t>(s->d_S), P_<uint8_t>(s->d_Sb));
    LAUNCH_ROW(s, "k_row_miller_neg_g1",
               lsg_row_miller_neg_g1(S_(s), (int)ng, P_<uint8_t>(s->d_Sb), P_<uint8_t>(s->d_fgb)));
  }
  LAUNCH(s, k_blobs_to_fp12, ng, (int)ng, P_<uint8_t>(s->d_fgb), P_<uint32_t>(s->d_fall) + W_F12 * n);
  LSG_HIP(s, hipEventRecord(s->ev_grp, s->st[1]));
  s->cur = 0;
  LSG_HIP(s, hipStreamWaitEvent(s->st[0], s->ev_grp, 0));
  std::vector<std::vector<int32_t>> fg = item_groups(s, groups);
  for (size_t g = 0; g < ng; g++) fg[g].push_back((int32_t)(n + g));
  if ((rc = tree_reduce<2>(s, 0, "tree_fp12_product", P_<uint32_t>(s->d_fall), fg, P_<uint32_t>(s->d_F)))) return rc;
  if (fe) {
    LAUNCH(s, k_fp12_to_canon, ng, (int)ng, P_<uint32_t>(s->d_F), P_<uint8_t>(s->d_Fb));
    LAUNCH_ROW(s, "k_row_final_exp", lsg_row_final_exp(S_(s), (int)ng, P_<uint8_t>(s->d_Fb), P_<int32_t>(s->d_verdict)));
  }
  return LSG_OK;
}

// enqueue D2H copies of per-set status (and ng verdicts) into the pinned mirrors, then
// record ev_done on the main stream (which has joined the side stream through events)
int launch_readback(Slot* s, bool status, size_t ng) {
  hipStream_t S = s->st[0];
  size_t n = s->in->n_sets, np = s->in->n_pks;
  if (s->own_streams) {  // join the side stream even when no group was launched
    LSG_HIP(s, hipEventRecord(s->ev_grp, s->st[1]));
    LSG_HIP(s, hipStreamWaitEvent(S, s->ev_grp, 0));
  }
  if (status) {
    if (n) {
      LSG_HIP(s, hipMemcpyAsync(s->h_err.p, s->d_seterr.p, 4 * n, hipMemcpyDeviceToHost, S));
      LSG_HIP(s, hipMemcpyAsync(s->h_pinf.p, s->d_pinf.p, n, hipMemcpyDeviceToHost, S));
    }
    if (np) LSG_HIP(s, hipMemcpyAsync(s->h_pkerr.p, s->d_pkerr.p, 4 * np, hipMemcpyDeviceToHost, S));
  }
  s->n_verdicts = ng;
  if (ng) LSG_HIP(s, hipMemcpyAsync(s->h_verdict.p, s->d_verdict.p, 4 * ng, hipMemcpyDeviceToHost, S));
  LSG_HIP(s, hipEventRecord(s->ev_done, S));
  return LSG_OK;
}

struct SetStatus {
  const int32_t* err;    // per set: BLST code (0 ok)
  std::vector<uint8_t> pinf;   // per set: aggregated pk is infinity (2: no keys at all)
  const int32_t* pkerr;  // per pubkey
};

SetStatus read_status(Slot* s) {
  SetStatus ss;
  size_t n = s->in->n_sets;
  ss.err = H_<int32_t>(s->h_err);
  ss.pkerr = H_<int32_t>(s->h_pkerr);
  ss.pinf.assign(H_<uint8_t>(s->h_pinf), H_<uint8_t>(s->h_pinf) + n);
  for (size_t i = 0; i < n; i++)
    if (s->in->pk_cnt[i] == 0) ss.pinf[i] = 2;  // PublicKey.aggregate([]) throws
  return ss;
}

int32_t set_error(const SetStatus& ss, size_t s) {
  if (ss.err[s]) return ss.err[s];
  if (ss.pinf[s] == 2) return LSG_ERR_EMPTY_AGGREGATE;
  return ss.pinf[s] ? LSG_BLST_PK_IS_INFINITY : 0;
}

// Error a job's maybeBatch call would throw, in the reference's order:
// Signature.fromBytes over all sets first (maybeBatch.ts:17-26 map), then
// mul_n_aggregate rejecting an infinite public key (BLST_PK_IS_INFINITY).
int32_t job_error(const SetStatus& ss, size_t first, size_t count) {
  if (count == 0) return LSG_ERR_EMPTY_SET;
  for (size_t k = 0; k < count; k++)
    if (ss.err[first + k]) return ss.err[first + k];
  for (size_t k = 0; k < count; k++)
    if (ss.pinf[first + k]) return set_error(ss, first + k);
  return 0;
}

Slot* free_slot(lsg_ctx* c, Slot* pool, int n) {
  for (int i = 0; i < n; i++)
    if (pool[i].kind == SLOT_FREE) return &pool[i];
  return nullptr;
}

uint64_t make_ticket(lsg_ctx* c, Slot* s, int kind) {
  s->kind = kind;
  s->serial = c->next_serial++;
  return (s->serial << 16) | ((uint64_t)kind << 8) | (uint64_t)s->index;
}

Slot* ticket_slot(lsg_ctx* c, uint64_t t, int kind) {
  int k = (int)((t >> 8) & 255), i = (int)(t & 255);
  if (k != kind) return nullptr;
  Slot* s = nullptr;
  if (kind == SLOT_FINAL) {
    if (i < LSG_FINALS) s = &c->finals[i];
  } else if (i < LSG_SLOTS) {
    s = &c->slots[i];
  }
  if (!s || s->kind != kind || s->serial != (t >> 16)) return nullptr;
  return s;
}

void release(lsg_ctx* c, Slot* s) {
  s->kind = SLOT_FREE;
  c->last = s;
}

}  // namespace

// ---------------------------------------------------------------------------- C ABI
namespace {

void sync_slot(Slot* s) {
  for (int k = 0; k < 2; k++)
    if (s->st[k]) (void)hipStreamSynchronize(s->st[k]);
}

// Phase A of verifyManySignatureSets, launched speculatively: every batchable chunk and
// every non-batchable job gets its group (sum of [r_i] sig_i, Miller product, final
// exponentiation) before the per-set status is known, so a package costs one host
// synchronisation.  The wait applies the reference's verdict rules (worker.ts:51-96).
int submit_jobs(lsg_ctx* c, Slot* s, const lsg_job* jobs, size_t n_jobs, uint64_t seed) {
  JobsPlan& P = s->plan;
  P = JobsPlan();
  memset(&P.stats, 0, sizeof(P.stats));
  P.stats.start_ns = now_ns();
  timer_reset(s);
  std::vector<const lsg_set*> flat;
  P.jfirst.resize(n_jobs);
  P.jcount.resize(n_jobs);
  for (size_t j = 0; j < n_jobs; j++) {
    P.jfirst[j] = flat.size();
    P.jcount[j] = jobs[j].n_sets;
    for (uint32_t k = 0; k < jobs[j].n_sets; k++) flat.push_back(&jobs[j].sets[k]);
  }
  P.results.assign(n_jobs, {LSG_INVALID, 0});
  std::vector<size_t> batchable, nonbatch;
  for (size_t j = 0; j < n_jobs; j++) (jobs[j].flags & LSG_JOB_BATCHABLE ? batchable : nonbatch).push_back(j);
  auto job_group = [&](size_t j) {
    std::vector<int32_t> m;
    for (size_t k = 0; k < P.jcount[j]; k++) m.push_back((int32_t)(P.jfirst[j] + k));
    return m;
  };
  // batchable chunks (worker.ts:51-86) + non-batchable jobs (worker.ts:88-96)
  if (!batchable.empty()) {
    for (auto ch : chunkify(batchable.size(), 16)) {
      std::vector<int32_t> m;
      std::vector<size_t> js;
      for (size_t q = ch.first; q < ch.second; q++) {
        size_t j = batchable[q];
        js.push_back(j);
        std::vector<int32_t> jm = job_group(j);
        m.insert(m.end(), jm.begin(), jm.end());
      }
      if (m.empty()) {
        P.empty_chunks.push_back(js);
        continue;
      }
      P.groups.push_back(m);
      P.group_jobs.push_back(js);
      P.group_is_chunk.push_back(true);
    }
  }
  for (size_t j : nonbatch) {
    if (P.jcount[j] == 0) {
      P.results[j] = {LSG_ERROR, LSG_ERR_EMPTY_SET};
      continue;
    }
    P.groups.push_back(job_group(j));
    P.group_jobs.push_back({j});
    P.group_is_chunk.push_back(false);
  }
  s->in = &s->own;
  s->msm = false;  // job groups are small (<= 128 sets) and are re-summed per job on retry
  int rc;
  if ((rc = stage_sets(s, &s->own, flat.data(), flat.size(), seed, true, s->st[0]))) return rc;
  if ((rc = size_state(s, std::max(P.groups.size(), n_jobs)))) return rc;
  {
    std::vector<std::pair<size_t, size_t>> ranges;
    for (size_t j = 0; j < n_jobs; j++)
      if (P.jcount[j]) ranges.push_back({P.jfirst[j], P.jfirst[j] + P.jcount[j]});
    plan_items(s, ranges);
  }
  if ((rc = launch_set_stages(s))) return rc;
  if ((rc = launch_groups(s, P.groups, true))) return rc;
  return launch_readback(s, true, P.groups.size());
}

int wait_jobs(lsg_ctx* c, Slot* s, lsg_job_result* results, lsg_stats* stats) {
  JobsPlan& P = s->plan;
  LSG_HIP(s, hipEventSynchronize(s->ev_done));
  size_t n_jobs = P.results.size();
  SetStatus ss = read_status(s);
  std::vector<int32_t> verdict(H_<int32_t>(s->h_verdict), H_<int32_t>(s->h_verdict) + P.groups.size());
  P.stats.n_final_exps += (uint32_t)P.groups.size();
  // worker.ts:108-114: deserializeSet runs before anything else; a bad pubkey throws
  // out of verifyManySignatureSets and rejects every job of the package.
  int32_t pkfail = 0;
  for (size_t k = 0; k < s->in->n_pks && !pkfail; k++) pkfail = ss.pkerr[k];
  if (pkfail) {
    for (size_t j = 0; j < n_jobs; j++) P.results[j] = {LSG_ERROR, pkfail};
  } else {
    std::vector<size_t> retry;
    for (auto& js : P.empty_chunks) {
      P.stats.batch_retries++;
      retry.insert(retry.end(), js.begin(), js.end());
    }
    for (size_t g = 0; g < P.groups.size(); g++) {
      if (P.group_is_chunk[g]) {
        bool throws = false;
        for (int32_t x : P.groups[g])
          if (set_error(ss, (size_t)x)) throws = true;
        if (!throws && verdict[g]) {
          for (size_t j : P.group_jobs[g]) {
            P.results[j] = {LSG_VALID, 0};
            P.stats.batch_sigs_success += (uint32_t)P.jcount[j];
          }
        } else {
          P.stats.batch_retries++;
          retry.insert(retry.end(), P.group_jobs[g].begin(), P.group_jobs[g].end());
        }
      } else {
        size_t j = P.group_jobs[g][0];
        int32_t e = job_error(ss, P.jfirst[j], P.jcount[j]);
        P.results[j] = e ? lsg_job_result{LSG_ERROR, e} : lsg_job_result{verdict[g] ? LSG_VALID : LSG_INVALID, 0};
      }
    }
    // Phase B: per-job retry of failed chunks (worker.ts:74-96) on the resident per-set state
    if (!retry.empty()) {
      std::vector<std::vector<int32_t>> g2;
      std::vector<size_t> g2job;
      for (size_t j : retry) {
        int32_t e = job_error(ss, P.jfirst[j], P.jcount[j]);
        if (e) {
          P.results[j] = {LSG_ERROR, e};
        } else {
          std::vector<int32_t> m;
          for (size_t k = 0; k < P.jcount[j]; k++) m.push_back((int32_t)(P.jfirst[j] + k));
          g2.push_back(m);
          g2job.push_back(j);
        }
      }
      int rc;
      if ((rc = launch_groups(s, g2, true))) return rc;
      if ((rc = launch_readback(s, false, g2.size()))) return rc;
      LSG_HIP(s, hipEventSynchronize(s->ev_done));
      P.stats.n_final_exps += (uint32_t)g2.size();
      const int32_t* v2 = H_<int32_t>(s->h_verdict);
      for (size_t g = 0; g < g2.size(); g++) P.results[g2job[g]] = {v2[g] ? LSG_VALID : LSG_INVALID, 0};
    }
  }
  for (size_t j = 0; j < n_jobs; j++) results[j] = P.results[j];
  P.stats.end_ns = now_ns();
  if (stats) *stats = P.stats;
  return LSG_OK;
}

// per-shard Miller product over the slot's inputs (errored sets contribute identities, so
// the partial covers exactly the valid sets; an empty package gives the identity)
// per-group Miller products over the slot's inputs: groups of group_size consecutive sets
// (errored sets contribute identities, so each partial covers exactly its valid sets; an
// empty package gives one identity partial)
int submit_batch(Slot* s, size_t group_size) {
  int rc;
  const size_t n = s->in->n_sets;
  if (group_size == 0 || group_size > n) group_size = std::max(n, (size_t)1);
  size_t ng = std::max((n + group_size - 1) / group_size, (size_t)1);
  if ((rc = size_state(s, ng))) return rc;
  std::vector<std::pair<size_t, size_t>> ranges;
  std::vector<std::vector<int32_t>> groups(ng);
  for (size_t g = 0; g < ng; g++) {
    size_t a = g * group_size, b = std::min(n, a + group_size);
    if (a < b) ranges.push_back({a, b});
    for (size_t i = a; i < b; i++) groups[g].push_back((int32_t)i);
  }
  plan_items(s, ranges);
  s->msm = n > 0 && std::min(group_size, n - (ng - 1) * group_size) >= msm_min_group();
  if (s->msm && (rc = msm_plan(s, s->in, group_size, ng))) return rc;
  if ((rc = launch_set_stages(s))) return rc;
  if ((rc = launch_groups(s, groups, false))) return rc;
  if ((rc = ensure(s, s->d_blob, 576 * ng)) || (rc = ensure_host(s, s->h_blob, 576 * ng))) return rc;
  LAUNCH(s, k_fp12_to_canon, ng, (int)ng, P_<uint32_t>(s->d_F), P_<uint8_t>(s->d_blob));
  LSG_HIP(s, hipMemcpyAsync(s->h_blob.p, s->d_blob.p, 576 * ng, hipMemcpyDeviceToHost, s->st[0]));
  s->n_partials = ng;
  return launch_readback(s, true, 0);
}

int wait_batch(Slot* s, uint8_t* out576, int32_t* set_err, int32_t* any_error) {
  LSG_HIP(s, hipEventSynchronize(s->ev_done));
  memcpy(out576, s->h_blob.p, 576 * s->n_partials);
  SetStatus ss = read_status(s);
  *any_error = 0;
  for (size_t i = 0; i < s->in->n_sets; i++) {
    int32_t e = set_error(ss, i);
    if (set_err) set_err[i] = e;
    if (e) *any_error = 1;
  }
  for (size_t k = 0; k < s->in->n_pks; k++)
    if (ss.pkerr[k]) *any_error = 1;
  return LSG_OK;
}

// ng groups of pg partials each (group g: partials g*pg .. g*pg+pg-1) -> per group the
// product of its partials and one final exponentiation; all groups in one launch per stage
int submit_final(Slot* s, const uint8_t* partials576, size_t ng, size_t pg) {
  timer_reset(s);
  s->n_verdicts = 0;
  int rc;
  const size_t n = ng * pg, np = std::max(n, (size_t)1), gq = std::max(ng, (size_t)1);
  if ((rc = ensure_host(s, s->h_blob, 576 * np)) || (rc = ensure(s, s->d_blob, 576 * np)) ||
      (rc = ensure(s, s->d_aux, 4 * W_F12 * np)) || (rc = ensure(s, s->d_F, 4 * W_F12 * gq)) ||
      (rc = ensure(s, s->d_verdict, 4 * gq)) || (rc = ensure_host(s, s->h_verdict, 4 * gq)))
    return rc;
  if (n) {
    hipStream_t S = s->st[0];
    memcpy(s->h_blob.p, partials576, 576 * n);
    LSG_HIP(s, hipMemcpyAsync(s->d_blob.p, s->h_blob.p, 576 * n, hipMemcpyHostToDevice, S));
    LAUNCH(s, k_blobs_to_fp12, n, (int)n, P_<uint8_t>(s->d_blob), P_<uint32_t>(s->d_aux));
    std::vector<std::vector<int32_t>> g(ng);
    for (size_t k = 0; k < n; k++) g[k / pg].push_back((int32_t)k);
    if ((rc = tree_reduce<2>(s, 0, "tree_fp12_product", P_<uint32_t>(s->d_aux), g, P_<uint32_t>(s->d_F)))) return rc;
    LAUNCH(s, k_fp12_to_canon, ng, (int)ng, P_<uint32_t>(s->d_F), P_<uint8_t>(s->d_blob));
    LAUNCH_ROW(s, "k_row_final_exp", lsg_row_final_exp(S, (int)ng, P_<uint8_t>(s->d_blob), P_<int32_t>(s->d_verdict)));
    LSG_HIP(s, hipMemcpyAsync(s->h_verdict.p, s->d_verdict.p, 4 * ng, hipMemcpyDeviceToHost, S));
    s->n_verdicts = ng;
  }
  LSG_HIP(s, hipEventRecord(s->ev_done, s->st[0]));
  return LSG_OK;
}

// valid[0 .. max(n_verdicts, 1)) (0 for a ticket without partials)
int wait_final(Slot* s, int32_t* valid) {
  LSG_HIP(s, hipEventSynchronize(s->ev_done));
  if (!s->n_verdicts) valid[0] = 0;
  for (size_t g = 0; g < s->n_verdicts; g++) valid[g] = H_<int32_t>(s->h_verdict)[g];
  return LSG_OK;
}

Slot* take_slot(lsg_ctx* c) {
  Slot* s = free_slot(c, c->slots, LSG_SLOTS);
  if (!s) c->err = "all pipeline slots are busy (wait on an outstanding ticket first)";
  return s;
}

// stage + expand + hash on the utility slot (synchronous callers only)
int util_hash(Slot* s, const uint8_t* msgs, uint32_t msg_len, size_t n, const uint8_t* dst, uint32_t dst_len) {
  std::vector<lsg_set> sets(n);
  std::vector<const lsg_set*> sp(n);
  for (size_t i = 0; i < n; i++) {
    memset(&sets[i], 0, sizeof(lsg_set));
    sets[i].msg = msgs + (size_t)msg_len * i;
    sets[i].msg_len = msg_len;
    sp[i] = &sets[i];
  }
  s->in = &s->own;
  int rc;
  if ((rc = stage_sets(s, &s->own, sp.data(), n, 0, false, s->st[0]))) return rc;
  if ((rc = size_state(s, 0))) return rc;
  LSG_HIP(s, hipMemcpyAsync(s->d_dst.p, dst, dst_len, hipMemcpyHostToDevice, s->st[0]));
  int nn = (int)n;
  LAUNCH_T(s, "k_expand_msg", k_expand_msg, (nn + 63) / 64, 64, nn, P_<uint8_t>(s->own.d_msg),
           P_<uint32_t>(s->own.d_msgoff), P_<uint32_t>(s->own.d_msglen), P_<uint8_t>(s->d_dst), dst_len,
           P_<uint8_t>(s->d_ub));
  return launch_hash(s, nn);
}

#define LSG_ENTER(c)                         \
  std::lock_guard<std::mutex> _lk((c)->mu); \
  LSG_HIPC((c), hipSetDevice((c)->device))

// Block until a ticket's device work is done WITHOUT holding the context mutex, so a
// waiter (e.g. an N-API worker thread) never stalls submissions from another thread.  The
// ticket's slot cannot be recycled meanwhile: only the ticket's own wait call releases it.
int presync(lsg_ctx* c, lsg_ticket ticket, int kind) {
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    Slot* s = ticket_slot(c, ticket, kind);
    if (!s) return LSG_ERR_INVALID_ARG;
    ev = s->ev_done;
  }
  hipError_t e = hipEventSynchronize(ev);
  if (e != hipSuccess) return fail_c(c, "hipEventSynchronize", e);
  return LSG_OK;
}

}  // namespace

extern "C" {

int lsg_init(int device_ordinal, lsg_ctx** out) {
  if (!out) return LSG_ERR_INVALID_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return LSG_ERR_NO_DEVICE;
  int dev = device_ordinal < 0 ? 0 : device_ordinal;
  if (dev >= count) return LSG_ERR_NO_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return LSG_ERR_NO_DEVICE;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return LSG_ERR_NO_DEVICE;
  lsg_ctx* c = new lsg_ctx();
  c->device = dev;
  bool ok = hipSetDevice(dev) == hipSuccess && hipStreamCreateWithFlags(&c->s_final, hipStreamNonBlocking) == hipSuccess;
  for (int i = 0; i < LSG_SLOTS && ok; i++) ok = slot_create(c, &c->slots[i], i, nullptr) == LSG_OK;
  // each final exponentiation entry has its own stream: consecutive batches' FEs overlap
  for (int i = 0; i < LSG_FE_STREAMS && ok; i++)
    ok = hipStreamCreateWithFlags(&c->s_fe[i], hipStreamNonBlocking) == hipSuccess;
  for (int i = 0; i < LSG_FINALS && ok; i++) ok = slot_create(c, &c->finals[i], i, c->s_fe[i % LSG_FE_STREAMS]) == LSG_OK;
  if (ok) ok = slot_create(c, &c->util, 0, c->s_final) == LSG_OK;
  if (!ok) {
    lsg_destroy(c);
    return LSG_ERR_DEVICE;
  }
  *out = c;
  return LSG_OK;
}

int lsg_destroy(lsg_ctx* c) {
  if (!c) return LSG_ERR_INVALID_ARG;
  (void)hipSetDevice(c->device);
  for (Slot& s : c->slots) slot_destroy(&s);
  for (Slot& s : c->finals) slot_destroy(&s);
  slot_destroy(&c->util);
  free_dev(c->d_pktab);
  free_dev(c->d_pktab_ok);
  if (c->s_final) (void)hipStreamDestroy(c->s_final);
  for (hipStream_t st : c->s_fe)
    if (st) (void)hipStreamDestroy(st);
  delete c;
  return LSG_OK;
}

const char* lsg_last_error(lsg_ctx* c) { return c ? c->err.c_str() : "null context"; }

int lsg_device_name(lsg_ctx* c, char* buf, size_t len) {
  if (!c || !buf || !len) return LSG_ERR_INVALID_ARG;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) return LSG_ERR_DEVICE;
  snprintf(buf, len, "%s (%s, %d CUs)", prop.name, prop.gcnArchName, prop.multiProcessorCount);
  return LSG_OK;
}

int lsg_submit_jobs(lsg_ctx* c, const lsg_job* jobs, size_t n_jobs, uint64_t seed, lsg_ticket* ticket) {
  if (!c || !ticket || (n_jobs && !jobs)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = take_slot(c);
  if (!s) return LSG_ERR_BUSY;
  int rc = submit_jobs(c, s, jobs, n_jobs, seed);
  if (rc) {
    sync_slot(s);
    return rc;
  }
  *ticket = make_ticket(c, s, SLOT_JOBS);
  return LSG_OK;
}

int lsg_wait_jobs(lsg_ctx* c, lsg_ticket ticket, lsg_job_result* results, lsg_stats* stats) {
  if (!c) return LSG_ERR_INVALID_ARG;
  if (int prc = presync(c, ticket, SLOT_JOBS)) return prc;
  LSG_ENTER(c);
  Slot* s = ticket_slot(c, ticket, SLOT_JOBS);
  if (!s || (s->plan.results.size() && !results)) return LSG_ERR_INVALID_ARG;
  int rc = wait_jobs(c, s, results, stats);
  if (rc) sync_slot(s);
  release(c, s);
  return rc;
}

int lsg_verify_jobs(lsg_ctx* c, const lsg_job* jobs, size_t n_jobs, uint64_t seed, lsg_job_result* results,
                    lsg_stats* stats) {
  if (!c || (n_jobs && (!jobs || !results))) return LSG_ERR_INVALID_ARG;
  lsg_ticket t;
  int rc = lsg_submit_jobs(c, jobs, n_jobs, seed, &t);
  if (rc) return rc;
  return lsg_wait_jobs(c, t, results, stats);
}

int lsg_verify_sets(lsg_ctx* c, const lsg_set* sets, size_t n_sets, uint64_t seed, lsg_job_result* result) {
  if (!c || !result || (n_sets && !sets)) return LSG_ERR_INVALID_ARG;
  lsg_job job;
  job.sets = sets;
  job.n_sets = (uint32_t)n_sets;
  job.flags = 0;
  return lsg_verify_jobs(c, &job, 1, seed, result, nullptr);
}

int lsg_pipeline_slots(lsg_ctx* c, int32_t* n) {
  if (!c || !n) return LSG_ERR_INVALID_ARG;
  *n = LSG_SLOTS;
  return LSG_OK;
}

int lsg_poll(lsg_ctx* c, lsg_ticket ticket, int32_t* done) {
  if (!c || !done) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = ticket_slot(c, ticket, (int)((ticket >> 8) & 255));
  if (!s) return LSG_ERR_INVALID_ARG;
  hipError_t e = hipEventQuery(s->ev_done);
  if (e == hipErrorNotReady) {
    *done = 0;
    return LSG_OK;
  }
  if (e != hipSuccess) return fail(s, "hipEventQuery", e);
  *done = 1;
  return LSG_OK;
}

int lsg_stage(lsg_ctx* c, const lsg_set* sets, size_t n_sets, uint64_t seed, lsg_staged** out) {
  if (!c || !out || (n_sets && !sets)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  *out = nullptr;
  lsg_staged* in = new lsg_staged();
  std::vector<const lsg_set*> sp(n_sets);
  for (size_t i = 0; i < n_sets; i++) sp[i] = &sets[i];
  Slot* u = &c->util;
  int rc = stage_sets(u, in, sp.data(), n_sets, seed, true, u->st[0]);
  if (!rc && hipStreamSynchronize(u->st[0]) != hipSuccess) rc = fail(u, "hipStreamSynchronize", hipGetLastError());
  if (rc) {
    staged_free(in);
    delete in;
    return rc;
  }
  *out = in;
  return LSG_OK;
}

int lsg_staged_free(lsg_ctx* c, lsg_staged* staged) {
  if (!c || !staged) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  for (Slot& s : c->slots)
    if (s.kind != SLOT_FREE && s.in == staged) {
      c->err = "staged package still in use by an outstanding ticket";
      return LSG_ERR_BUSY;
    }
  staged_free(staged);
  delete staged;
  return LSG_OK;
}

int lsg_batch_submit(lsg_ctx* c, const lsg_staged* staged, lsg_ticket* ticket) {
  return lsg_batch_submit_groups(c, staged, 0, ticket);
}

int lsg_batch_submit_groups(lsg_ctx* c, const lsg_staged* staged, size_t group_size, lsg_ticket* ticket) {
  if (!c || !staged || !ticket) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = take_slot(c);
  if (!s) return LSG_ERR_BUSY;
  timer_reset(s);
  s->in = staged;
  int rc = submit_batch(s, group_size);
  if (rc) {
    sync_slot(s);
    return rc;
  }
  *ticket = make_ticket(c, s, SLOT_BATCH);
  return LSG_OK;
}

int lsg_batch_wait(lsg_ctx* c, lsg_ticket ticket, uint8_t* out576, int32_t* set_err, int32_t* any_error) {
  if (!c || !out576 || !any_error) return LSG_ERR_INVALID_ARG;
  if (int prc = presync(c, ticket, SLOT_BATCH)) return prc;
  LSG_ENTER(c);
  Slot* s = ticket_slot(c, ticket, SLOT_BATCH);
  if (!s) return LSG_ERR_INVALID_ARG;
  int rc = wait_batch(s, out576, set_err, any_error);
  if (rc) sync_slot(s);
  release(c, s);
  return rc;
}

int lsg_batch_partial(lsg_ctx* c, const lsg_set* sets, size_t n_sets, uint64_t seed, uint8_t* out576,
                      int32_t* set_err, int32_t* any_error) {
  if (!c || !out576 || !any_error || (n_sets && !sets)) return LSG_ERR_INVALID_ARG;
  lsg_ticket t;
  {
    LSG_ENTER(c);
    Slot* s = take_slot(c);
    if (!s) return LSG_ERR_BUSY;
    timer_reset(s);
    std::vector<const lsg_set*> sp(n_sets);
    for (size_t i = 0; i < n_sets; i++) sp[i] = &sets[i];
    s->in = &s->own;
    int rc = stage_sets(s, &s->own, sp.data(), n_sets, seed, true, s->st[0]);
    if (!rc) rc = submit_batch(s, 0);
    if (rc) {
      sync_slot(s);
      return rc;
    }
    t = make_ticket(c, s, SLOT_BATCH);
  }
  return lsg_batch_wait(c, t, out576, set_err, any_error);
}

int lsg_final_submit_groups(lsg_ctx* c, const uint8_t* partials576, size_t n_groups, size_t per_group,
                            lsg_ticket* ticket) {
  if (!c || !ticket || (n_groups && per_group && !partials576) || (n_groups && !per_group)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = free_slot(c, c->finals, LSG_FINALS);
  if (!s) {
    c->err = "all final-exponentiation entries are busy";
    return LSG_ERR_BUSY;
  }
  int rc = submit_final(s, partials576, n_groups, per_group);
  if (rc) {
    sync_slot(s);
    return rc;
  }
  *ticket = make_ticket(c, s, SLOT_FINAL);
  return LSG_OK;
}

int lsg_final_submit(lsg_ctx* c, const uint8_t* partials576, size_t n_partials, lsg_ticket* ticket) {
  if (!c || !ticket || (n_partials && !partials576)) return LSG_ERR_INVALID_ARG;
  return lsg_final_submit_groups(c, partials576, n_partials ? 1 : 0, n_partials, ticket);
}

int lsg_final_wait_groups(lsg_ctx* c, lsg_ticket ticket, int32_t* valid) {
  if (!c || !valid) return LSG_ERR_INVALID_ARG;
  if (int prc = presync(c, ticket, SLOT_FINAL)) return prc;
  LSG_ENTER(c);
  Slot* s = ticket_slot(c, ticket, SLOT_FINAL);
  if (!s) return LSG_ERR_INVALID_ARG;
  int rc = wait_final(s, valid);
  release(c, s);
  return rc;
}

int lsg_final_wait(lsg_ctx* c, lsg_ticket ticket, int32_t* valid) {
  if (!c || !valid) return LSG_ERR_INVALID_ARG;
  if (int prc = presync(c, ticket, SLOT_FINAL)) return prc;
  LSG_ENTER(c);
  Slot* s = ticket_slot(c, ticket, SLOT_FINAL);
  if (!s) return LSG_ERR_INVALID_ARG;
  if (s->n_verdicts > 1) {
    c->err = "ticket carries several groups: use lsg_final_wait_groups";
    return LSG_ERR_INVALID_ARG;
  }
  int rc = wait_final(s, valid);
  release(c, s);
  return rc;
}

int lsg_final_verify(lsg_ctx* c, const uint8_t* partials576, size_t n_partials, int32_t* valid) {
  if (!c || !valid || (n_partials && !partials576)) return LSG_ERR_INVALID_ARG;
  lsg_ticket t;
  int rc = lsg_final_submit(c, partials576, n_partials, &t);
  if (rc) return rc;
  return lsg_final_wait(c, t, valid);
}

int lsg_aggregate_pubkeys(lsg_ctx* c, const uint8_t* pks, uint32_t pk_len, size_t n, uint8_t* out96,
                          int32_t* err_code) {
  if (!c || !out96 || !err_code || (n && !pks)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->util;
  timer_reset(s);
  *err_code = 0;
  if (n == 0) {
    *err_code = LSG_ERR_EMPTY_AGGREGATE;
    return LSG_OK;
  }
  lsg_set q;
  memset(&q, 0, sizeof(q));
  q.pks = pks;
  q.pk_len = pk_len;
  q.n_pks = (uint32_t)n;
  const lsg_set* qp = &q;
  s->in = &s->own;
  int rc;
  if ((rc = stage_sets(s, &s->own, &qp, 1, 0, false, s->st[0]))) return rc;
  if ((rc = size_state(s, 0))) return rc;
  int np = (int)n;
  LAUNCH(s, k_pk_decode, np, np, P_<uint8_t>(s->own.d_pk), P_<uint32_t>(s->own.d_pklen), P_<uint32_t>(s->d_pkp),
         P_<int32_t>(s->d_pkerr), P_<uint32_t>(c->d_pktab), P_<uint8_t>(c->d_pktab_ok), (uint32_t)c->pktab_n);
  if ((rc = tree_reduce<0>(s, 1, "tree_g1_aggregate", P_<uint32_t>(s->d_pkp), s->own.sets_pks, P_<uint32_t>(s->d_agg))))
    return rc;
  LAUNCH(s, k_g1p_to_bytes, 1, 1, P_<uint32_t>(s->d_agg), P_<uint8_t>(s->d_blob));
  std::vector<int32_t> pkerr(n);
  LSG_HIP(s, hipMemcpyAsync(pkerr.data(), s->d_pkerr.p, 4 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipMemcpyAsync(out96, s->d_blob.p, 96, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  c->last = s;
  for (size_t k = 0; k < n; k++)
    if (pkerr[k]) {
      *err_code = pkerr[k];
      break;
    }
  return LSG_OK;
}

// pubkey table: keys decoded once on the device, gathered by index
int lsg_pubkey_table_set(lsg_ctx* c, size_t first, const uint8_t* pks, uint32_t pk_len, size_t n, int32_t* err) {
  if (!c || (n && !pks) || (pk_len != 48 && pk_len != 96) || first + n > 0xffffffffull) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  const size_t need = first + n, WG = lane_words<g1p_t>();
  if (need > c->pktab_cap) {
    // tickets in flight read the table: drain the device before moving it
    LSG_HIPC(c, hipDeviceSynchronize());
    size_t cap = std::max(std::max(need, 2 * c->pktab_cap), (size_t)1024);
    DevBuf nt, nok;
    LSG_HIPC(c, hipMalloc(&nt.p, 4 * WG * cap));
    nt.cap = 4 * WG * cap;
    hipError_t e = hipMalloc(&nok.p, cap);
    if (e != hipSuccess) {
      free_dev(nt);
      return fail_c(c, "hipMalloc", e);
    }
    nok.cap = cap;
    LSG_HIPC(c, hipMemset(nok.p, 0, cap));
    if (c->pktab_n) {
      LSG_HIPC(c, hipMemcpy(nt.p, c->d_pktab.p, 4 * WG * c->pktab_n, hipMemcpyDeviceToDevice));
      LSG_HIPC(c, hipMemcpy(nok.p, c->d_pktab_ok.p, c->pktab_n, hipMemcpyDeviceToDevice));
    }
    free_dev(c->d_pktab);
    free_dev(c->d_pktab_ok);
    c->d_pktab = nt;
    c->d_pktab_ok = nok;
    c->pktab_cap = cap;
  }
  lsg_set q;
  memset(&q, 0, sizeof(q));
  q.pks = pks;
  q.pk_len = pk_len;
  q.n_pks = (uint32_t)n;
  const lsg_set* qp = &q;
  s->in = &s->own;
  int rc;
  if ((rc = stage_sets(s, &s->own, &qp, 1, 0, false, s->st[0]))) return rc;
  if ((rc = size_state(s, 0))) return rc;
  // decode straight into the table rows first .. first + n - 1
  LAUNCH(s, k_pk_decode, n, (int)n, P_<uint8_t>(s->own.d_pk), P_<uint32_t>(s->own.d_pklen),
         P_<uint32_t>(c->d_pktab) + WG * first, P_<int32_t>(s->d_pkerr), (const uint32_t*)nullptr,
         (const uint8_t*)nullptr, 0u);
  std::vector<int32_t> pkerr(n);
  LSG_HIP(s, hipMemcpyAsync(pkerr.data(), s->d_pkerr.p, 4 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  std::vector<uint8_t> ok(n);
  for (size_t k = 0; k < n; k++) {
    ok[k] = pkerr[k] == 0 ? 1 : 0;
    if (err) err[k] = pkerr[k];
  }
  LSG_HIP(s, hipMemcpy(P_<uint8_t>(c->d_pktab_ok) + first, ok.data(), n, hipMemcpyHostToDevice));
  c->pktab_n = std::max(c->pktab_n, need);
  c->last = s;
  return LSG_OK;
}

int lsg_pubkey_table_size(lsg_ctx* c, size_t* n) {
  if (!c || !n) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  *n = c->pktab_n;
  return LSG_OK;
}

// batched KeyValidate
int lsg_pubkey_validate(lsg_ctx* c, const uint8_t* pks, uint32_t pk_len, size_t n, uint8_t* out96, int32_t* err) {
  if (!c || !err || (n && !pks) || (pk_len != 48 && pk_len != 96) || n > 0x7fffffffull) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  lsg_set q;
  memset(&q, 0, sizeof(q));
  q.pks = pks;
  q.pk_len = pk_len;
  q.n_pks = (uint32_t)n;
  const lsg_set* qp = &q;
  s->in = &s->own;
  int rc;
  if ((rc = stage_sets(s, &s->own, &qp, 1, 0, false, s->st[0]))) return rc;
  if ((rc = size_state(s, 0))) return rc;
  if ((rc = ensure(s, s->d_ub, 96 * n))) return rc;
  LAUNCH(s, k_pk_validate, n, (int)n, P_<uint8_t>(s->own.d_pk), pk_len, P_<uint32_t>(s->d_pkp), P_<int32_t>(s->d_pkerr));
  LSG_HIP(s, hipMemcpyAsync(err, s->d_pkerr.p, 4 * n, hipMemcpyDeviceToHost, s->st[0]));
  if (out96) {
    LAUNCH(s, k_g1p_to_bytes, n, (int)n, P_<uint32_t>(s->d_pkp), P_<uint8_t>(s->d_ub));
    LSG_HIP(s, hipMemcpyAsync(out96, s->d_ub.p, 96 * n, hipMemcpyDeviceToHost, s->st[0]));
  }
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  c->last = s;
  return LSG_OK;
}

int lsg_hash_to_g2(lsg_ctx* c, const uint8_t* msgs, uint32_t msg_len, size_t n, const uint8_t* dst,
                   uint32_t dst_len, uint8_t* out192) {
  if (!c || !out192 || (n && msg_len && !msgs) || dst_len > 255 || (dst_len && !dst)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  int rc;
  if ((rc = util_hash(s, msgs, msg_len, n, dst, dst_len))) return rc;
  if ((rc = ensure(s, s->d_blob, 192 * n))) return rc;
  int nn = (int)n;
  LAUNCH(s, k_g2a_to_bytes, nn, nn, P_<uint32_t>(s->d_H), P_<uint8_t>(s->d_hinf), P_<uint8_t>(s->d_blob));
  LSG_HIP(s, hipMemcpyAsync(out192, s->d_blob.p, 192 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  c->last = s;
  return LSG_OK;
}

int lsg_sig_decode(lsg_ctx* c, const uint8_t* sigs, uint32_t sig_len, size_t n, uint8_t* out192, int32_t* err) {
  if (!c || !out192 || !err || (n && !sigs)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  std::vector<lsg_set> sets(n);
  std::vector<const lsg_set*> sp(n);
  for (size_t i = 0; i < n; i++) {
    memset(&sets[i], 0, sizeof(lsg_set));
    sets[i].sig = sigs + (size_t)sig_len * i;
    sets[i].sig_len = sig_len;
    sp[i] = &sets[i];
  }
  s->in = &s->own;
  int rc;
  if ((rc = stage_sets(s, &s->own, sp.data(), n, 0, false, s->st[0]))) return rc;
  if ((rc = size_state(s, 0)) || (rc = ensure(s, s->d_blob, 192 * n))) return rc;
  int nn = (int)n;
  LAUNCH(s, k_sig_decode, nn, nn, P_<uint8_t>(s->own.d_sig), P_<uint32_t>(s->own.d_siglen), P_<uint32_t>(s->d_sigaff),
         P_<uint8_t>(s->d_siginf), P_<int32_t>(s->d_seterr));
  LAUNCH(s, k_sig_subgroup, nn, nn, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf), P_<int32_t>(s->d_seterr));
  LAUNCH(s, k_g2a_to_bytes, nn, nn, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf), P_<uint8_t>(s->d_blob));
  LSG_HIP(s, hipMemcpyAsync(out192, s->d_blob.p, 192 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipMemcpyAsync(err, s->d_seterr.p, 4 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  c->last = s;
  return LSG_OK;
}

// G2 signature aggregation for the op pools: n_groups independent
// Signature.aggregate calls in one pass -- decode without the subgroup check
// (signatureFromBytesNoCheck, opPools/utils.ts:32-34), projective sums as a segmented tree,
// one compression per group
int lsg_aggregate_signatures(lsg_ctx* c, const uint8_t* sigs, uint32_t sig_len, const uint32_t* offsets,
                             size_t n_groups, uint8_t* out96, int32_t* err) {
  if (!c || !offsets || (n_groups && (!out96 || !err)) || offsets[0] != 0 || n_groups > 0x7fffffffull)
    return LSG_ERR_INVALID_ARG;
  for (size_t g = 0; g < n_groups; g++)
    if (offsets[g + 1] < offsets[g]) return LSG_ERR_INVALID_ARG;
  const size_t n = offsets[n_groups];
  if (n && !sigs) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->util;
  timer_reset(s);
  std::vector<std::vector<int32_t>> groups;
  std::vector<size_t> gid;  // groups[k] is caller group gid[k]
  for (size_t g = 0; g < n_groups; g++) {
    err[g] = offsets[g + 1] == offsets[g] ? LSG_ERR_EMPTY_AGGREGATE : 0;
    memset(out96 + 96 * g, 0, 96);
    if (offsets[g + 1] == offsets[g]) continue;
    std::vector<int32_t> m;
    for (uint32_t i = offsets[g]; i < offsets[g + 1]; i++) m.push_back((int32_t)i);
    groups.push_back(std::move(m));
    gid.push_back(g);
  }
  if (n == 0) return LSG_OK;
  std::vector<lsg_set> sets(n);
  std::vector<const lsg_set*> sp(n);
  for (size_t i = 0; i < n; i++) {
    memset(&sets[i], 0, sizeof(lsg_set));
    sets[i].sig = sigs + (size_t)sig_len * i;
    sets[i].sig_len = sig_len;
    sp[i] = &sets[i];
  }
  s->in = &s->own;
  int rc;
  const size_t ng = groups.size();
  if ((rc = stage_sets(s, &s->own, sp.data(), n, 0, false, s->st[0]))) return rc;
  if ((rc = size_state(s, ng)) || (rc = ensure(s, s->d_blob, 96 * ng))) return rc;
  int nn = (int)n;
  LAUNCH(s, k_sig_decode, nn, nn, P_<uint8_t>(s->own.d_sig), P_<uint32_t>(s->own.d_siglen), P_<uint32_t>(s->d_sigaff),
         P_<uint8_t>(s->d_siginf), P_<int32_t>(s->d_seterr));
  LAUNCH(s, k_sig_proj, nn, nn, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf), P_<int32_t>(s->d_seterr),
         P_<uint32_t>(s->d_rs));
  if ((rc = tree_reduce<1>(s, 1, "tree_g2_aggregate", P_<uint32_t>(s->d_rs), groups, P_<uint32_t>(s->d_S)))) return rc;
  LAUNCH(s, k_g2p_compress, ng, (int)ng, P_<uint32_t>(s->d_S), P_<uint8_t>(s->d_blob));
  std::vector<int32_t> serr(n);
  std::vector<uint8_t> blob(96 * ng);
  LSG_HIP(s, hipMemcpyAsync(serr.data(), s->d_seterr.p, 4 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipMemcpyAsync(blob.data(), s->d_blob.p, 96 * ng, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  c->last = s;
  // Signature.aggregate throws on the first signature that fails to deserialize
  for (size_t k = 0; k < ng; k++) {
    const size_t g = gid[k];
    for (uint32_t i = offsets[g]; i < offsets[g + 1] && !err[g]; i++) err[g] = serr[i];
    if (!err[g]) memcpy(out96 + 96 * g, blob.data() + 96 * k, 96);
  }
  return LSG_OK;
}

// SSZ signing roots; kind 0: object roots given, 1: AttestationData bytes
static int signing_roots(lsg_ctx* c, int kind, const uint8_t* objs, size_t n, const uint8_t* domain,
                         uint32_t dstride, uint8_t* out32) {
  const size_t ob = kind ? 128 : 32;
  if (!c || !domain || (dstride != 0 && dstride != 32) || (n && (!objs || !out32)) || n > 0x7fffffffull)
    return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  const size_t nd = dstride ? n : 1;
  int rc;
  if ((rc = ensure(s, s->d_aux, ob * n + 32 * nd)) || (rc = ensure(s, s->d_blob, 32 * n))) return rc;
  uint8_t* d_obj = P_<uint8_t>(s->d_aux);
  uint8_t* d_dom = d_obj + ob * n;
  LSG_HIP(s, hipMemcpyAsync(d_obj, objs, ob * n, hipMemcpyHostToDevice, s->st[0]));
  LSG_HIP(s, hipMemcpyAsync(d_dom, domain, 32 * nd, hipMemcpyHostToDevice, s->st[0]));
  const int nn = (int)n;
  const unsigned blocks = (unsigned)((n + 63) / 64);
  if (kind)
    LAUNCH_T(s, "k_attestation_signing_root", k_attestation_signing_root, blocks, 64, nn, d_obj, d_dom, dstride,
             P_<uint8_t>(s->d_blob));
  else
    LAUNCH_T(s, "k_signing_root", k_signing_root, blocks, 64, nn, d_obj, d_dom, dstride, P_<uint8_t>(s->d_blob));
  LSG_HIP(s, hipMemcpyAsync(out32, s->d_blob.p, 32 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  c->last = s;
  return LSG_OK;
}

int lsg_signing_roots(lsg_ctx* c, const uint8_t* roots32, size_t n, const uint8_t* domain32, uint32_t domain_stride,
                      uint8_t* out32) {
  return signing_roots(c, 0, roots32, n, domain32, domain_stride, out32);
}

int lsg_attestation_signing_roots(lsg_ctx* c, const uint8_t* data128, size_t n, const uint8_t* domain32,
                                  uint32_t domain_stride, uint8_t* out32) {
  return signing_roots(c, 1, data128, n, domain32, domain_stride, out32);
}

int lsg_sign(lsg_ctx* c, const uint8_t* sks32, const uint8_t* msgs, uint32_t msg_len, size_t n, uint8_t* out96) {
  if (!c || !out96 || (n && (!sks32 || !msgs))) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  int rc;
  if ((rc = util_hash(s, msgs, msg_len, n, DST_POP, DST_POP_LEN))) return rc;
  if ((rc = ensure(s, s->d_blob, 96 * n)) || (rc = ensure(s, s->d_aux, 32 * n))) return rc;
  LSG_HIP(s, hipMemcpyAsync(s->d_aux.p, sks32, 32 * n, hipMemcpyHostToDevice, s->st[0]));
  int nn = (int)n;
  LAUNCH(s, k_sign, nn, nn, P_<uint8_t>(s->d_aux), P_<uint32_t>(s->d_H), P_<uint8_t>(s->d_blob));
  LSG_HIP(s, hipMemcpyAsync(out96, s->d_blob.p, 96 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  return LSG_OK;
}

int lsg_sk_to_pk(lsg_ctx* c, const uint8_t* sks32, size_t n, uint8_t* out96) {
  if (!c || !out96 || (n && !sks32)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  int rc;
  if ((rc = ensure(s, s->d_blob, 96 * n)) || (rc = ensure(s, s->d_aux, 32 * n))) return rc;
  LSG_HIP(s, hipMemcpyAsync(s->d_aux.p, sks32, 32 * n, hipMemcpyHostToDevice, s->st[0]));
  int nn = (int)n;
  LAUNCH(s, k_sk_to_pk, nn, nn, P_<uint8_t>(s->d_aux), P_<uint8_t>(s->d_blob));
  LSG_HIP(s, hipMemcpyAsync(out96, s->d_blob.p, 96 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  return LSG_OK;
}

int lsg_probe_fp_mul_rate(lsg_ctx* c, double* fp_mul_per_s, double* mad_per_s) {
  if (!c || !fp_mul_per_s || !mad_per_s) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->util;
  hipDeviceProp_t prop;
  LSG_HIP(s, hipGetDeviceProperties(&prop, c->device));
  int items = prop.multiProcessorCount * 32 * (64 / LSG_GROUP);  // 32 waves per CU
  int rc;
  if ((rc = ensure(s, s->d_aux, 4 * 16 * (size_t)items))) return rc;
  std::vector<uint32_t> init(16 * (size_t)items, 0);
  for (size_t i = 0; i < init.size(); i += 4) init[i] = (uint32_t)(i * 2654435761u);  // small values < p
  LSG_HIP(s, hipMemcpy(s->d_aux.p, init.data(), 4 * init.size(), hipMemcpyHostToDevice));
  const int iters = 64;
  hipStream_t S = s->st[0];
  hipLaunchKernelGGL(k_probe_fp_mul, dim3(lane_blocks(items)), dim3(LSG_TPB), 0, S, items, 2, P_<uint32_t>(s->d_aux));
  hipEvent_t a, b;
  LSG_HIP(s, hipEventCreate(&a));
  LSG_HIP(s, hipEventCreate(&b));
  LSG_HIP(s, hipEventRecord(a, S));
  hipLaunchKernelGGL(k_probe_fp_mul, dim3(lane_blocks(items)), dim3(LSG_TPB), 0, S, items, iters,
                     P_<uint32_t>(s->d_aux));
  LSG_HIP(s, hipEventRecord(b, S));
  LSG_HIP(s, hipEventSynchronize(b));
  float ms = 0;
  LSG_HIP(s, hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  double muls = (double)items * iters * 4.0;
  *fp_mul_per_s = muls / (ms * 1e-3);
  *mad_per_s = *fp_mul_per_s * 300.0;
  return LSG_OK;
}

int lsg_probe_mad_peak(lsg_ctx* c, double* mad_per_s) {
  if (!c || !mad_per_s) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->util;
  hipDeviceProp_t prop;
  LSG_HIP(s, hipGetDeviceProperties(&prop, c->device));
  const int blocks = prop.multiProcessorCount * 32;  // 32 waves per CU (8 per SIMD)
  const size_t threads = (size_t)blocks * 256;
  int rc;
  if ((rc = ensure(s, s->d_aux, 8 * threads))) return rc;
  hipStream_t S = s->st[0];
  const int iters = 4096;
  hipLaunchKernelGGL(k_probe_mad, dim3(blocks), dim3(256), 0, S, 16, 3u, P_<uint64_t>(s->d_aux));
  hipEvent_t a, b;
  LSG_HIP(s, hipEventCreate(&a));
  LSG_HIP(s, hipEventCreate(&b));
  LSG_HIP(s, hipEventRecord(a, S));
  hipLaunchKernelGGL(k_probe_mad, dim3(blocks), dim3(256), 0, S, iters, 5u, P_<uint64_t>(s->d_aux));
  LSG_HIP(s, hipEventRecord(b, S));
  LSG_HIP(s, hipEventSynchronize(b));
  float ms = 0;
  LSG_HIP(s, hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *mad_per_s = (double)threads * iters * 16.0 / (ms * 1e-3);
  return LSG_OK;
}

int lsg_last_kernel_times(lsg_ctx* c, const char** names, double* ms, int max) {
  if (!c) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  const Slot* s = c->last;
  if (!s) return 0;
  for (int k = 0; k < 2; k++) (void)hipStreamSynchronize(s->st[k]);
  int n = 0;
  for (size_t i = 0; i < s->ntimers && n < max; i++) {
    float t = 0;
    if (hipEventElapsedTime(&t, s->timers[i].a, s->timers[i].b) != hipSuccess) t = -1;
    if (names) names[n] = s->timers[i].name;
    if (ms) ms[n] = t;
    n++;
  }
  return n;
}

}  // extern "C"
