// lsg_launch.h -- launch wrappers of the gfx950 kernels, one per kernel, for the host
// orchestration (lsg_host.hip).  The kernels live in five translation units built in
// parallel (lsg_k_hash / lsg_k_sig / lsg_k_pk / lsg_k_miller / lsg_k_reduce .hip); each
// wrapper sizes the grid from its item count, launches on `st` and returns
// hipGetLastError().  Pointers are device pointers; lane-form arrays use the item-major layout
// of lsg_layout.h.  Counts of 0 launch nothing.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace lsgk {
// ---- hash_to_G2 (lsg_k_hash.hip)                                      SURVEY 8a M3
hipError_t expand_msg(hipStream_t st, int n, const uint8_t* msg, const uint32_t* off, const uint32_t* len,
                      const uint8_t* dst, uint32_t dst_len, uint8_t* ub);
hipError_t h2c_prep(hipStream_t st, int n, const uint8_t* ub, uint32_t* U, uint32_t* norms);
hipError_t h2c_map(hipStream_t st, int n, const uint32_t* U, const uint32_t* ninv, uint32_t* Hp);
hipError_t h2c_clear(hipStream_t st, int n, uint32_t* Hp, uint32_t* zN, uint8_t* hinf);
hipError_t h2c_gather(hipStream_t st, int n, const uint32_t* mid, const uint32_t* Hm, const uint8_t* hinfm, uint32_t* H,
                      uint8_t* hinf);
hipError_t h2c_affine(hipStream_t st, int n, const uint32_t* Hp, const uint32_t* ninv, const uint8_t* hinf,
                      uint32_t* H);
hipError_t signing_root(hipStream_t st, int n, const uint8_t* roots, const uint8_t* domains, uint32_t dstride,
                        uint8_t* out32);
hipError_t attestation_signing_root(hipStream_t st, int n, const uint8_t* data, const uint8_t* domains,
                                    uint32_t dstride, uint8_t* out32);

// ---- signatures (lsg_k_sig.hip)                                       SURVEY 8a M2, M4
hipError_t sig_decode(hipStream_t st, int n, const uint8_t* sig, const uint32_t* sig_len, uint32_t* sig_aff,
                      uint8_t* inf, int32_t* err);
hipError_t sig_subgroup(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, int32_t* err);
// out[i] = the projective point set i adds to its group's RLC signature sum: the identity
// when the signature did not decode (err), is the point at infinity (inf) or the set's
// aggregated key is infinity (pinf, may be null); else [r_i] sig_i when rnd is given and
// (mode == null or mode[i] != 0), else sig_i itself (the bucket MSM scales later).
hipError_t sig_prep(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, const int32_t* err,
                    const uint8_t* pinf, const uint64_t* rnd, const uint8_t* mode, uint32_t* out);
// [r_i] sig_i (or the identity, as sig_prep) for the sets with mode[i] != 0 only; other
// entries of out are left as they are (fallback phases fill one scaled array in turns)
hipError_t sig_scale_only(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, const int32_t* err,
                          const uint8_t* pinf, const uint64_t* rnd, const uint8_t* mode, uint32_t* out);
hipError_t g2a_to_bytes(hipStream_t st, int n, const uint32_t* pts, const uint8_t* inf, uint8_t* out192);
hipError_t g2p_compress(hipStream_t st, int n, const uint32_t* pts, uint8_t* out96);
hipError_t g2p_to_canon(hipStream_t st, int n, const uint32_t* pts, uint8_t* out288);
hipError_t sign(hipStream_t st, int n, const uint8_t* sks, const uint32_t* H, uint8_t* out96);

// ---- public keys (lsg_k_pk.hip)                                       SURVEY 8a H8, M1, M4
// pk: key slots of `stride` bytes (96, or 4 when every key is a table index)
hipError_t pk_decode(hipStream_t st, int n, const uint8_t* pk, uint32_t stride, const uint32_t* pk_len, uint32_t* pts,
                     int32_t* err, const uint32_t* tab, const uint8_t* tab_ok, uint32_t tab_n);
hipError_t pk_validate(hipStream_t st, int n, const uint8_t* pk, uint32_t len, uint32_t* pts, int32_t* err);
// keys -> pubkey-table rows (lsgl::W_TAB words: affine point) + infinity flags + per-key errors
hipError_t pk_gather_aff(hipStream_t st, int n, const uint8_t* pk, uint32_t stride, const uint32_t* pk_len, uint32_t* pts,
                         uint8_t* inf, int32_t* err, const uint32_t* tab, const uint8_t* tab_ok, uint32_t tab_n);
// the first pass of a segmented G1 sum over staged keys (plan_seg chunks; later passes:
// seg_reduce op 0 over tmp): keys fetched and folded with mixed additions, errors to err
hipError_t pk_agg_seg(hipStream_t st, int n_chunks, int ips_log2, const int32_t* chunks, const uint8_t* pk, uint32_t stride,
                      const uint32_t* pk_len, int32_t* err, const uint32_t* tab, const uint8_t* tab_ok, uint32_t tab_n,
                      uint32_t* dst, uint32_t* tmp);
// the batch-affine aggregation tree (lsg_k_pk.hip k_agg_*; plan: lsg_host.hip plan_agg_tree).
// Level 0 holds every tree set's keys at an offset aligned to 2^L, padded with infinity up to
// the next multiple (N0 points); level t + 1 point q is the sum of level t points 2q and
// 2q + 1, so level L holds each set's sum in ceil(len / 2^L) points.  Level t's items (point
// pairs) q = c + j n_c(t) belong to lane pair c (j < T; n_c(t) = n_c0 >> t).
struct AggTreeArgs {
  int L = 0, T = 1;          // levels, items per lane pair
  int64_t n_c0 = 0, N0 = 0;  // level-0 lane pairs (a multiple of 128 << (L - 1)), points
  const int32_t* blk_set = nullptr;  // set of each 2^L block of level 0
  const int32_t* set_o0 = nullptr;   // per set: level-0 offset, key count, first staged key
  const int32_t* set_len = nullptr;
  const int32_t* set_pk0 = nullptr;
  const uint8_t* pk = nullptr;  // staged keys (bytes or table indices), as for pk_decode
  uint32_t stride = 0;
  const uint32_t* pk_len = nullptr;
  int32_t* pk_err = nullptr;
  const uint32_t* tab = nullptr;
  const uint8_t* tab_ok = nullptr;
  uint32_t tab_n = 0;
  uint32_t* pts = nullptr;  // point arena: level t at point offset 2 N0 - (N0 >> (t - 1)) (0 for t = 0)
  uint8_t* inf = nullptr;   // infinity flags, same offsets
  uint32_t* pre[2] = {nullptr, nullptr};   // per level (t & 1): prefix products, T n_c(t) items
  uint32_t* cinv[2] = {nullptr, nullptr};  // per level and lane pair: 1 / (chunk product)
  uint8_t* flag[2] = {nullptr, nullptr};   // per level and lane pair: chunk had an equal-x pair
};
hipError_t agg_leaf(hipStream_t st, const AggTreeArgs& a);
hipError_t agg_step(hipStream_t st, const AggTreeArgs& a, int t);
// per set: (0, level-L offset, count) or (1, first staged key, count) -> projective sum
hipError_t agg_final(hipStream_t st, const AggTreeArgs& a, int n_sets, const int32_t* src, uint32_t* agg);
hipError_t pk_scale(hipStream_t st, int n, const uint32_t* agg, const uint64_t* rnd, uint32_t* Pp, uint32_t* zP,
                    uint8_t* pinf);
hipError_t pk_affine(hipStream_t st, int n, const uint32_t* Pp, const uint32_t* zinv, uint32_t* P);
hipError_t pk_mask(hipStream_t st, int n, const uint32_t* Pp, const int32_t* err, const uint8_t* pinf, uint32_t* out);
hipError_t g1p_affine_inv(hipStream_t st, int n, const uint32_t* Pp, uint32_t* P, uint8_t* pinf);
hipError_t g1p_to_bytes(hipStream_t st, int n, const uint32_t* pts, uint8_t* out96);
hipError_t sk_to_pk(hipStream_t st, int n, const uint8_t* sks, uint8_t* out96);

// ---- Miller loop (lsg_k_miller.hip)                                   SURVEY 8a M5
// lines in LDS, four waves per item of <= 4 sets (f_item = prod of the item's pairs)
hipError_t miller_fused(hipStream_t st, int n_items, const int32_t* item_first, const int32_t* item_cnt,
                        const uint32_t* P, const uint8_t* pinf, const uint8_t* hinf, const int32_t* err,
                        const uint32_t* H, uint32_t* f);
hipError_t miller_lines(hipStream_t st, int n, const uint32_t* H, uint32_t* lines);
// list form, one pair per item: item k = set list[k]; lines stored by item (n items)
hipError_t miller_lines_list(hipStream_t st, int n, const int32_t* list, const uint32_t* H, uint32_t* lines);
hipError_t miller_accum_list(hipStream_t st, int n, const int32_t* list, const uint32_t* P, const uint8_t* pinf,
                             const uint8_t* hinf, const int32_t* err, const uint32_t* lines, uint32_t* f);
// K = pairs per item (1, 2 or 4)
hipError_t miller_accum(hipStream_t st, int K, int n_items, const int32_t* item_first, const int32_t* item_cnt,
                        const uint32_t* P, const uint8_t* pinf, const uint8_t* hinf, const int32_t* err, int n_sets,
                        const uint32_t* lines, uint32_t* f);

// ---- reductions, inversions, conversions, probes (lsg_k_reduce.hip)
// Segmented reduction (op 0: G1 add, 1: G2 add, 2: Fp12 product): chunk c = chunks[3c..3c+2]
// = {off, len, out} combines elements idx[off .. off+len) of src (idx == null: off .. off+len)
// into out >= 0 ? dst[out] : tmp[-out-1].  2^ips_log2 lane pairs share a chunk: each folds
// every 2^ips_log2-th element serially, then a lane butterfly combines them.
hipError_t seg_reduce(hipStream_t st, int op, int n_chunks, int ips_log2, const int32_t* chunks, const int32_t* idx,
                      const uint32_t* src, uint32_t* dst, uint32_t* tmp);
// batched inversion, chunks of LSG_BINV_T values per lane pair: fold (prefix products pre and
// chunk products tot), root (one inversion), unfold (out = 1/in, 0 for zeros when zero_to_one)
hipError_t binv_fold(hipStream_t st, int n, int zero_to_one, const uint32_t* in, uint32_t* pre, uint32_t* tot);
hipError_t binv_root(hipStream_t st, const uint32_t* top, uint32_t* inv);
// one-launch form: every block inverts its own 128 x T values (one divstep root per block)
hipError_t binv_block(hipStream_t st, int n, int T, int zero_to_one, const uint32_t* in, uint32_t* pre, uint32_t* out);
hipError_t binv_unfold(hipStream_t st, int n, int zero_to_one, const uint32_t* in, const uint32_t* pre,
                       const uint32_t* tinv, uint32_t* out);
hipError_t blobs_to_fp12(hipStream_t st, int n, const uint8_t* blobs, uint32_t* out);
hipError_t fp12_to_canon(hipStream_t st, int n, const uint32_t* in, uint8_t* out576);
// out576 = in576^r (canonical Fp12 blobs, one item): an exported partial's RLC randomizer
hipError_t fp12_pow_u64(hipStream_t st, const uint8_t* in576, uint64_t r, uint8_t* out576);
hipError_t probe_fp_mul(hipStream_t st, int items, int iters, uint32_t* io);
hipError_t check_fp2_mul(hipStream_t st, int n, const uint32_t* in, uint32_t* out);
hipError_t probe_mad(hipStream_t st, int blocks, int iters, uint32_t seed, uint64_t* io);
}  // namespace lsgk
