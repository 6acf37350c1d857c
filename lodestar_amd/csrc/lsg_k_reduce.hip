// lsg_k_reduce.hip -- segmented reductions of lane-form values (G1/G2 sums, Fp12 products),
// batched field inversions, canonical-blob conversions and the roofline probes.
//
// The segmented reduction serves every "sum over a list" of the path with one launch per pass:
//   PublicKey.aggregate of each set's keys      (utils.ts:11)      G1 add
//   the RLC bucket MSM: buckets, per-bit sums   (blst mul_n_aggregate; 8a M4)      G2 add
//   small groups' signature sums, op-pool sums  (8a M4, 8f(4))                     G2 add
//   each group's Miller product                 (blst miller_loop_n/commit; 8a M5) Fp12 mul
// A chunk (a list of up to ips x F elements) belongs to 2^ips_log2 lane pairs of one wave:
// pair j folds elements j, j + ips, j + 2 ips, ... serially (every fold is a full-width
// SIMD operation), then the ips partial values are combined by a butterfly over lanes
// (shuffles, no LDS round trip).  Segments longer than one chunk get a second pass over the
// chunk results (lsg_host.hip plan_seg), so a reduction is one or two launches instead of
// one launch per tree level.
#include "lsg_kcommon.hpp"
namespace {
#include "lsg_inv.hpp"
}  // namespace

template <int OP>
struct seg_op;
template <>
struct seg_op<0> {
  typedef g1p_t T;
  static LSG_DEVI T ident() { return proj_inf<fp_t>(); }
  static LSG_DEVI T op(const T& a, const T& b) { return g1_add(a, b); }
};
template <>
struct seg_op<1> {
  typedef g2p_t T;
  static LSG_DEVI T ident() { return proj_inf<fp2_t>(); }
  static LSG_DEVI T op(const T& a, const T& b) { return g2_add(a, b); }
};
template <>
struct seg_op<2> {
  typedef fp12_t T;
  static LSG_DEVI T ident() { return fp12_one(); }
  static LSG_DEVI T op(const T& a, const T& b) { return fp12_mul(a, b); }
};

// Every lane runs the butterfly (no early return): a chunk's lanes are all active or all
// inactive, and a chunk never straddles a wave (ips <= 32 pairs, chunk-aligned items).
template <int OP>
__global__ void LSG_KERNEL_ATTR_W(OP == 2 ? 1 : LSG_WAVES_PER_EU)
    k_seg_reduce(int n_chunks, int ips_log2, const int32_t* __restrict__ chunks, const int32_t* __restrict__ idx,
                 const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t* __restrict__ tmp) {
  typedef seg_op<OP> O;
  typedef typename O::T T;
  lsg_lane_setup();
#if LSG_RED_PRIO  // A/B builds: issue priority of the reductions' waves
  __builtin_amdgcn_s_setprio(LSG_RED_PRIO);
#endif
  const size_t item = gtid() / LSG_GROUP;
  const size_t c = item >> ips_log2;
  const int ips = 1 << ips_log2, j = (int)(item & (size_t)(ips - 1));
  const bool active = c < (size_t)n_chunks;
  T acc = O::ident();
  int out = 0;
  if (active) {
    const int off = chunks[3 * c], len = chunks[3 * c + 1];
    out = chunks[3 * c + 2];
    if (j < len) {
      acc = lane_load<T>(src, idx ? (size_t)idx[off + j] : (size_t)(off + j));
#pragma unroll 1
      for (int k = j + ips; k < len; k += ips) acc = O::op(acc, lane_load<T>(src, idx ? (size_t)idx[off + k] : (size_t)(off + k)));
    }
  }
#pragma unroll 1
  for (int o = ips >> 1; o >= 1; o >>= 1) acc = O::op(acc, shfl_xor_t(acc, LSG_GROUP * o));
  if (active && j == 0) {
    if (out >= 0)
      lane_store(dst, (size_t)out, acc);
    else
      lane_store(tmp, (size_t)(-out - 1), acc);
  }
}

// ---- batched field inversion (Montgomery's trick, chunked): every field inversion of a
// stage -- 1/Z of the scaled pubkeys, 1/N(tv1) of the SSWU maps, 1/N(Z) of the hashed points
// -- shares one exponentiation per batch instead of one per set.  A level folds chunks of
// LSG_BINV_T consecutive values per lane pair (prefix products, one chunk product each); the
// chunk products are the next level's values, up to one value, whose inverse unfolds back
// down (two products per value).  log_T(n) launches each way instead of log_2(n).  Zero
// inputs (points at infinity, the SSWU exceptional case) are carried as 1 and come out as 0,
// the value fp_inv(0) gives.
__global__ void LSG_KERNEL_ATTR k_binv_fold(int n, int zero_to_one, const uint32_t* __restrict__ in,
                                            uint32_t* __restrict__ pre, uint32_t* __restrict__ tot) {
  const int n_chunks = (n + LSG_BINV_T - 1) / LSG_BINV_T;
  LANE_ITEM(n_chunks);
  (void)lead;
  const fp_t one = fp_one();
  const int first = (int)item * LSG_BINV_T, last = min(n, first + LSG_BINV_T);
  fp_t acc = one;
#pragma unroll 1
  for (int k = first; k < last; k++) {
    fp_t x = lane_load<fp_t>(in, k);
    if (zero_to_one) x = fp_select(fp_is_zero(x), one, x);
    acc = k == first ? x : fp_mul(acc, x);
    lane_store(pre, k, acc);
  }
  lane_store(tot, item, acc);
}
// the one inversion of a batched inversion: the divstep GCD (lsg_inv.hpp, ~30 us) instead of
// the ~455-product Fermat chain (~0.4 ms of dependent products on one lane pair)
__global__ void LSG_KERNEL_ATTR k_binv_root(const uint32_t* __restrict__ top, uint32_t* __restrict__ inv) {
  LANE_ITEM(1);
  (void)lead;
  const fp_t d = pair_inv_gcd(pair_canon(lane_load<fp_t>(top, 0)));  // (x R)^-1 as an integer, 0 -> 0
  lane_store(inv, 0, pair_mont_mul(d, fp_t(FP_RCUBE)));              // x^-1 R
}
// out[k] = 1 / in[k] from the chunk's inverse product tinv[chunk] and the prefix products
__global__ void LSG_KERNEL_ATTR k_binv_unfold(int n, int zero_to_one, const uint32_t* __restrict__ in,
                                              const uint32_t* __restrict__ pre, const uint32_t* __restrict__ tinv,
                                              uint32_t* __restrict__ out) {
  const int n_chunks = (n + LSG_BINV_T - 1) / LSG_BINV_T;
  LANE_ITEM(n_chunks);
  (void)lead;
  const fp_t one = fp_one();
  const int first = (int)item * LSG_BINV_T, last = min(n, first + LSG_BINV_T);
  fp_t acc = lane_load<fp_t>(tinv, item);  // 1 / (in[first] * ... * in[last-1])
#pragma unroll 1
  for (int k = last - 1; k >= first; k--) {
    fp_t x = lane_load<fp_t>(in, k);
    const bool z = zero_to_one && fp_is_zero(x);
    fp_t r = k > first ? fp_mul(acc, lane_load<fp_t>(pre, k - 1)) : acc;
    lane_store(out, k, z ? fp_zero() : r);
    if (k > first && !z) acc = fp_mul(acc, x);
  }
}

// One-launch batched inversion: every workgroup inverts its own share --
// lane pair l of block b folds the T consecutive values from (b * 128 + l) * T into prefix
// products, the block's 128 chunk products go through an LDS heap with ONE divstep inversion
// at its root (block_inv), and each lane pair unfolds its chunk.  No level crosses a block,
// so the fold / root / unfold launches of the multi-level form (2 log16 n + 1 of them, each a
// latency-bound stub between real kernels) become one.  zero_to_one: zeros fold as one and
// come out as zero (fp_inv(0) = 0).
__global__ void LSG_KERNEL_ATTR k_binv_block(int n, int T, int zero_to_one, const uint32_t* __restrict__ in,
                                             uint32_t* __restrict__ pre, uint32_t* __restrict__ out) {
  __shared__ uint32_t H[2 * LSG_ITEMS_PER_BLOCK * lsgl::W_FP], I[2 * LSG_ITEMS_PER_BLOCK * lsgl::W_FP];
  lsg_lane_setup();
#if LSG_RED_PRIO
  __builtin_amdgcn_s_setprio(LSG_RED_PRIO);
#endif
  const int l = (int)(threadIdx.x / LSG_GROUP);
  const int64_t first = ((int64_t)blockIdx.x * LSG_ITEMS_PER_BLOCK + l) * T;
  const int64_t last = first + T < (int64_t)n ? first + T : (int64_t)n;
  const fp_t one = fp_one();
  fp_t acc = one;
#pragma unroll 1
  for (int64_t k = first; k < last; k++) {
    fp_t x = lane_load<fp_t>(in, (size_t)k);
    if (zero_to_one) x = fp_select(fp_is_zero(x), one, x);
    acc = k == first ? x : fp_mul(acc, x);
    if (T > 1) lane_store(pre, (size_t)k, acc);
  }
  fp_t inv = block_inv<LSG_ITEMS_PER_BLOCK>(H, I, l, acc);  // every lane pair is a leaf (one when idle)
#pragma unroll 1
  for (int64_t k = last - 1; k >= first; k--) {
    const fp_t x = lane_load<fp_t>(in, (size_t)k);
    const bool z = zero_to_one && fp_is_zero(x);
    const fp_t r = k > first ? fp_mul(inv, lane_load<fp_t>(pre, (size_t)k - 1)) : inv;
    lane_store(out, (size_t)k, z ? fp_zero() : r);
    if (k > first && !z) inv = fp_mul(inv, x);
  }
}

// partials: canonical big-endian 576-byte Fp12 blobs <-> lane form (one item each)
__global__ void LSG_KERNEL_ATTR k_blobs_to_fp12(int n, const uint8_t* __restrict__ blobs, uint32_t* __restrict__ out) {
  LANE_ITEM(n);
  (void)lead;
  lane_store(out, item, fp12_from_canon_bytes(blobs + 576 * item));
}
__global__ void LSG_KERNEL_ATTR k_fp12_to_canon(int n, const uint32_t* __restrict__ in, uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  (void)lead;
  fp12_to_canon_bytes(out + 576 * item, lane_load<fp12_t>(in, item));
}

// f^r for a nonzero 64-bit r (square-and-multiply, one item): the partial of a package group
// that is one set verified unscaled leaves the slot as f^r, so that FE(product of partials) is
// the RLC check prod_i e_i^(r_i) whatever the other partials are (FE(f^r) = FE(f)^r)
__global__ void LSG_KERNEL_ATTR_W(1) k_fp12_pow_u64(const uint8_t* __restrict__ in576, uint64_t r,
                                                    uint8_t* __restrict__ out576) {
  LANE_ITEM(1);
  (void)lead;
  const fp12_t f = fp12_from_canon_bytes(in576);
  fp12_t acc = f;
  int top = 63;
  while (top > 0 && !((r >> top) & 1u)) top--;
#pragma unroll 1
  for (int b = top - 1; b >= 0; b--) {
    acc = fp12_sqr(acc);
    if ((r >> b) & 1u) acc = fp12_mul(acc, f);
  }
  fp12_to_canon_bytes(out576, acc);
}

// parity hook of the Fp2 product leaf (pair_fp2_mul_v: the SOP form) at its lazy bounds: per
// item, c0 + c1 u = (a0 + a1 u)(b0 + b1 u) R^-1 from four raw pair-layout operands, stored raw
// (not reduced, not canonical) so that the test checks the value and the leaf's output bound
__global__ void LSG_KERNEL_ATTR k_check_fp2_mul(int n, const uint32_t* __restrict__ in, uint32_t* __restrict__ out) {
  LANE_ITEM(n);
  (void)lead;
  const fp2_t a(lane_load<fp_t>(in, 4 * item), lane_load<fp_t>(in, 4 * item + 1));
  const fp2_t b(lane_load<fp_t>(in, 4 * item + 2), lane_load<fp_t>(in, 4 * item + 3));
  const fp2_t c = fp2_mul(a, b);
  lane_store(out, 2 * item, c.c0);
  lane_store(out, 2 * item + 1, c.c1);
}

// roofline probe: 4 independent limb-parallel Montgomery chains per pair
__global__ void LSG_KERNEL_ATTR k_probe_fp_mul(int n, int iters, uint32_t* __restrict__ io) {
  LANE_ITEM(n);
  (void)lead;
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

namespace lsgk {
hipError_t seg_reduce(hipStream_t st, int op, int n_chunks, int ips_log2, const int32_t* chunks, const int32_t* idx,
                      const uint32_t* src, uint32_t* dst, uint32_t* tmp) {
  const size_t items = (size_t)n_chunks << ips_log2;
  if (op == 0) LSG_LAUNCH_ITEMS(k_seg_reduce<0>, items, st, n_chunks, ips_log2, chunks, idx, src, dst, tmp);
  if (op == 1) LSG_LAUNCH_ITEMS(k_seg_reduce<1>, items, st, n_chunks, ips_log2, chunks, idx, src, dst, tmp);
  LSG_LAUNCH_ITEMS(k_seg_reduce<2>, items, st, n_chunks, ips_log2, chunks, idx, src, dst, tmp);
}
hipError_t binv_fold(hipStream_t st, int n, int zero_to_one, const uint32_t* in, uint32_t* pre, uint32_t* tot) {
  LSG_LAUNCH_ITEMS(k_binv_fold, (n + LSG_BINV_T - 1) / LSG_BINV_T, st, n, zero_to_one, in, pre, tot);
}
hipError_t binv_block(hipStream_t st, int n, int T, int zero_to_one, const uint32_t* in, uint32_t* pre, uint32_t* out) {
  if (n <= 0) return hipSuccess;
  const size_t chunks = ((size_t)n + T - 1) / T;
  hipLaunchKernelGGL(k_binv_block, dim3(lane_blocks(chunks)), dim3(LSG_TPB), 0, st, n, T, zero_to_one, in, pre, out);
  return hipGetLastError();
}
hipError_t binv_root(hipStream_t st, const uint32_t* top, uint32_t* inv) {
  LSG_LAUNCH_ITEMS(k_binv_root, 1, st, top, inv);
}
hipError_t binv_unfold(hipStream_t st, int n, int zero_to_one, const uint32_t* in, const uint32_t* pre,
                       const uint32_t* tinv, uint32_t* out) {
  LSG_LAUNCH_ITEMS(k_binv_unfold, (n + LSG_BINV_T - 1) / LSG_BINV_T, st, n, zero_to_one, in, pre, tinv, out);
}
hipError_t blobs_to_fp12(hipStream_t st, int n, const uint8_t* blobs, uint32_t* out) {
  LSG_LAUNCH_ITEMS(k_blobs_to_fp12, n, st, n, blobs, out);
}
hipError_t fp12_to_canon(hipStream_t st, int n, const uint32_t* in, uint8_t* out576) {
  LSG_LAUNCH_ITEMS(k_fp12_to_canon, n, st, n, in, out576);
}
hipError_t fp12_pow_u64(hipStream_t st, const uint8_t* in576, uint64_t r, uint8_t* out576) {
  LSG_LAUNCH_ITEMS(k_fp12_pow_u64, 1, st, in576, r, out576);
}
hipError_t check_fp2_mul(hipStream_t st, int n, const uint32_t* in, uint32_t* out) {
  LSG_LAUNCH_ITEMS(k_check_fp2_mul, n, st, n, in, out);
}
hipError_t probe_fp_mul(hipStream_t st, int items, int iters, uint32_t* io) {
  LSG_LAUNCH_ITEMS(k_probe_fp_mul, items, st, items, iters, io);
}
hipError_t probe_mad(hipStream_t st, int blocks, int iters, uint32_t seed, uint64_t* io) {
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_probe_mad, dim3(blocks), dim3(256), 0, st, iters, seed, io);
  return hipGetLastError();
}
}  // namespace lsgk
