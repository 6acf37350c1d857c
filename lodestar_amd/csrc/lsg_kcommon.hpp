// lsg_kcommon.hpp -- shared prologue of the per-set kernel translation units (lsg_k_*.hip).
//
// Every per-set kernel runs the pair backend (lsg_fp_pair.hpp): one field element per lane
// pair, so one work item (a set, a pubkey, a Miller item) is one pair and a wave64 carries
// 32 items.  The math headers sit in an anonymous namespace: lsg_serial.hip instantiates the
// same generic code over the row backend and the two fp_t must never meet at link time.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lodestar_bls.h"
#include "lsg_launch.h"
#include "lsg_layout.h"

namespace {
#include "lsg_fp_pair.hpp"
#include "lsg_h2c.hpp"
#include "lsg_io.hpp"
#include "lsg_inv.hpp"  // block_inv's divstep root (below)

static_assert(lane_words<fp_t>() == lsgl::W_FP, "layout: Fp");
static_assert(lane_words<g1a_t>() == lsgl::W_G1A, "layout: G1 affine");
static_assert(lane_words<g1p_t>() == lsgl::W_G1P, "layout: G1 projective");
static_assert(lane_words<g2a_t>() == lsgl::W_G2A, "layout: G2 affine");
static_assert(lane_words<g2p_t>() == lsgl::W_G2P, "layout: G2 projective");
static_assert(lane_words<fp12_t>() == lsgl::W_F12, "layout: Fp12");
static_assert(lane_words<line_t>() == lsgl::W_LINE, "layout: line");
static_assert(ML_STEPS == lsgl::ML_STEPS, "layout: Miller steps");
}  // namespace

#define LSG_TPB 256  // threads per block: 128 lane-pair items
// Register budget: waves per SIMD the compiler must leave room for (it spills beyond that).
// 2 waves (256 VGPRs) for the pair backend: 1.32M vs 1.15M sets/s at 3.
#ifndef LSG_WAVES_PER_EU
#define LSG_WAVES_PER_EU 2
#endif
#define LSG_KERNEL_ATTR __launch_bounds__(LSG_TPB) __attribute__((amdgpu_waves_per_eu(LSG_WAVES_PER_EU)))
// kernels whose live state does not fit 256 registers: at 1 wave per SIMD a wave owns 512
// (VGPRs + AGPRs) instead of spilling
#define LSG_KERNEL_ATTR_W(w) __launch_bounds__(LSG_TPB) __attribute__((amdgpu_waves_per_eu(w)))
#define LSG_ITEMS_PER_BLOCK (LSG_TPB / LSG_GROUP)

// A value parked in LDS for the thread's own use: word k of thread t at l[k * LSG_TPB + t]
// (consecutive lanes, consecutive banks).  Long-lived points of the per-set kernels wait here
// across the leaf calls instead of spilling to scratch.
template <class T>
static __device__ __forceinline__ void lds_park(uint32_t* l, const T& v) {
  constexpr int W = sizeof(T) / 4;
  uint32_t w[W];
  __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
  for (int k = 0; k < W; k++) l[k * LSG_TPB + threadIdx.x] = w[k];
}
template <class T>
static __device__ __forceinline__ T lds_unpark(const uint32_t* l) {
  constexpr int W = sizeof(T) / 4;
  uint32_t w[W];
#pragma unroll
  for (int k = 0; k < W; k++) w[k] = l[k * LSG_TPB + threadIdx.x];
  T v;
  __builtin_memcpy(&v, w, sizeof(T));
  return v;
}

// v from lane (lane id ^ lane_mask), word by word
template <class T>
static __device__ __forceinline__ T shfl_xor_t(const T& v, int lane_mask) {
  constexpr int W = sizeof(T) / 4;
  uint32_t w[W];
  __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
  for (int k = 0; k < W; k++) w[k] = (uint32_t)__shfl_xor((int)w[k], lane_mask, 64);
  T r;
  __builtin_memcpy(&r, w, sizeof(T));
  return r;
}

static __device__ __forceinline__ size_t gtid() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }
#define LANE_ITEM(n)                        \
  lsg_lane_setup();                         \
  const size_t item = gtid() / LSG_GROUP;   \
  if (item >= (size_t)(n)) return;          \
  const bool lead = (threadIdx.x % LSG_GROUP) == 0

// The LDS heap of a fold group of G leaves (nodes G..2G-1; node 1 = the product of all):
// lane pair `leaf` (< 0: none) contributes v.  Every thread of the block calls it.
template <int G>
static __device__ __forceinline__ void heap_up(uint32_t* Hg, int leaf, const fp_t& v) {
  if (leaf >= 0) lane_store(Hg, G + leaf, v);
#pragma unroll 1
  for (int w = G / 2; w >= 1; w >>= 1) {
    __syncthreads();
    if (leaf >= 0 && leaf < w)
      lane_store(Hg, w + leaf, fp_mul(lane_load<fp_t>(Hg, 2 * (w + leaf)), lane_load<fp_t>(Hg, 2 * (w + leaf) + 1)));
  }
  __syncthreads();
}
// ... and down: Ig[1] (set by the caller) = 1 / Hg[1]; leaves' inverses in Ig[G..2G-1]
template <int G>
static __device__ __forceinline__ void heap_down(const uint32_t* Hg, uint32_t* Ig, int leaf) {
#pragma unroll 1
  for (int w = 2; w <= G; w <<= 1) {
    __syncthreads();
    if (leaf < w) {
      const int i = w + leaf;
      lane_store(Ig, i, fp_mul(lane_load<fp_t>(Ig, i >> 1), lane_load<fp_t>(Hg, i ^ 1)));
    }
  }
  __syncthreads();
}

// every participating lane pair's 1 / v: heap up, the root inverted (lane pair 0, divsteps),
// heap down.  G leaves; every thread of the block calls it; H, I: 2G-node LDS heaps.
template <int G>
static __device__ __forceinline__ fp_t block_inv(uint32_t* H, uint32_t* I, int leaf, const fp_t& v) {
  heap_up<G>(H, leaf, v);
  if (leaf == 0) {
    const fp_t d = pair_inv_gcd(pair_canon(lane_load<fp_t>(H, 1)));  // (x R)^-1 as an integer
    lane_store(I, 1, pair_mont_mul(d, fp_t(FP_RCUBE)));                // x^-1 R
  }
  heap_down<G>(H, I, leaf < 0 ? G : leaf);
  return leaf >= 0 ? lane_load<fp_t>(I, G + leaf) : v;
}

static inline int lane_blocks(size_t items) { return (int)((items + LSG_ITEMS_PER_BLOCK - 1) / LSG_ITEMS_PER_BLOCK); }

// launch `kern` over `items` lane-pair items on `st` (nothing for 0 items)
#define LSG_LAUNCH_ITEMS(kern, items, st, ...)                                                      \
  do {                                                                                              \
    if ((items) <= 0) return hipSuccess;                                                            \
    hipLaunchKernelGGL(kern, dim3(lane_blocks((size_t)(items))), dim3(LSG_TPB), 0, st, __VA_ARGS__); \
    return hipGetLastError();                                                                       \
  } while (0)
