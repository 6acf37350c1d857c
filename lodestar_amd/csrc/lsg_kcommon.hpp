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

static inline int lane_blocks(size_t items) { return (int)((items + LSG_ITEMS_PER_BLOCK - 1) / LSG_ITEMS_PER_BLOCK); }

// launch `kern` over `items` lane-pair items on `st` (nothing for 0 items)
#define LSG_LAUNCH_ITEMS(kern, items, st, ...)                                                      \
  do {                                                                                              \
    if ((items) <= 0) return hipSuccess;                                                            \
    hipLaunchKernelGGL(kern, dim3(lane_blocks((size_t)(items))), dim3(LSG_TPB), 0, st, __VA_ARGS__); \
    return hipGetLastError();                                                                       \
  } while (0)
