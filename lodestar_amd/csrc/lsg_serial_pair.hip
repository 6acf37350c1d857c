// lsg_serial_pair.hip -- the per-group serial stages (final exponentiation, blst finalverify;
// the signature-side Miller loop ML(-G1, S_g); Horner over the MSM bit sums + that loop) on
// the PAIR backend (lsg_fp_pair.hpp: one Fp per lane pair, 7 x 29-bit limbs per lane).
// Under packages/beacon-node/src/chain/bls/maybeBatch.ts:18,37.
//
// Built twice (lsg_serial.h picks by group count):
//   LSG_PAIR_SPLIT (this file)    one group per wave: every lane pair holds the group's
//       state and each batch of independent products is split over the 32 lane pairs
//       (fp_mul_list) -- the latency build, for the few groups of a clean package.  A product
//       on a lane pair is ~390 instructions issued back to back; on a 16-lane row (the row
//       backend, lsg_serial.hip) it is a latency-bound DPP chain of ~2 us.
//   lsg_serial_pair_wide.hip      one group per lane pair, 32 per wave, no replicated work
//       -- the throughput build, for the thousands of per-job groups of a fallback phase.
// Inputs and outputs are the canonical byte blobs of lsg_io.hpp, as for the row kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lsg_serial.h"

#ifndef LSG_PAIR_WIDE
#define LSG_PAIR_SPLIT 1
#define LSG_PAIR_FN(x) x##_ps
#else
#define LSG_PAIR_FN(x) x##_pw
#endif

namespace {
#include "lsg_fp_pair.hpp"
#include "lsg_io.hpp"
}  // namespace

#define LSG_PS_TPB 64
#ifdef LSG_PAIR_SPLIT
#define PAIR_ITEM() ((int)blockIdx.x)                        // one group per wave
#define PAIR_LEAD() (__lane_id() == 0)
static int pair_blocks(int n) { return n; }
#else
#define PAIR_ITEM() ((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 1))  // one group per lane pair
#define PAIR_LEAD() ((threadIdx.x & 1) == 0)
static int pair_blocks(int n) { return (2 * n + LSG_PS_TPB - 1) / LSG_PS_TPB; }
#endif

// a wave's lane pairs past the last group run group ng-1's data and store nothing (the split
// build needs every lane of the wave in its batches)
#define PAIR_GROUP(ng)        \
  const int g0 = PAIR_ITEM(); \
  const bool live = g0 < (ng);  \
  const int item = live ? g0 : (ng) - 1

__global__ void __launch_bounds__(LSG_PS_TPB) __attribute__((amdgpu_waves_per_eu(1)))
LSG_PAIR_FN(k_pair_final_exp)(int ng, const uint8_t* __restrict__ F576, int32_t* __restrict__ verdict) {
  PAIR_GROUP(ng);
  const bool one = fp12_is_one(final_exp(fp12_from_canon_bytes(F576 + 576 * (size_t)item)));
  if (live && PAIR_LEAD()) verdict[item] = one ? 1 : 0;
}

LSG_DEVI fp12_t pair_neg_g1_loop(const g2p_t& s) {
  fp12_t r = fp12_one();
  if (!proj_is_inf(s)) {
    g1a_t ng1;
    ng1.x = fp_t(G1_GEN_X);
    ng1.y = fp_t(G1_GEN_NEG_Y);
    r = miller_loop(ng1, proj_to_aff(s));
  }
  return r;
}

__global__ void __launch_bounds__(LSG_PS_TPB) __attribute__((amdgpu_waves_per_eu(1)))
LSG_PAIR_FN(k_pair_miller_neg_g1)(int ng, const uint8_t* __restrict__ S288, uint8_t* __restrict__ out576) {
  PAIR_GROUP(ng);
  (void)live;  // pairs past the end rewrite group ng-1's bytes with the same values
  fp12_to_canon_bytes(out576 + 576 * (size_t)item, pair_neg_g1_loop(g2p_from_canon_bytes(S288 + 288 * (size_t)item)));
}

// S_g = sum_k 2^k C_{g,k} by Horner over the 64 per-bit sums, then ML(-G1, S_g)
__global__ void __launch_bounds__(LSG_PS_TPB) __attribute__((amdgpu_waves_per_eu(1)))
LSG_PAIR_FN(k_pair_horner_miller)(int ng, const uint8_t* __restrict__ C288, uint8_t* __restrict__ out576) {
  PAIR_GROUP(ng);
  const uint8_t* c = C288 + (size_t)288 * 64 * item;
  g2p_t s = g2p_from_canon_bytes(c + 288 * 63);
#pragma unroll 1
  for (int k = 62; k >= 0; k--) s = g2_add(g2_dbl(s), g2p_from_canon_bytes(c + 288 * k));
  (void)live;
  fp12_to_canon_bytes(out576 + 576 * (size_t)item, pair_neg_g1_loop(s));
}

#define PAIR_LAUNCH(kern, ng, st, ...)                                                                  \
  do {                                                                                              \
    if ((ng) <= 0) return hipSuccess;                                                               \
    hipLaunchKernelGGL(LSG_PAIR_FN(kern), dim3(pair_blocks(ng)), dim3(LSG_PS_TPB), 0, st, __VA_ARGS__); \
    return hipGetLastError();                                                                       \
  } while (0)

hipError_t LSG_PAIR_FN(lsg_pair_final_exp)(hipStream_t st, int ng, const uint8_t* F576, int32_t* verdict) {
  PAIR_LAUNCH(k_pair_final_exp, ng, st, ng, F576, verdict);
}
hipError_t LSG_PAIR_FN(lsg_pair_miller_neg_g1)(hipStream_t st, int ng, const uint8_t* S288, uint8_t* out576) {
  PAIR_LAUNCH(k_pair_miller_neg_g1, ng, st, ng, S288, out576);
}
hipError_t LSG_PAIR_FN(lsg_pair_horner_miller)(hipStream_t st, int ng, const uint8_t* C288, uint8_t* out576) {
  PAIR_LAUNCH(k_pair_horner_miller, ng, st, ng, C288, out576);
}
