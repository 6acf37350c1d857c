// lsg_serial.hip -- the per-group serial stages with the row backend (one Fp per 16-lane DPP
// row, lsg_fp_lane.hpp): the final exponentiation (blst finalverify, under
// packages/beacon-node/src/chain/bls/maybeBatch.ts:18,37) and the signature-side Miller loop
// ML(-G1, sum r_i sig_i) of an RLC batch.  There is one such item per batch, so its latency
// is what counts: a row spreads each Montgomery product over 16 lanes and finishes the chain
// about three times sooner than the quad backend the per-set kernels use.  Inputs and outputs
// are canonical byte blobs (lsg_io.hpp).  All math is in an anonymous namespace so that this
// translation unit's fp_t and the quad one's never meet at link time.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lsg_serial.h"

// Built twice: lsg_serial.hip (LSG_ROWS_PER_ITEM 4, the rows of a wave share one item: latency
// for the few groups of a clean package) and lsg_serial_wide.hip (1: four items per wave, no
// replicated work, for the thousands of per-job groups of a fallback phase); lsg_serial.h
// picks by the number of groups.
#ifndef LSG_ROWS_PER_ITEM
#define LSG_ROWS_PER_ITEM 4
#endif
#if LSG_ROWS_PER_ITEM == 4
#define LSG_ROW_FN(x) x##_r4
#else
#define LSG_ROW_FN(x) x##_r1
#endif

namespace {
#include "lsg_fp_lane.hpp"
#include "lsg_io.hpp"
}  // namespace

#define LSG_ROW_TPB 64  // one wave: LSG_ROWS_PER_ITEM rows per item, 4 / LSG_ROWS_PER_ITEM items
#define ROW_ITEM() ((int)((blockIdx.x * blockDim.x + threadIdx.x) / (16 * LSG_ROWS_PER_ITEM)))

__global__ void __launch_bounds__(LSG_ROW_TPB) LSG_ROW_FN(k_row_final_exp)(int ng, const uint8_t* __restrict__ F576,
                                                               int32_t* __restrict__ verdict) {
  lsg_lane_setup();
  const int item = ROW_ITEM();
  if (item >= ng) return;
  bool one = fp12_is_one(final_exp(fp12_from_canon_bytes(F576 + 576 * (size_t)item)));
  if ((threadIdx.x & 15) == 0) verdict[item] = one ? 1 : 0;
}

__global__ void __launch_bounds__(LSG_ROW_TPB) LSG_ROW_FN(k_row_miller_neg_g1)(int ng, const uint8_t* __restrict__ S288,
                                                                   uint8_t* __restrict__ out576) {
  lsg_lane_setup();
  const int item = ROW_ITEM();
  if (item >= ng) return;
  g2p_t s = g2p_from_canon_bytes(S288 + 288 * (size_t)item);
  fp12_t r = fp12_one();
  if (!proj_is_inf(s)) {
    g1a_t ng1;
    ng1.x = fp_t(G1_GEN_X);
    ng1.y = fp_t(G1_GEN_NEG_Y);
    r = miller_loop(ng1, proj_to_aff(s));
  }
  fp12_to_canon_bytes(out576 + 576 * (size_t)item, r);
}

// The bucket MSM's last step fused with the signature Miller loop: S_g = sum_k 2^k C_{g,k}
// by Horner over the group's 64 per-bit sums (63 doublings + 63 additions, complete
// formulas), then ML(-G1, S_g).  Both are single dependency chains, so they run on rows.
__global__ void __launch_bounds__(LSG_ROW_TPB) LSG_ROW_FN(k_row_horner_miller)(int ng, const uint8_t* __restrict__ C288,
                                                                   uint8_t* __restrict__ out576) {
  lsg_lane_setup();
  const int item = ROW_ITEM();
  if (item >= ng) return;
  const uint8_t* c = C288 + (size_t)288 * 64 * item;
  g2p_t s = g2p_from_canon_bytes(c + 288 * 63);
#pragma unroll 1
  for (int k = 62; k >= 0; k--) s = g2_add(g2_dbl(s), g2p_from_canon_bytes(c + 288 * k));
  fp12_t r = fp12_one();
  if (!proj_is_inf(s)) {
    g1a_t ng1;
    ng1.x = fp_t(G1_GEN_X);
    ng1.y = fp_t(G1_GEN_NEG_Y);
    r = miller_loop(ng1, proj_to_aff(s));
  }
  fp12_to_canon_bytes(out576 + 576 * (size_t)item, r);
}

static int row_blocks(int n) { return (n * 16 * LSG_ROWS_PER_ITEM + LSG_ROW_TPB - 1) / LSG_ROW_TPB; }

hipError_t LSG_ROW_FN(lsg_row_final_exp)(hipStream_t st, int ng, const uint8_t* F576, int32_t* verdict) {
  if (ng <= 0) return hipSuccess;
  hipLaunchKernelGGL(LSG_ROW_FN(k_row_final_exp), dim3(row_blocks(ng)), dim3(LSG_ROW_TPB), 0, st, ng, F576, verdict);
  return hipGetLastError();
}

hipError_t LSG_ROW_FN(lsg_row_miller_neg_g1)(hipStream_t st, int ng, const uint8_t* S288, uint8_t* out576) {
  if (ng <= 0) return hipSuccess;
  hipLaunchKernelGGL(LSG_ROW_FN(k_row_miller_neg_g1), dim3(row_blocks(ng)), dim3(LSG_ROW_TPB), 0, st, ng, S288, out576);
  return hipGetLastError();
}

hipError_t LSG_ROW_FN(lsg_row_horner_miller)(hipStream_t st, int ng, const uint8_t* C288, uint8_t* out576) {
  if (ng <= 0) return hipSuccess;
  hipLaunchKernelGGL(LSG_ROW_FN(k_row_horner_miller), dim3(row_blocks(ng)), dim3(LSG_ROW_TPB), 0, st, ng, C288, out576);
  return hipGetLastError();
}
