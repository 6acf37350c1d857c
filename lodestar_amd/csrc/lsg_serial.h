// Launchers of the per-group serial stages, built with the row backend (lsg_serial.hip):
// one final exponentiation or one signature Miller loop is a single long dependency chain,
// and a 16-lane row finishes it in about a third of the time a 4-lane quad needs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Two builds of each stage: _r4 (the four rows of a wave share one item and split its product
// batches: latency) and _r1 (one item per row, four per wave: no replicated work).  From
// LSG_ROW_WIDE_MIN groups on -- a fallback phase's per-job groups -- the _r1 build runs.
#ifndef LSG_ROW_WIDE_MIN
#define LSG_ROW_WIDE_MIN 512
#endif
#define LSG_ROW_DECL(name, ...)                      \
  hipError_t name##_r4(hipStream_t st, __VA_ARGS__); \
  hipError_t name##_r1(hipStream_t st, __VA_ARGS__);
// verdict[g] = (FE(F_g) == 1) for ng canonical 576-byte Fp12 blobs
LSG_ROW_DECL(lsg_row_final_exp, int ng, const uint8_t* F576, int32_t* verdict)
// out576[g] = ML(-G1, S_g) for ng canonical 288-byte projective G2 points (1 if S_g = O)
LSG_ROW_DECL(lsg_row_miller_neg_g1, int ng, const uint8_t* S288, uint8_t* out576)
// out576[g] = ML(-G1, sum_k 2^k C_{g,k}) for ng groups of 64 canonical 288-byte projective G2
// points each (the bucket MSM's per-bit sums): Horner and the Miller loop in one row chain
LSG_ROW_DECL(lsg_row_horner_miller, int ng, const uint8_t* C288, uint8_t* out576)
inline hipError_t lsg_row_final_exp(hipStream_t st, int ng, const uint8_t* F576, int32_t* verdict) {
  return ng >= LSG_ROW_WIDE_MIN ? lsg_row_final_exp_r1(st, ng, F576, verdict) : lsg_row_final_exp_r4(st, ng, F576, verdict);
}
inline hipError_t lsg_row_miller_neg_g1(hipStream_t st, int ng, const uint8_t* S288, uint8_t* out576) {
  return ng >= LSG_ROW_WIDE_MIN ? lsg_row_miller_neg_g1_r1(st, ng, S288, out576)
                                : lsg_row_miller_neg_g1_r4(st, ng, S288, out576);
}
inline hipError_t lsg_row_horner_miller(hipStream_t st, int ng, const uint8_t* C288, uint8_t* out576) {
  return ng >= LSG_ROW_WIDE_MIN ? lsg_row_horner_miller_r1(st, ng, C288, out576)
                                : lsg_row_horner_miller_r4(st, ng, C288, out576);
}
