// Launchers of the per-group serial stages, built with the row backend (lsg_serial.hip):
// one final exponentiation or one signature Miller loop is a single long dependency chain,
// and a 16-lane row finishes it in about a third of the time a 4-lane quad needs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// verdict[g] = (FE(F_g) == 1) for ng canonical 576-byte Fp12 blobs
hipError_t lsg_row_final_exp(hipStream_t st, int ng, const uint8_t* F576, int32_t* verdict);
// out576[g] = ML(-G1, S_g) for ng canonical 288-byte projective G2 points (1 if S_g = O)
hipError_t lsg_row_miller_neg_g1(hipStream_t st, int ng, const uint8_t* S288, uint8_t* out576);
// out576[g] = ML(-G1, sum_k 2^k C_{g,k}) for ng groups of 64 canonical 288-byte projective G2
// points each (the bucket MSM's per-bit sums): Horner and the Miller loop in one row chain
hipError_t lsg_row_horner_miller(hipStream_t st, int ng, const uint8_t* C288, uint8_t* out576);
