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
// The same stages as straight-line programs (lsg_slp.hip, tools/gen_slp.py): one group per
// workgroup, each step's independent products spread over the lane pairs.
hipError_t lsg_slp_final_exp(hipStream_t st, int ng, const uint8_t* F576, int32_t* verdict);
hipError_t lsg_slp_miller_neg_g1(hipStream_t st, int ng, const uint8_t* S288, uint8_t* out576);
hipError_t lsg_slp_horner_miller(hipStream_t st, int ng, const uint8_t* C288, uint8_t* out576);
// hash_to_G2's cofactor clearing and affine conversion: Hp (projective lane form, the SSWU
// map's Q0 + Q1) -> H (affine lane form), hinf
hipError_t lsg_slp_h2c_clear(hipStream_t st, int n, const uint32_t* Hp, uint32_t* H, uint8_t* hinf);
// signature side of small packages: G2 membership (k_sig_subgroup's contract) and [r_i] sig_i
// (k_sig_scale's: mode selects the sets, r_i = 0 leaves a point unscaled)
hipError_t lsg_slp_g2_subgroup(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, int32_t* err);
hipError_t lsg_slp_g2_scale(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, const int32_t* err,
                            const uint8_t* pinf, const uint64_t* rnd, const uint8_t* mode, uint32_t* out);
// Miller items of one set each (lane-form P, pinf, hinf, err, H as for k_miller_fused):
// f[item] = ML(P_i, H_i) of set item_first[item], 1 for a set that does not take part
hipError_t lsg_slp_miller_items1(hipStream_t st, int n_items, const int32_t* item_first, const uint32_t* P,
                                 const uint8_t* pinf, const uint8_t* hinf, const int32_t* err, const uint32_t* H,
                                 uint32_t* f);
// The straight-line programs run the serial stages.  The row kernels above are compiled only
// into the A/B build (liblodestar_bls_ab.so, -DLSG_AB; lsg_ab.h), where env LSG_SERIAL=row
// selects them; the shipped library has no runtime switch here.
#include "lsg_ab.h"
enum { LSG_SERIAL_SLP = 0, LSG_SERIAL_ROW = 1 };
#ifdef LSG_AB
static inline int lsg_serial_mode() {
  static const int v = lsg_ab_str_is("LSG_SERIAL", "row") ? (int)LSG_SERIAL_ROW : (int)LSG_SERIAL_SLP;
  return v;
}
#define LSG_SERIAL_PICK(name, ng, ...)                                                                  \
  (lsg_serial_mode() == LSG_SERIAL_SLP                                                                   \
       ? lsg_slp_##name(__VA_ARGS__)                                                                     \
       : ((ng) >= LSG_ROW_WIDE_MIN ? lsg_row_##name##_r1(__VA_ARGS__) : lsg_row_##name##_r4(__VA_ARGS__)))
#else
static constexpr int lsg_serial_mode() { return LSG_SERIAL_SLP; }
#define LSG_SERIAL_PICK(name, ng, ...) lsg_slp_##name(__VA_ARGS__)
#endif
static inline hipError_t lsg_row_final_exp(hipStream_t st, int ng, const uint8_t* F576, int32_t* verdict) {
  return LSG_SERIAL_PICK(final_exp, ng, st, ng, F576, verdict);
}
static inline hipError_t lsg_row_miller_neg_g1(hipStream_t st, int ng, const uint8_t* S288, uint8_t* out576) {
  return LSG_SERIAL_PICK(miller_neg_g1, ng, st, ng, S288, out576);
}
static inline hipError_t lsg_row_horner_miller(hipStream_t st, int ng, const uint8_t* C288, uint8_t* out576) {
  return LSG_SERIAL_PICK(horner_miller, ng, st, ng, C288, out576);
}
