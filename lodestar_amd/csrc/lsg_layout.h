// lsg_layout.h -- HBM layout of the lane-form values the kernels exchange, visible to the
// host orchestration (lsg_host.hip) without the math headers.
//
// Every per-set kernel runs the pair backend (lsg_fp_pair.hpp): one Fp is 14 signed
// radix-2^29 limbs over a lane pair, so one Fp of one work item is 14 u32 words in global
// memory.  Item-major storage: word k of item i lives at mem[(i * W + k) * 2 + h] for lane h
// of the pair (lane_load / lane_store).  The kernel translation units static_assert these
// sizes against lane_words<T>() of the backend they are built on.
#pragma once
#include <stddef.h>

namespace lsgl {
constexpr size_t W_FP = 14;          // u32 words per item: one Fp
constexpr size_t W_G1A = 2 * W_FP;   // affine G1 (x, y)
constexpr size_t W_TAB = 32;         // a pubkey-table row: affine G1 padded to one 128-byte line
constexpr size_t W_G1P = 3 * W_FP;   // projective G1 (X : Y : Z)
constexpr size_t W_G2A = 4 * W_FP;   // affine G2 over Fp2
constexpr size_t W_G2P = 6 * W_FP;   // projective G2
constexpr size_t W_F12 = 12 * W_FP;  // Fp12 (Miller values)
constexpr size_t W_H2CU = 4 * W_FP;  // hash_to_field output (u0, u1 in Fp2)
constexpr size_t W_LINE = 6 * W_FP;  // an unevaluated Miller line (3 Fp2)
constexpr int ML_STEPS = 68;         // lines per Miller loop: 63 doublings + 5 additions for |x|
constexpr int MSM_WINDOWS = 8;       // bucket MSM of the RLC signature sums: 8-bit windows of r_i
constexpr int MSM_DIGITS = 255;      // nonzero digits per window
constexpr int MSM_BITS = 64;         // per-bit sums C_k, S = sum_k 2^k C_k
}  // namespace lsgl
#define LSG_BINV_T 16  // values per lane pair in one level of the batched inversion
