// Shared macros and the constant-literal types of the BLS12-381 field code.
//
// Field elements have two device representations ("backends") behind one API:
//   lsg_fp_elem.hpp  one thread owns a whole Fp (12 x u32 limbs in registers);
//                    used by the host build of the math (tests/native/hostcheck.hip)
//   lsg_fp_lane.hpp  one 16-lane DPP row owns an Fp, lane j holding limb j (lanes 12..15
//                    are zero); the gfx950 product kernels use this one.
// The tower, curve, hash-to-curve and pairing code (lsg_tower.hpp ... lsg_pairing.hpp) is
// written once against that API.  Constants are emitted as fpc_t / fp2c_t literals
// (tools/gen_constants.py) and convert implicitly to either backend's fp_t / fp2_t.
#pragma once
#include <stdint.h>

#define LSG_INL __host__ __device__ __forceinline__
#define LSG_NOINL __host__ __device__ __noinline__
#define LSG_DEVI __device__ __forceinline__
#define LSG_DEVNOINL __device__ __noinline__
#define LSG_CONST static constexpr

// limbs per constant literal: 12 x 32-bit (quad / row / element backends) or 14 x 29-bit
// (pair backend; lsg_constants_r29.hpp defines LSG_NLIMBS before including this file)
#ifndef LSG_NLIMBS
#define LSG_NLIMBS 12
#endif
struct fpc_t {
  uint32_t l[LSG_NLIMBS];
};
struct fp2c_t {
  fpc_t c0, c1;
};
