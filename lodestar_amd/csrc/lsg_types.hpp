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

struct fpc_t {
  uint32_t l[12];
};
struct fp2c_t {
  fpc_t c0, c1;
};
