// Dev microbenchmark (not product): throughput of the two Fp backends on gfx950.
//   mad     : raw v_mad_u64_u32 issue rate (8 independent chains per thread)
//   elem    : thread-per-element 12-limb CIOS Montgomery product (lsg_fp_elem.hpp)
//   elem_ml : thread-per-element Miller loop (register pressure / spill check)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lodestar_amd/csrc tools/micro/thru_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "lsg_fp_elem.hpp"
#include "lsg_h2c.hpp"
#include "lsg_pairing.hpp"

__global__ void __launch_bounds__(256) k_mad(int iters, uint64_t* io) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc[8];
  uint32_t a = t * 2654435761u + 1, b = t ^ 0x9e3779b9u;
#pragma unroll
  for (int k = 0; k < 8; k++) acc[k] = t + k;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      acc[k] = (uint64_t)(a + k) * (b ^ (uint32_t)i) + acc[k];
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= acc[k];
  io[t] = s;
}

template <int CH>
__global__ void __launch_bounds__(256) k_elem_mul(int iters, uint32_t* io) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fp_t a[CH];
#pragma unroll
  for (int k = 0; k < CH; k++) {
    a[k] = fp_t(FP_R2);
    a[k].l[0] ^= t + k;
  }
  fp_t b = fp_t(FP_R3);
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < CH; k++) a[k] = fp_mul(a[k], b);
  }
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; k++)
    for (int j = 0; j < 12; j++) s ^= a[k].l[j];
  io[t] = s;
}

__global__ void __launch_bounds__(256) k_elem_ml(uint32_t* io) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  g1a_t P;
  P.x = fp_t(G1_GEN_X);
  P.y = fp_t(G1_GEN_Y);
  P.x.l[0] ^= t & 1;
  g2a_t Q;
  Q.x = fp2_t(fp_t(FP_R2), fp_t(FP_R3));
  Q.y = fp2_t(fp_t(FP_R3), fp_t(FP_R2));
  fp12_t f = miller_loop(P, Q);
  io[t] = f.c0.c0.c0.l[0] ^ f.c1.c2.c1.l[11];
}

int main() {
  int blocks = 256 * 8, tpb = 256;
  size_t n = (size_t)blocks * tpb;
  uint64_t* io64;
  uint32_t* io;
  hipMalloc(&io64, n * 8);
  hipMalloc(&io, n * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float ms;
  int iters = 4096;
  for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(a);
    hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(tpb), 0, 0, iters, io64);
    hipEventRecord(b);
    hipEventSynchronize(b);
  }
  hipEventElapsedTime(&ms, a, b);
  printf("mad: %.3f ms  %.3e v_mad_u64_u32/s\n", ms, (double)n * iters * 8 / (ms * 1e-3));
  iters = 64;
  for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(a);
    hipLaunchKernelGGL(k_elem_mul<4>, dim3(blocks), dim3(tpb), 0, 0, iters, io);
    hipEventRecord(b);
    hipEventSynchronize(b);
  }
  hipEventElapsedTime(&ms, a, b);
  printf("elem_mul4 (%d blocks): %.3f ms  %.3e fp_mul/s\n", blocks, ms, (double)n * iters * 4 / (ms * 1e-3));
  for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(a);
    hipLaunchKernelGGL(k_elem_mul<1>, dim3(blocks), dim3(tpb), 0, 0, iters, io);
    hipEventRecord(b);
    hipEventSynchronize(b);
  }
  hipEventElapsedTime(&ms, a, b);
  printf("elem_mul1 (%d blocks): %.3f ms  %.3e fp_mul/s\n", blocks, ms, (double)n * iters * 1 / (ms * 1e-3));
  int mlb[] = {16, 64, 256, 1024};
  for (int q = 0; q < 4; q++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k_elem_ml, dim3(mlb[q]), dim3(tpb), 0, 0, io);
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    hipEventElapsedTime(&ms, a, b);
    printf("elem_miller_loop %6d pairs: %.3f ms  %.3e pairs/s\n", mlb[q] * tpb, ms, mlb[q] * tpb / (ms * 1e-3));
  }
  return 0;
}
