// Dev microbenchmark (not product): where the time of a straight-line-program step goes, on
// the real final-exponentiation program (lsg_slp_progs.h).  Variants of the interpreter loop
// of lsg_slp.hip, one workgroup, cycles per step (s_memtime):
//   0 the loop as in lsg_slp.hip        1 entries fetched, no gather (one product per step)
//   2 gather + carry, no product        3 loop + entry fetch only
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I lodestar_amd/csrc tools/micro/slp_fe_probe.hip -o tools/micro/slp_fe_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "lsg_fp_pair.hpp"
#include "lsg_slp_exec.hpp"
#define LSG_SLP_ARRAY __device__ const
#include "lsg_slp_progs.h"

template <int VAR>
__global__ void __launch_bounds__(64) k_fe(const uint8_t* in, uint32_t* sink, long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t tid = threadIdx.x, h = tid & 1u, q = tid >> 1;
  for (uint32_t j = q; j < LSG_SLP_FINAL_EXP_N_SLOTS; j += 32) slot_store(lds, j, h, fp_from_arr(lsg_slp_final_exp_consts));
  __syncthreads();
  const uint32_t* ops = lsg_slp_final_exp_ops;
  const uint32_t* steps = lsg_slp_final_exp_steps;
  const long long t0 = clock64();
  uint32_t d = steps[0];
  uint4 e0 = make_uint4(0, 0, 0, 0), e1 = e0;
  if (q < (d & 255u)) {
    const uint4* e = (const uint4*)(ops + 8 * ((d >> 16) + q));
    e0 = e[0];
    e1 = e[1];
  }
  fp_t acc = fp_t(FP_R2);
#pragma unroll 1
  for (int s = 0; s < LSG_SLP_FINAL_EXP_N_STEPS; s++) {
    const uint32_t dn = steps[s + 1];
    uint4 f0 = make_uint4(0, 0, 0, 0), f1 = f0;
    if (q < (dn & 255u)) {
      const uint4* e = (const uint4*)(ops + 8 * ((dn >> 16) + q));
      f0 = e[0];
      f1 = e[1];
    }
    if (q < (d & 255u)) {
      const uint32_t ew[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
      if (VAR == 0) {
        slp_exec(lds, ew, in, h, d);
      } else if (VAR == 1) {
        fp_t r;
        pair_mont_mul_n<1>(&r, &acc, &acc);
        acc = r;
        slot_store(lds, ew[0] & 1023u, h, r);
      } else if (VAR == 2) {
        slp_exec(lds, ew, in, h, d & ~(1u << 15));  // products off: LIN path only
      } else {
        slot_store(lds, ew[0] & 1023u, h, fp_from_arr(ew));
      }
    }
    __syncthreads();
    d = dn;
    e0 = f0;
    e1 = f1;
  }
  const long long t1 = clock64();
  fp_t o = slot_load(lds, q, h);
  for (int j = 0; j < LSG_PL; j++) sink[threadIdx.x * LSG_PL + j] = o.l[j] + acc.l[j];
  if (threadIdx.x == 0) cyc[VAR] = t1 - t0;
}

int main() {
  uint8_t* in;
  uint32_t* sink;
  long long* cyc;
  hipMalloc(&in, 4096);
  hipMemset(in, 1, 4096);
  hipMalloc(&sink, 64 * 64 * 4);
  hipMalloc(&cyc, 64 * 8);
  const size_t shm = LSG_SLP_FINAL_EXP_N_SLOTS * LSG_SLP_STRIDE * 4;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_fe<0>, dim3(1), dim3(64), shm, 0, in, sink, cyc);
    hipLaunchKernelGGL(k_fe<1>, dim3(1), dim3(64), shm, 0, in, sink, cyc);
    hipLaunchKernelGGL(k_fe<2>, dim3(1), dim3(64), shm, 0, in, sink, cyc);
    hipLaunchKernelGGL(k_fe<3>, dim3(1), dim3(64), shm, 0, in, sink, cyc);
    hipDeviceSynchronize();
  }
  long long t[4];
  hipMemcpy(t, cyc, sizeof t, hipMemcpyDeviceToHost);
  const char* nm[4] = {"full step", "fetch + one product", "gather + carry (no product)", "loop + fetch"};
  for (int v = 0; v < 4; v++)
    printf("%-30s %7.0f cycles/step  (%d steps, %.3f ms at 2.4 GHz)\n", nm[v], (double)t[v] / LSG_SLP_FINAL_EXP_N_STEPS,
           LSG_SLP_FINAL_EXP_N_STEPS, t[v] / 2.4e6);
  return 0;
}
