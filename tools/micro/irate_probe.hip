// Issue cost of the integer VALU instructions in the pair backend's Montgomery leaf
// (lsg_fp_pair.hpp pair_mont_mul: v_mad_i64_i32, v_mul_lo_u32, v_mov_b32_dpp, v_and_b32,
// v_lshl_add_u64, v_ashrrev_i64, v_cndmask_b32) on gfx950: SIMD cycles per wave-instruction,
// from 8 independent chains per lane at 8 waves per SIMD (throughput, not latency).
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/irate_probe.hip -o tools/micro/irate_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048
#define BODY8(ins)                                     \
  asm volatile(ins : "+v"(a0) : "v"(x), "v"(y) : "s40", "s41"); \
  asm volatile(ins : "+v"(a1) : "v"(x), "v"(y) : "s40", "s41"); \
  asm volatile(ins : "+v"(a2) : "v"(x), "v"(y) : "s40", "s41"); \
  asm volatile(ins : "+v"(a3) : "v"(x), "v"(y) : "s40", "s41"); \
  asm volatile(ins : "+v"(a4) : "v"(x), "v"(y) : "s40", "s41"); \
  asm volatile(ins : "+v"(a5) : "v"(x), "v"(y) : "s40", "s41"); \
  asm volatile(ins : "+v"(a6) : "v"(x), "v"(y) : "s40", "s41"); \
  asm volatile(ins : "+v"(a7) : "v"(x), "v"(y) : "s40", "s41")

// 64-bit accumulator forms: "+v"(uint64_t)
template <int KIND>
__global__ void __launch_bounds__(256) k64(uint32_t seed, uint64_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3, a4 = t + 4, a5 = t + 5, a6 = t + 6, a7 = t + 7;
  uint32_t x = t * 2654435761u ^ seed, y = seed | 1u;
  for (int i = 0; i < ITERS; i++) {
    if (KIND == 0) {
      BODY8("v_mad_i64_i32 %0, s[40:41], %1, %2, %0");
    } else if (KIND == 1) {
      BODY8("v_mad_u64_u32 %0, s[40:41], %1, %2, %0");
    } else if (KIND == 2) {
      BODY8("v_lshl_add_u64 %0, %0, 1, %0");
    } else {
      BODY8("v_ashrrev_i64 %0, 29, %0");
    }
  }
  out[t] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int KIND>
__global__ void __launch_bounds__(256) k32(uint32_t seed, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3, a4 = t + 4, a5 = t + 5, a6 = t + 6, a7 = t + 7;
  uint32_t x = t * 2654435761u ^ seed, y = seed | 1u;
  for (int i = 0; i < ITERS; i++) {
    if (KIND == 0) {
      BODY8("v_mul_lo_u32 %0, %0, %1");
    } else if (KIND == 1) {
      BODY8("v_mov_b32_dpp %0, %1 quad_perm:[0,0,2,2] row_mask:0xf bank_mask:0xf");
    } else if (KIND == 2) {
      BODY8("v_and_b32 %0, %0, %1");
    } else if (KIND == 3) {
      BODY8("v_mul_u32_u24 %0, %0, %1");
    } else {
      BODY8("v_add_u32 %0, %0, %1");
    }
  }
  out[t] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <class K, class T>
void run(const char* name, K kern, T* buf, int blocks, double clk_ghz, int simds) {
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, 1u, buf);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, 0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, 3u, buf);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double wave_instr = (double)blocks * 4 * ITERS * 8;  // 4 waves per block
  const double simd_cycles = ms * 1e-3 * clk_ghz * 1e9 * simds;
  printf("%-16s %8.3f ms  %.2f SIMD cycles per wave-instruction\n", name, ms, simd_cycles / wave_instr);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * 8;  // 8 waves per SIMD
  const double clk = p.clockRate / 1e6;           // GHz
  const int simds = p.multiProcessorCount * 4;
  printf("%s  %d CUs  %.3f GHz\n", p.gcnArchName, p.multiProcessorCount, clk);
  uint64_t* b64;
  uint32_t* b32;
  hipMalloc(&b64, sizeof(uint64_t) * blocks * 256);
  hipMalloc(&b32, sizeof(uint32_t) * blocks * 256);
  run("v_mad_i64_i32", k64<0>, b64, blocks, clk, simds);
  run("v_mad_u64_u32", k64<1>, b64, blocks, clk, simds);
  run("v_lshl_add_u64", k64<2>, b64, blocks, clk, simds);
  run("v_ashrrev_i64", k64<3>, b64, blocks, clk, simds);
  run("v_mul_lo_u32", k32<0>, b32, blocks, clk, simds);
  run("v_mov_b32_dpp", k32<1>, b32, blocks, clk, simds);
  run("v_and_b32", k32<2>, b32, blocks, clk, simds);
  run("v_mul_u32_u24", k32<3>, b32, blocks, clk, simds);
  run("v_add_u32", k32<4>, b32, blocks, clk, simds);
  hipFree(b64);
  hipFree(b32);
  return 0;
}
