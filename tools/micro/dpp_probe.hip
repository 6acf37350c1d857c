// Dev microbenchmark (not product): DPP row semantics + v_mad_u64_u32 throughput on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("ERR %s %s\n",#x,hipGetErrorString(e)); return 1;}}while(0)

__global__ void k_dpp(int* out) {
  int l = threadIdx.x;
  int v = l * 10;
  out[l]       = __builtin_amdgcn_update_dpp(-1, v, 0x101, 0xf, 0xf, false); // row_shl:1
  out[64 + l]  = __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xf, 0xf, false); // row_shr:1
  out[128 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x153, 0xf, 0xf, false); // row_newbcast:3
  out[192 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x121, 0xf, 0xf, false); // row_ror:1
  out[256 + l] = __builtin_amdgcn_update_dpp(0, v, 0x101, 0xf, 0xf, true);   // row_shl:1 bound_ctrl
}

__global__ void k_mad(int iters, uint64_t* io) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = (uint32_t)io[i], b = (uint32_t)(io[i] >> 32);
  uint64_t c0 = a, c1 = b, c2 = a ^ b, c3 = a + b, c4 = a - b, c5 = a * 3, c6 = b * 5, c7 = a * 7;
  for (int k = 0; k < iters; k++) {
    c0 = (uint64_t)(uint32_t)c0 * a + c1; c1 = (uint64_t)(uint32_t)c1 * b + c2;
    c2 = (uint64_t)(uint32_t)c2 * a + c3; c3 = (uint64_t)(uint32_t)c3 * b + c4;
    c4 = (uint64_t)(uint32_t)c4 * a + c5; c5 = (uint64_t)(uint32_t)c5 * b + c6;
    c6 = (uint64_t)(uint32_t)c6 * a + c7; c7 = (uint64_t)(uint32_t)c7 * b + c0;
  }
  io[i] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

__global__ void k_add(int iters, uint32_t* io) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = io[i], b = a * 3, c = a * 5, d = a * 7, e = a ^ 9, f = a ^ 13, g = a + 1, h = a + 2;
  for (int k = 0; k < iters; k++) {
    a += b; b += c; c += d; d += e; e += f; f += g; g += h; h += a;
    a ^= h; b ^= g; c ^= f; d ^= e;
  }
  io[i] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}

int main() {
  int* d; CHK(hipMalloc(&d, 320 * 4));
  hipLaunchKernelGGL(k_dpp, dim3(1), dim3(64), 0, 0, d);
  int h[320]; CHK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  const char* nm[5] = {"row_shl:1", "row_shr:1", "row_newbcast:3", "row_ror:1", "row_shl:1 bc"};
  for (int r = 0; r < 5; r++) { printf("%-16s", nm[r]); for (int l = 0; l < 20; l++) printf(" %d", h[r*64+l]); printf("\n"); }
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  int threads = p.multiProcessorCount * 2048;
  uint64_t* m; CHK(hipMalloc(&m, threads * 8)); CHK(hipMemset(m, 7, threads * 8));
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  int iters = 4096;
  hipLaunchKernelGGL(k_mad, dim3(threads / 256), dim3(256), 0, 0, 16, m);
  hipEventRecord(a); hipLaunchKernelGGL(k_mad, dim3(threads / 256), dim3(256), 0, 0, iters, m); hipEventRecord(b);
  hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b);
  double mads = (double)threads * iters * 8;
  printf("v_mad_u64_u32: %.3e /s (%.1f ms)  = %.2f per CU per clk @2.4GHz\n", mads / (ms * 1e-3), ms, mads / (ms * 1e-3) / p.multiProcessorCount / 2.4e9);
  uint32_t* q; CHK(hipMalloc(&q, threads * 4)); CHK(hipMemset(q, 3, threads * 4));
  hipLaunchKernelGGL(k_add, dim3(threads / 256), dim3(256), 0, 0, 16, q);
  hipEventRecord(a); hipLaunchKernelGGL(k_add, dim3(threads / 256), dim3(256), 0, 0, iters, q); hipEventRecord(b);
  hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
  double ops = (double)threads * iters * 12;
  printf("v_add/xor_u32: %.3e /s (%.1f ms) = %.2f per CU per clk @2.4GHz\n", ops / (ms * 1e-3), ms, ops / (ms * 1e-3) / p.multiProcessorCount / 2.4e9);
  return 0;
}
