// Dev microbenchmark (not product): single-wave latency (cycles) of lane-backend primitives.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "lsg_fp_lane.hpp"
#include "lsg_h2c.hpp"
#include "lsg_pairing.hpp"

#define ITER 64
__global__ void k_lat(uint32_t* io, long long* cyc) {
  lsg_lane_setup();
  fp_t a = lane_load<fp_t>(io, threadIdx.x >> 4), b = fp_t(FP_R2);
  fp2_t x(a, b), y(b, a);
  fp12_t f;
  f.c0 = fp6_make(x, y, x);
  f.c1 = fp6_make(y, x, y);
  long long t[12];
  int k = 0;
  t[k++] = clock64();
  for (int i = 0; i < ITER; i++) a = fp_mul(a, b);
  t[k++] = clock64();
  for (int i = 0; i < ITER; i++) a = fp_add(a, b);
  t[k++] = clock64();
  for (int i = 0; i < ITER; i++) a = fp_sub(a, b);
  t[k++] = clock64();
  for (int i = 0; i < ITER; i++) { fp_t r[9], xs[9], ys[9]; for (int q = 0; q < 9; q++) { xs[q] = a; ys[q] = b; } fp_mul9(r, xs, ys); a = r[0]; b = r[8]; }
  t[k++] = clock64();
  for (int i = 0; i < ITER; i++) x = fp2_mul(x, y);
  t[k++] = clock64();
  for (int i = 0; i < 8; i++) f = fp12_mul(f, f);
  t[k++] = clock64();
  for (int i = 0; i < 8; i++) f = fp12_cyclotomic_sqr(f);
  t[k++] = clock64();
  for (int i = 0; i < 8; i++) f = fp12_mul_line(f, x, y, x);
  t[k++] = clock64();
  g2p_t T = proj_from_aff(g2a_t{x, y});
  for (int i = 0; i < 8; i++) { line_t L = ml_dbl_step(T, a, b); x = L.l00; }
  t[k++] = clock64();
  for (int i = 0; i < 8; i++) T = g2_add(T, T);
  t[k++] = clock64();
  lane_store(io, threadIdx.x >> 4, fp_add(fp_add(a, x.c0), fp_add(f.c0.c0.c0, T.X.c1)));
  if (threadIdx.x == 0) for (int i = 0; i < k; i++) cyc[i] = t[i];
}

int main() {
  uint32_t* io; long long* cyc;
  hipMalloc(&io, 64 * 16 * 4); hipMemset(io, 1, 64 * 16 * 4);
  hipMalloc(&cyc, 16 * 8);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, io, cyc);
    hipDeviceSynchronize();
  }
  long long h[16]; hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[] = {"fp_mul", "fp_add", "fp_sub", "fp_mul9(9 muls)", "fp2_mul", "fp12_mul", "fp12_cyclo_sqr", "fp12_mul_line", "ml_dbl_step", "g2_add"};
  int per[] = {ITER, ITER, ITER, ITER, ITER, 8, 8, 8, 8, 8};
  for (int i = 0; i < 10; i++) printf("%-18s %8.1f cycles/op\n", nm[i], (double)(h[i + 1] - h[i]) / per[i]);
  return 0;
}
