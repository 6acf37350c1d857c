// Dev microbenchmark (not product): thread-per-element 381-bit Montgomery products on
// gfx950, to choose the per-set Fp backend.  (The quad backend's rate is
// lsg_probe_fp_mul_rate in the library: 2.86e10 Fp-mul/s on MI355X,
// profiles/r01_bench_default.jsonl.)
//   elem_c   12 x 32-bit limbs, operand-scanning CIOS in plain C (lsg_fp_elem.hpp's host fp_mul)
//   elem_ps  12 x 32-bit limbs, product scanning: every partial product is one
//            v_mad_u64_u32 into a 64-bit column accumulator whose carry-out is counted by one
//            v_addc_co_u32 (inline asm)
//   r29      14 x 29-bit limbs, product scanning; column sums stay below 2^64, so every term
//            is exactly one v_mad_u64_u32 (R = 2^406, outputs < 2p, no final subtraction)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/probe_fpmul.hip -o tools/micro/fpmul_probe
// Run:   tools/micro/fpmul_probe [iters]; tools/micro/check_fpmul.py checks the SAMPLE lines.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static constexpr uint32_t P32[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                                     0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
static constexpr uint32_t N0P32 = 0xfffcfffdu;

struct f12 {
  uint32_t l[12];
};
struct f14 {
  uint32_t l[14];
};

// ---------------------------------------------------------------- elem_c
__device__ __noinline__ f12 mul_c(f12 a, f12 b) {
  uint32_t t[12];
  for (int j = 0; j < 12; j++) t[j] = 0;
  for (int i = 0; i < 12; i++) {
    uint64_t s = (uint64_t)a.l[0] * b.l[i] + t[0];
    t[0] = (uint32_t)s;
    uint64_t A = s >> 32;
    uint32_t m = t[0] * N0P32;
    uint64_t C = ((uint64_t)m * P32[0] + t[0]) >> 32;
    for (int j = 1; j < 12; j++) {
      s = (uint64_t)a.l[j] * b.l[i] + t[j] + A;
      A = s >> 32;
      uint64_t s2 = (uint64_t)m * P32[j] + (uint32_t)s + C;
      t[j - 1] = (uint32_t)s2;
      C = s2 >> 32;
    }
    t[11] = (uint32_t)(C + A);
  }
  f12 r, s;
  uint32_t br = 0;
  for (int i = 0; i < 12; i++) s.l[i] = __builtin_subc(t[i], P32[i], br, &br);
  for (int i = 0; i < 12; i++) r.l[i] = br ? t[i] : s.l[i];
  return r;
}

// ---------------------------------------------------------------- elem_ps
// acc (64-bit) += x * y; ov += carry out of the 64-bit accumulation (y in a VGPR or an SGPR)
#define MADC(acc, ov, x, y, ycons)                                             \
  do {                                                                         \
    uint64_t cy_;                                                              \
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_addc_co_u32 %1, %2, 0, %1, %2" \
        : "+v"(acc), "+v"(ov), "=&s"(cy_)                                      \
        : "v"(x), ycons(y));                                                   \
  } while (0)

__device__ __noinline__ f12 mul_ps(f12 a, f12 b) {
  uint32_t m[12], r[12];
  uint64_t acc = 0;
  uint32_t ov = 0;
#pragma unroll
  for (int k = 0; k < 12; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) MADC(acc, ov, a.l[i], b.l[k - i], "v");
#pragma unroll
    for (int i = 0; i < k; i++) MADC(acc, ov, m[i], P32[k - i], "s");
    m[k] = (uint32_t)acc * N0P32;
    MADC(acc, ov, m[k], P32[0], "s");
    acc = (acc >> 32) | ((uint64_t)ov << 32);
    ov = 0;
  }
#pragma unroll
  for (int k = 12; k < 23; k++) {
#pragma unroll
    for (int i = k - 11; i < 12; i++) MADC(acc, ov, a.l[i], b.l[k - i], "v");
#pragma unroll
    for (int i = k - 11; i < 12; i++) MADC(acc, ov, m[i], P32[k - i], "s");
    r[k - 12] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)ov << 32);
    ov = 0;
  }
  r[11] = (uint32_t)acc;  // the result is < 2p < 2^382: nothing above limb 11
  f12 o, s;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s.l[i] = __builtin_subc(r[i], P32[i], br, &br);
#pragma unroll
  for (int i = 0; i < 12; i++) o.l[i] = br ? r[i] : s.l[i];
  return o;
}

// ---------------------------------------------------------------- r29
static constexpr uint32_t M29 = (1u << 29) - 1;
struct p29_t {
  uint32_t l[14];
};
static constexpr p29_t make_p29() {
  p29_t r{};
  for (int k = 0; k < 14; k++) {
    uint32_t v = 0;
    for (int b = 0; b < 29; b++) {
      int bit = 29 * k + b;
      if (bit < 384 && ((P32[bit / 32] >> (bit % 32)) & 1u)) v |= 1u << b;
    }
    r.l[k] = v;
  }
  return r;
}
static constexpr p29_t P29 = make_p29();
static constexpr uint32_t make_n0p29() {  // -p^-1 mod 2^29
  uint32_t x = 1;
  for (int i = 0; i < 6; i++) x = x * (2u - P29.l[0] * x);
  return (0u - x) & M29;
}
static constexpr uint32_t N0P29 = make_n0p29();

__device__ __noinline__ f14 mul_r29(f14 a, f14 b) {
  uint32_t m[14];
  f14 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 14; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * P29.l[k - i];
    m[k] = ((uint32_t)acc * N0P29) & M29;
    acc += (uint64_t)m[k] * P29.l[0];
    acc >>= 29;
  }
#pragma unroll
  for (int k = 14; k < 27; k++) {
#pragma unroll
    for (int i = k - 13; i < 14; i++) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = k - 13; i < 14; i++) acc += (uint64_t)m[i] * P29.l[k - i];
    r.l[k - 14] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  r.l[13] = (uint32_t)acc;
  return r;
}


// ---------------------------------------------------------------- pair29
// 14 x 29-bit limbs over a lane PAIR: lane h (0/1) holds limbs 7h..7h+6 and the matching
// seven 64-bit CIOS accumulators.  Per step: b_i and m are DPP broadcasts inside the pair;
// the retiring accumulator is split into its carry (into the next accumulator, same lane)
// and its low 29 bits (moved one lane down by DPP), so only one 32-bit value crosses lanes
// per step and no carry bookkeeping is needed.
struct h7 {
  uint32_t l[7];
};
template <int CTRL>
__device__ __forceinline__ uint32_t pdpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
}
__device__ __noinline__ h7 mul_pair(h7 a, h7 b) {
  const bool hi = __lane_id() & 1u;
  uint32_t p[7];
#pragma unroll
  for (int j = 0; j < 7; j++) p[j] = hi ? P29.l[7 + j] : P29.l[j];
  uint64_t t[7];
#pragma unroll
  for (int j = 0; j < 7; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const uint32_t bs = b.l[i % 7];
    const uint32_t bi = i < 7 ? pdpp<0xA0>(bs) : pdpp<0xF5>(bs);
#pragma unroll
    for (int j = 0; j < 7; j++) t[j] += (uint64_t)a.l[j] * bi;
    const uint32_t m = pdpp<0xA0>(((uint32_t)t[0] * N0P29) & M29);
#pragma unroll
    for (int j = 0; j < 7; j++) t[j] += (uint64_t)m * p[j];
    const uint64_t c = t[0] >> 29;
    uint32_t mv = pdpp<0xF5>((uint32_t)t[0] & M29);
    mv = hi ? 0u : mv;
#pragma unroll
    for (int j = 0; j < 6; j++) t[j] = t[j + 1];
    t[0] += c;
    t[6] = mv;
  }
  // normalise: in-lane carries, lane 0's carry-out into lane 1, in-lane carries again
#pragma unroll
  for (int j = 0; j < 6; j++) {
    t[j + 1] += t[j] >> 29;
    t[j] &= M29;
  }
  uint32_t co = pdpp<0xA0>((uint32_t)(t[6] >> 29));
  t[6] = hi ? t[6] : (t[6] & M29);
  t[0] += hi ? co : 0u;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    t[j + 1] += t[j] >> 29;
    t[j] &= M29;
  }
  h7 r;
#pragma unroll
  for (int j = 0; j < 7; j++) r.l[j] = (uint32_t)t[j];
  return r;
}

template <int WPE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE)))
k_rate_pair(int iters, const f14* __restrict__ in, f14* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t e = t >> 1;
  const int h = (int)(t & 1);
  h7 v[4];
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int j = 0; j < 7; j++) v[k].l[j] = in[4 * e + k].l[7 * h + j];
  for (int k = 0; k < iters; k++) {
    v[0] = mul_pair(v[0], v[1]);
    v[1] = mul_pair(v[1], v[2]);
    v[2] = mul_pair(v[2], v[3]);
    v[3] = mul_pair(v[3], v[0]);
  }
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int j = 0; j < 7; j++) out[4 * e + k].l[7 * h + j] = v[k].l[j];
}

// ---------------------------------------------------------------- rate kernels: 4 chains/thread
template <class F, F (*MUL)(F, F), int WPE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE)))
k_rate(int iters, const F* __restrict__ in, F* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  F a = in[4 * t], b = in[4 * t + 1], c = in[4 * t + 2], d = in[4 * t + 3];
  for (int k = 0; k < iters; k++) {
    a = MUL(a, b);
    b = MUL(b, c);
    c = MUL(c, d);
    d = MUL(d, a);
  }
  out[4 * t] = a;
  out[4 * t + 1] = b;
  out[4 * t + 2] = c;
  out[4 * t + 3] = d;
}

template <class F>
static void fill(F* h, size_t n, int limbs, int bits) {
  uint64_t s = 0x1234567890abcdefull;
  for (size_t i = 0; i < n; i++)
    for (int k = 0; k < limbs; k++) {
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      uint32_t v = (uint32_t)(s >> 32);
      if (bits < 32) v &= (1u << bits) - 1;
      if (k == limbs - 1) v &= (bits == 32 ? 0x0fffffffu : 0x7u);  // value < p
      h[i].l[k] = v;
    }
}

template <class F, F (*MUL)(F, F), int WPE>
struct LaunchElem {
  static constexpr int lanes = 1;
  static void go(int blocks, int iters, const F* i, F* o) { k_rate<F, MUL, WPE><<<blocks, 64>>>(iters, i, o); }
};
template <int WPE>
struct LaunchPair {
  static constexpr int lanes = 2;
  static void go(int blocks, int iters, const f14* i, f14* o) { k_rate_pair<WPE><<<blocks, 64>>>(iters, i, o); }
};

template <class F, class L>
static void run(const char* name, int limbs, int bits, int iters, int waves_per_simd) {
  int dev;
  CHECK(hipGetDevice(&dev));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, dev));
  const int blocks = prop.multiProcessorCount * 4 * waves_per_simd;  // one wave per block
  const size_t threads = (size_t)blocks * 64 / L::lanes, n = 4 * threads;  // threads = elements per chain
  F* h = (F*)malloc(n * sizeof(F));
  fill(h, n, limbs, bits);
  F *din, *dout;
  CHECK(hipMalloc(&din, n * sizeof(F)));
  CHECK(hipMalloc(&dout, n * sizeof(F)));
  CHECK(hipMemcpy(din, h, n * sizeof(F), hipMemcpyHostToDevice));
  L::go(blocks, 1, din, dout);  // correctness sample: one iteration
  CHECK(hipDeviceSynchronize());
  F* o = (F*)malloc(n * sizeof(F));
  CHECK(hipMemcpy(o, dout, n * sizeof(F), hipMemcpyDeviceToHost));
  for (int s = 0; s < 2; s++) {  // a' = a b, b' = b c, c' = c d, d' = d a'
    printf("SAMPLE %s %d", name, limbs);
    for (int k = 0; k < 4; k++) {
      printf(" ");
      for (int j = limbs - 1; j >= 0; j--) printf("%08x", h[4 * s + k].l[j]);
    }
    for (int k = 0; k < 4; k++) {
      printf(" ");
      for (int j = limbs - 1; j >= 0; j--) printf("%08x", o[4 * s + k].l[j]);
    }
    printf("\n");
  }
  L::go(blocks, iters, din, dout);  // warm
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  L::go(blocks, iters, din, dout);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  double muls = 4.0 * threads * iters;
  printf("RATE %-8s waves/SIMD %d  %.4g fp_mul/s  (%.3f ms, %zu threads, %d iters)\n", name, waves_per_simd,
         muls / (ms * 1e-3), ms, threads, iters);
  fflush(stdout);
  free(h);
  free(o);
  CHECK(hipFree(din));
  CHECK(hipFree(dout));
}

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 256;
  run<f12, LaunchElem<f12, mul_c, 2>>("elem_c", 12, 32, iters, 2);
  run<f12, LaunchElem<f12, mul_c, 4>>("elem_c", 12, 32, iters, 4);
  run<f12, LaunchElem<f12, mul_ps, 1>>("elem_ps", 12, 32, iters, 1);
  run<f12, LaunchElem<f12, mul_ps, 2>>("elem_ps", 12, 32, iters, 2);
  run<f12, LaunchElem<f12, mul_ps, 4>>("elem_ps", 12, 32, iters, 4);
  run<f14, LaunchElem<f14, mul_r29, 2>>("r29", 14, 29, iters, 2);
  run<f14, LaunchElem<f14, mul_r29, 4>>("r29", 14, 29, iters, 4);
  run<f14, LaunchPair<1>>("pair29", 14, 29, iters, 1);
  run<f14, LaunchPair<2>>("pair29", 14, 29, iters, 2);
  run<f14, LaunchPair<4>>("pair29", 14, 29, iters, 4);
  run<f14, LaunchPair<8>>("pair29", 14, 29, iters, 8);
  return 0;
}
