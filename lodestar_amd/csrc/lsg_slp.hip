// lsg_slp.hip -- the per-group serial stages as straight-line programs (tools/gen_slp.py):
// the final exponentiation (blst finalverify under packages/beacon-node/src/chain/bls/
// maybeBatch.ts:18,37), the signature-side Miller loop ML(-G1, S_g) of an RLC group and the
// bucket MSM's Horner fused with that loop.
//
// One group per workgroup of W waves.  The program's values live in LDS slots (64 bytes: the
// pair backend's 7 limbs per lane, lsg_fp_pair.hpp, padded to 8 words); a step holds up to
// 32 W independent operations and lane pair q of the workgroup executes operation q:
//   gather its operand forms (up to 7 slots each, 64-bit accumulation of coef * limb, one
//   carry round), then LIN: store their sum; MUL: store the Montgomery product; LOADMUL:
//   the product of the item's input Fp #j (read from global memory) with its B form.
// A dependency chain of ~10^4 products thus runs in ~10^3 steps of one product each, where
// the row kernels (lsg_serial.hip) spend ~2 us per dependent product.  Inputs and outputs are
// the canonical byte blobs of lsg_io.hpp, exactly as for the row kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lsg_serial.h"
#include "../../include/lodestar_bls.h"

namespace {
#include "lsg_fp_pair.hpp"
#include "lsg_slp_exec.hpp"
}  // namespace

#define LSG_SLP_ARRAY __device__ const
#include "lsg_slp_progs.h"
#include "lsg_layout.h"
// lane-form words per lane of one item (lsg_layout.h counts both lanes of the pair)
constexpr size_t lsgl_w_g1a = lsgl::W_G1A / 2, lsgl_w_g2a = lsgl::W_G2A / 2, lsgl_w_g2p = lsgl::W_G2P / 2,
                 lsgl_w_f12 = lsgl::W_F12 / 2;

namespace {

// s_waitcnt vmcnt(0) with expcnt and lgkmcnt left at their maxima (gfx9 encoding)
#define LSG_WAIT_VMCNT0 0x0F70

enum { SLP_FE = 0, SLP_ML = 1, SLP_HORNER = 2, SLP_ITEM1 = 3, SLP_H2C_CLEAR = 4, SLP_G2_SUBGROUP = 5, SLP_G2_SCALE = 6 };

template <int PROG, int W>
struct Prog;
#define LSG_SLP_PROG_W(ID, W, NAME, UP)                                                \
  template <>                                                                          \
  struct Prog<ID, W> {                                                                 \
    static constexpr int n_steps = LSG_SLP_##UP##_W##W##_N_STEPS;                      \
    static constexpr int n_slots = LSG_SLP_##UP##_W##W##_N_SLOTS;                      \
    static constexpr int n_consts = LSG_SLP_##UP##_W##W##_N_CONSTS;                    \
    static constexpr int n_in = LSG_SLP_##UP##_W##W##_N_IN;                            \
    static constexpr int n_load = LSG_SLP_##UP##_W##W##_N_LOAD;                        \
    static constexpr int n_out = LSG_SLP_##UP##_W##W##_N_OUT;                          \
    static __device__ const uint32_t* ops() { return lsg_slp_##NAME##_w##W##_ops; }     \
    static __device__ const uint32_t* steps() { return lsg_slp_##NAME##_w##W##_steps; } \
    static __device__ const uint32_t* consts() { return lsg_slp_##NAME##_w##W##_consts; } \
    static __device__ const uint16_t* in() { return lsg_slp_##NAME##_w##W##_in; }       \
    static __device__ const uint16_t* out() { return lsg_slp_##NAME##_w##W##_out; }     \
  };
#define LSG_SLP_PROG(ID, NAME, UP) LSG_SLP_PROG_W(ID, 1, NAME, UP) LSG_SLP_PROG_W(ID, 2, NAME, UP)
LSG_SLP_PROG(SLP_FE, final_exp, FINAL_EXP)
LSG_SLP_PROG(SLP_ML, miller_neg_g1, MILLER_NEG_G1)
LSG_SLP_PROG(SLP_HORNER, horner_miller, HORNER_MILLER)
LSG_SLP_PROG(SLP_ITEM1, miller_item1, MILLER_ITEM1)
LSG_SLP_PROG(SLP_H2C_CLEAR, h2c_clear, H2C_CLEAR)
LSG_SLP_PROG(SLP_G2_SUBGROUP, g2_subgroup, G2_SUBGROUP)
LSG_SLP_PROG(SLP_G2_SCALE, g2_scale, G2_SCALE)

// the program's steps (inputs and constants already in their slots): in every step lane pair
// q executes operation q; the next step's descriptor and this lane pair's entry of it are in
// flight while the current step computes (the program lives in global memory / L2)
template <class PR>
__device__ __forceinline__ void slp_steps(uint32_t* lds, const uint8_t* inp, uint32_t q, uint32_t h) {
#if LSG_SLP_PRIO  // A/B builds: issue priority of the programs' waves over co-resident kernels'
  __builtin_amdgcn_s_setprio(LSG_SLP_PRIO);
#endif
  const uint32_t* ops = PR::ops();
  const uint32_t* steps = PR::steps();
  uint32_t d = steps[0];
  uint4 e0 = make_uint4(0, 0, 0, 0), e1 = e0;
  if (q < (d & 255u)) {
    const uint4* e = (const uint4*)(ops + 8 * ((d >> 16) + q));
    e0 = e[0];
    e1 = e[1];
  }
  // the first entry is complete before the loop: otherwise the wait-count pass merges the
  // loop header's two predecessors and makes every step wait for its own prefetch of the
  // next entry (vmcnt(0) at the top of the step), exposing one L2 round trip per step
  __builtin_amdgcn_s_waitcnt(LSG_WAIT_VMCNT0);
#pragma unroll 1
  for (int s = 0; s < PR::n_steps; s++) {
    const uint32_t dn = steps[s + 1];  // (a zero sentinel follows the last step)
    uint4 f0 = make_uint4(0, 0, 0, 0), f1 = f0;
    if (q < (dn & 255u)) {
      const uint4* e = (const uint4*)(ops + 8 * ((dn >> 16) + q));
      f0 = e[0];
      f1 = e[1];
    }
    if (q < (d & 255u)) {
      const uint32_t ew[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
      slp_exec(lds, ew, inp, h, d);
    }
    __syncthreads();
    d = dn;
    e0 = f0;
    e1 = f1;
  }
}
template <class PR>
__device__ __forceinline__ void slp_consts(uint32_t* lds, uint32_t q, uint32_t h, uint32_t nq) {
  for (uint32_t j = q; j < (uint32_t)PR::n_consts; j += nq) {
    const uint32_t* c = PR::consts() + 14 * j + 7 * h;
    fp_t v;
#pragma unroll
    for (int k = 0; k < 7; k++) v.l[k] = c[k];
    slot_store(lds, j, h, v);
  }
}

// MODE: 0 = verdict (outputs == Fp12 one), 1 = Fp12 blob with the S = O test (outputs 12, 13
// are S.Z: the group's term is 1 when S is the point at infinity)
template <int PROG, int W, int MODE>
__global__ void __launch_bounds__(64 * W) k_slp(int n_items, const uint8_t* __restrict__ in, uint32_t in_stride,
                                                uint8_t* __restrict__ out, int32_t* __restrict__ verdict) {
  using PR = Prog<PROG, W>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int item = blockIdx.x;
  if (item >= n_items) return;
  const uint32_t tid = threadIdx.x, h = tid & 1u, q = tid >> 1;
  constexpr uint32_t NQ = 32 * W;
  const uint8_t* inp = in + (size_t)in_stride * item;
  slp_consts<PR>(lds, q, h, NQ);
  for (uint32_t j = q; j < (uint32_t)PR::n_in; j += NQ) slot_store(lds, PR::in()[j], h, fp_from_be_bytes(inp + 48 * j, 12));
  __syncthreads();
  slp_steps<PR>(lds, inp, q, h);
  // outputs: canonical values; lane pair j holds output j (n_out <= 32 W)
  static_assert(PR::n_out <= 32, "one output per lane pair of the first wave");
  __shared__ uint32_t s_flag;
  fp_t c = fp_zero();
  bool nz = false;
  if (q < (uint32_t)PR::n_out) {
    c = slp_output(lds, PR::out()[q], h);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 7; k++) x |= c.l[k];
    x |= pswap(x);
    nz = x != 0u;
  }
  if (MODE == 0) {
    // FE(F) == 1: output 0 is 1, the others 0
    bool bad = false;
    if (q < (uint32_t)PR::n_out) {
      uint32_t x = 0;
#pragma unroll
      for (int k = 0; k < 7; k++) x |= (q == 0 && h == 0 && k == 0) ? (c.l[k] ^ 1u) : c.l[k];
      x |= pswap(x);
      bad = x != 0u;
    }
    if (tid == 0) s_flag = 0;
    __syncthreads();
    if (bad) s_flag = 1;  // benign race: every writer stores 1
    __syncthreads();
    if (tid == 0) verdict[item] = s_flag ? 0 : 1;
  } else {
    // S = O (outputs 12, 13 zero): the group's term is 1
    if (tid == 0) s_flag = 0;
    __syncthreads();
    if ((q == 12 || q == 13) && nz) s_flag = 1;
    __syncthreads();
    const bool inf = s_flag == 0;
    if (q < 12) {
      fp_t v = c;
      if (inf) {
        v = fp_zero();
        if (q == 0 && h == 0) v.l[0] = 1u;
      }
      fp_to_be48(out + (size_t)576 * item + 48 * q, v);
    }
  }
}

// Miller items of one set each (SURVEY 8a M5 for small packages and per-job fallback items):
// the pair (P_i, H(m_i)) of set item_first[item] -> that item's Miller value in lane form in
// f (the layout k_miller_fused writes).  A set with an error or an infinite point takes part
// as (0, 0) with use flag 0: its lines are the identity and it contributes 1.
template <int W>
__global__ void __launch_bounds__(64 * W) k_slp_items1(int n_items, const int32_t* __restrict__ item_first,
                                                   const uint32_t* __restrict__ P, const uint8_t* __restrict__ pinf,
                                                   const uint8_t* __restrict__ hinf, const int32_t* __restrict__ err,
                                                   const uint32_t* __restrict__ H, uint32_t* __restrict__ f) {
  using PR = Prog<SLP_ITEM1, W>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int item = blockIdx.x;
  if (item >= n_items) return;
  const uint32_t tid = threadIdx.x, h = tid & 1u, q = tid >> 1;
  slp_consts<PR>(lds, q, h, 32 * W);
  static_assert(PR::n_in == 7, "P.x, P.y, H.x.c0, H.x.c1, H.y.c0, H.y.c1, use");
  if (q < 7) {
    const size_t s = (size_t)item_first[item];
    const bool use = err[s] == 0 && !pinf[s] && !hinf[s];
    fp_t v = fp_zero();
    const uint32_t* src = nullptr;
    if (q < 2) {
      if (use) src = P + (s * lsgl_w_g1a + 7 * q) * 2 + h;
    } else if (q < 6) {
      src = H + (s * lsgl_w_g2a + 7 * (q - 2)) * 2 + h;
    } else if (use) {
      v = fp_t(FP_ONE);
    }
    if (src)
#pragma unroll
      for (int w = 0; w < 7; w++) v.l[w] = src[2 * w];
    slot_store(lds, PR::in()[q], h, v);
  }
  __syncthreads();
  slp_steps<PR>(lds, nullptr, q, h);
  if (q < 12) {  // Montgomery outputs (< 2p) straight into the lane form
    const fp_t v = slot_load(lds, PR::out()[q], h);
    uint32_t* dst = f + ((size_t)item * lsgl_w_f12 + 7 * q) * 2 + h;
#pragma unroll
    for (int w = 0; w < 7; w++) dst[2 * w] = v.l[w];
  }
}

// hash_to_G2's last stages for small packages: Q = Q0 + Q1 (projective lane
// form, k_h2c_map) -> H = clear_cofactor(Q) in affine lane form, hinf = (H = O); the same
// outputs as k_h2c_clear + the batched inversion + k_h2c_affine
template <int W>
__global__ void __launch_bounds__(64 * W) k_slp_h2c(int n, const uint32_t* __restrict__ Hp, uint32_t* __restrict__ H,
                                                    uint8_t* __restrict__ hinf) {
  using PR = Prog<SLP_H2C_CLEAR, W>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_nz;
  const int item = blockIdx.x;
  if (item >= n) return;
  const uint32_t tid = threadIdx.x, h = tid & 1u, q = tid >> 1;
  slp_consts<PR>(lds, q, h, 32 * W);
  static_assert(PR::n_in == 6 && PR::n_out == 6, "projective in, affine + Z out");
  if (q < 6) {
    const uint32_t* src = Hp + ((size_t)item * lsgl_w_g2p + 7 * q) * 2 + h;
    fp_t v;
#pragma unroll
    for (int w = 0; w < 7; w++) v.l[w] = src[2 * w];
    slot_store(lds, PR::in()[q], h, v);
  }
  if (tid == 0) s_nz = 0;
  __syncthreads();
  slp_steps<PR>(lds, nullptr, q, h);
  fp_t v = fp_zero();
  if (q < 6) v = slot_load(lds, PR::out()[q], h);
  if (q == 4 || q == 5) {  // Z = 0: H is the point at infinity
    const fp_t c = pair_canon_small(v);
    uint32_t x = 0;
#pragma unroll
    for (int w = 0; w < 7; w++) x |= c.l[w];
    x |= pswap(x);
    if (x) s_nz = 1;  // benign race: every writer stores 1
  }
  __syncthreads();
  const bool inf = s_nz == 0;
  if (q < 4) {
    if (inf) v = fp_zero();
    uint32_t* dst = H + ((size_t)item * lsgl_w_g2a + 7 * q) * 2 + h;
#pragma unroll
    for (int w = 0; w < 7; w++) dst[2 * w] = v.l[w];
  }
  if (tid == 0) hinf[item] = inf ? 1 : 0;
}

// lane-form component c (7 words per lane) of item i in an array of W-word-per-lane items
__device__ __forceinline__ fp_t lane_comp(const uint32_t* mem, size_t i, size_t wlane, uint32_t c, uint32_t h) {
  const uint32_t* src = mem + (i * wlane + 7 * c) * 2 + h;
  fp_t v;
#pragma unroll
  for (int w = 0; w < 7; w++) v.l[w] = src[2 * w];
  return v;
}
__device__ __forceinline__ void lane_comp_store(uint32_t* mem, size_t i, size_t wlane, uint32_t c, uint32_t h,
                                                const fp_t& v) {
  uint32_t* dst = mem + (i * wlane + 7 * c) * 2 + h;
#pragma unroll
  for (int w = 0; w < 7; w++) dst[2 * w] = v.l[w];
}

// G2 membership of decoded signatures for small packages (k_sig_subgroup's contract, SURVEY
// 8a M2: Signature.fromBytes(validate)): psi(P) == [x]P with complete formulas
template <int W>
__global__ void __launch_bounds__(64 * W) k_slp_g2_subgroup(int n, const uint32_t* __restrict__ sig_aff,
                                                            const uint8_t* __restrict__ inf, int32_t* __restrict__ err) {
  using PR = Prog<SLP_G2_SUBGROUP, W>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_nz;
  const int item = blockIdx.x;
  if (item >= n || err[item] != 0 || inf[item]) return;  // (uniform over the workgroup)
  const uint32_t tid = threadIdx.x, h = tid & 1u, q = tid >> 1;
  slp_consts<PR>(lds, q, h, 32 * W);
  if (q < 4) slot_store(lds, PR::in()[q], h, lane_comp(sig_aff, (size_t)item, lsgl_w_g2a, q, h));
  if (tid == 0) s_nz = 0;
  __syncthreads();
  slp_steps<PR>(lds, nullptr, q, h);
  if (q < 4) {
    const fp_t c = pair_canon_small(slot_load(lds, PR::out()[q], h));
    uint32_t x = 0;
#pragma unroll
    for (int w = 0; w < 7; w++) x |= c.l[w];
    x |= pswap(x);
    if (x) s_nz = 1;  // benign race: every writer stores 1
  }
  __syncthreads();
  if (tid == 0 && s_nz) err[item] = LSG_BLST_POINT_NOT_IN_GROUP;
}

// [r_i] sig_i for the RLC of small packages (k_sig_scale's contract): mode (optional) selects
// the sets; unusable sets get O, r_i = 0 (a set verified alone) its point unscaled
template <int W>
__global__ void __launch_bounds__(64 * W) k_slp_g2_scale(int n, const uint32_t* __restrict__ sig_aff,
                                                         const uint8_t* __restrict__ inf, const int32_t* __restrict__ err,
                                                         const uint8_t* __restrict__ pinf, const uint64_t* __restrict__ rnd,
                                                         const uint8_t* __restrict__ mode, uint32_t* __restrict__ out) {
  using PR = Prog<SLP_G2_SCALE, W>;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int item = blockIdx.x;
  if (item >= n || (mode && !mode[item])) return;
  const uint32_t tid = threadIdx.x, h = tid & 1u, q = tid >> 1;
  const bool usable = err[item] == 0 && !inf[item] && !(pinf && pinf[item]);
  const uint64_t r = rnd[item];
  if (!usable || r == 0) {  // O = (0 : 1 : 0), or (x : y : 1)
    if (q < 6) {
      fp_t v = fp_zero();
      if (q == 2 && !usable) v = fp_t(FP_ONE);
      if (q == 4 && usable) v = fp_t(FP_ONE);
      if (usable && q < 4) v = lane_comp(sig_aff, (size_t)item, lsgl_w_g2a, q, h);
      lane_comp_store(out, (size_t)item, lsgl_w_g2p, q, h, v);
    }
    return;
  }
  slp_consts<PR>(lds, q, h, 32 * W);
  static_assert(PR::n_in == 68 && PR::n_out == 6, "point + 64 bits in, projective out");
  for (uint32_t j = q; j < 68; j += 32 * W) {
    fp_t v = fp_zero();
    if (j < 4)
      v = lane_comp(sig_aff, (size_t)item, lsgl_w_g2a, j, h);
    else if ((r >> (j - 4)) & 1u)
      v = fp_t(FP_ONE);
    slot_store(lds, PR::in()[j], h, v);
  }
  __syncthreads();
  slp_steps<PR>(lds, nullptr, q, h);
  if (q < 6) lane_comp_store(out, (size_t)item, lsgl_w_g2p, q, h, slot_load(lds, PR::out()[q], h));
}

template <int PROG, int W, int MODE>
hipError_t launch(hipStream_t st, int n, const uint8_t* in, uint32_t in_stride, uint8_t* out, int32_t* verdict) {
  if (n <= 0) return hipSuccess;
  const size_t shm = (size_t)Prog<PROG, W>::n_slots * LSG_SLP_STRIDE * 4;
  hipLaunchKernelGGL((k_slp<PROG, W, MODE>), dim3(n), dim3(64 * W), shm, st, n, in, in_stride, out, verdict);
  return hipGetLastError();
}

}  // namespace

// Two waves per item (steps of 64 operations, each wave on its own SIMD) for up to 128 items
// (latency: a lone set, a few groups); one wave per item beyond, where the launch shares the
// chip with other packages and throughput counts: a one-wave step fills 32 lane pairs with ~32
// of the ~39 operations a two-wave step spreads over 64 (final exponentiation: 771 one-wave
// steps against 630 two-wave steps, 39 % fewer wave-steps).  128 against 512:
// profiles/r05_slp_w2max_ab.txt (gossip +4 %, block bodies +1.4 %, adversarial +1 %).
#ifndef LSG_SLP_W2_MAX
#define LSG_SLP_W2_MAX 128
#endif
static int slp_waves(int n) { return n <= LSG_SLP_W2_MAX ? 2 : 1; }
hipError_t lsg_slp_final_exp(hipStream_t st, int ng, const uint8_t* F576, int32_t* verdict) {
  return slp_waves(ng) == 2 ? launch<SLP_FE, 2, 0>(st, ng, F576, 576, nullptr, verdict)
                            : launch<SLP_FE, 1, 0>(st, ng, F576, 576, nullptr, verdict);
}
hipError_t lsg_slp_miller_neg_g1(hipStream_t st, int ng, const uint8_t* S288, uint8_t* out576) {
  return slp_waves(ng) == 2 ? launch<SLP_ML, 2, 1>(st, ng, S288, 288, out576, nullptr)
                            : launch<SLP_ML, 1, 1>(st, ng, S288, 288, out576, nullptr);
}
hipError_t lsg_slp_horner_miller(hipStream_t st, int ng, const uint8_t* C288, uint8_t* out576) {
  return slp_waves(ng) == 2 ? launch<SLP_HORNER, 2, 1>(st, ng, C288, 288 * 64, out576, nullptr)
                            : launch<SLP_HORNER, 1, 1>(st, ng, C288, 288 * 64, out576, nullptr);
}
template <int W>
static hipError_t items1(hipStream_t st, int n_items, const int32_t* item_first, const uint32_t* P, const uint8_t* pinf,
                         const uint8_t* hinf, const int32_t* err, const uint32_t* H, uint32_t* f) {
  const size_t shm = (size_t)Prog<SLP_ITEM1, W>::n_slots * LSG_SLP_STRIDE * 4;
  hipLaunchKernelGGL((k_slp_items1<W>), dim3(n_items), dim3(64 * W), shm, st, n_items, item_first, P, pinf, hinf, err, H, f);
  return hipGetLastError();
}
hipError_t lsg_slp_miller_items1(hipStream_t st, int n_items, const int32_t* item_first, const uint32_t* P,
                                 const uint8_t* pinf, const uint8_t* hinf, const int32_t* err, const uint32_t* H,
                                 uint32_t* f) {
  if (n_items <= 0) return hipSuccess;
  return slp_waves(n_items) == 2 ? items1<2>(st, n_items, item_first, P, pinf, hinf, err, H, f)
                                 : items1<1>(st, n_items, item_first, P, pinf, hinf, err, H, f);
}
hipError_t lsg_slp_h2c_clear(hipStream_t st, int n, const uint32_t* Hp, uint32_t* H, uint8_t* hinf) {
  if (n <= 0) return hipSuccess;
  const size_t shm = (size_t)Prog<SLP_H2C_CLEAR, 1>::n_slots * LSG_SLP_STRIDE * 4;
  hipLaunchKernelGGL((k_slp_h2c<1>), dim3(n), dim3(64), shm, st, n, Hp, H, hinf);
  return hipGetLastError();
}
template <int W>
static hipError_t g2_subgroup_w(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, int32_t* err) {
  const size_t shm = (size_t)Prog<SLP_G2_SUBGROUP, W>::n_slots * LSG_SLP_STRIDE * 4;
  hipLaunchKernelGGL((k_slp_g2_subgroup<W>), dim3(n), dim3(64 * W), shm, st, n, sig_aff, inf, err);
  return hipGetLastError();
}
template <int W>
static hipError_t g2_scale_w(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, const int32_t* err,
                             const uint8_t* pinf, const uint64_t* rnd, const uint8_t* mode, uint32_t* out) {
  const size_t shm = (size_t)Prog<SLP_G2_SCALE, W>::n_slots * LSG_SLP_STRIDE * 4;
  hipLaunchKernelGGL((k_slp_g2_scale<W>), dim3(n), dim3(64 * W), shm, st, n, sig_aff, inf, err, pinf, rnd, mode, out);
  return hipGetLastError();
}
hipError_t lsg_slp_g2_subgroup(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, int32_t* err) {
  if (n <= 0) return hipSuccess;
  return slp_waves(n) == 2 ? g2_subgroup_w<2>(st, n, sig_aff, inf, err) : g2_subgroup_w<1>(st, n, sig_aff, inf, err);
}
hipError_t lsg_slp_g2_scale(hipStream_t st, int n, const uint32_t* sig_aff, const uint8_t* inf, const int32_t* err,
                            const uint8_t* pinf, const uint64_t* rnd, const uint8_t* mode, uint32_t* out) {
  if (n <= 0) return hipSuccess;
  return slp_waves(n) == 2 ? g2_scale_w<2>(st, n, sig_aff, inf, err, pinf, rnd, mode, out)
                           : g2_scale_w<1>(st, n, sig_aff, inf, err, pinf, rnd, mode, out);
}
