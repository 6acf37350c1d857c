// Pair backend: 381-bit Montgomery arithmetic with one Fp element per lane PAIR.
//
// Representation: 14 signed limbs of 29 bits (radix 2^29, Montgomery R = 2^406); lane h
// (0/1) of a pair holds limbs 7h..7h+6, so a wave64 carries 32 field elements.  Values are
// LAZY: an fp_t is any integer congruent to the element, |v| < 2^12 p, with every limb in
// [-8, 2^29 + 8) except the signed top limb (limb 13).  Nothing is reduced mod p except
// where a canonical value is needed (equality, zero tests, serialisation), so
//   fp_add / fp_sub / fp_neg  = one limb-wise add + one parallel carry round (no carry
//                               chains, no comparisons, no cross-lane lookahead)
//   fp_mul                    = CIOS over radix 2^29: the 64-bit accumulators never carry
//                               (|t| < 28 * 2^58 < 2^63), so every partial product is one
//                               v_mad_i64_i32; per step one DPP broadcast of b_i, one of m,
//                               and one 32-bit DPP move of the retiring limb.  For inputs
//                               |a|, |b| < 2^12.6 p the output satisfies |w| < 2p.
// Measured (tools/micro/probe_fpmul.hip, profiles/r01_fpmul_probe.txt): 4.26e10 Fp-mul/s on
// MI355X at 4 waves/SIMD against 2.86e10 for the quad backend (lsg_fp_quad.hpp): about 760
// lane-instructions per product instead of 1360, and an addition costs ~30 per lane.
//
// LSG_PAIR_G = 1 builds the same arithmetic for one "lane" holding all 14 limbs (no DPP):
// the host build (tests/native/hostcheck.hip) runs it on the CPU so the lazy bounds, the
// radix-2^29 constants and the byte conversions are checked against the oracle without a GPU.
#pragma once
#include "lsg_constants_r29.hpp"

#ifndef LSG_PAIR_G
#define LSG_PAIR_G 2
#endif
#define LSG_GROUP LSG_PAIR_G
#define LSG_PAIR_MODE 1
#define LSG_LEAN_TOWER 1  // register-lean (narrow-issue) tower formulas, see lsg_tower.hpp
constexpr int LSG_PL = 14 / LSG_GROUP;  // limbs per lane
constexpr uint32_t LSG_M29 = (1u << 29) - 1;

#if LSG_PAIR_G == 2
// the generic layers built on this backend are device-only code
#undef LSG_INL
#define LSG_INL __device__ __forceinline__
#undef LSG_NOINL
#define LSG_NOINL __device__ __noinline__
#define LSG_PFN __device__ __forceinline__
#define LSG_PLEAF __device__ __noinline__
LSG_PFN uint32_t pair_h() { return __lane_id() & 1u; }
template <int CTRL>
LSG_PFN uint32_t pdpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
}
// value of pair-lane S (quad_perm [0,0,2,2] / [1,1,3,3])
template <int S>
LSG_PFN uint32_t pbcast(uint32_t x) {
  return S == 0 ? pdpp<0xA0>(x) : pdpp<0xF5>(x);
}
LSG_PFN uint32_t pswap(uint32_t x) { return pdpp<0xB1>(x); }  // the other lane of the pair
LSG_PFN uint32_t pdown(uint32_t x) {                           // lane 0 <- lane 1, lane 1 <- 0
  const uint32_t v = pdpp<0xF5>(x);
  return pair_h() ? 0u : v;
}
#ifndef LSG_LEAF_DPP_AND  // A/B builds: 0 = the round-2 moves (DPP move, then and / select)
#define LSG_LEAF_DPP_AND 1
#endif
#if LSG_LEAF_DPP_AND
LSG_PFN uint32_t pup(uint32_t x) {  // lane 1 <- lane 0, lane 0 <- 0: one v_and_b32 with a DPP source
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xA0, 0xf, 0xf, true) & (0u - pair_h());
}
#else
LSG_PFN uint32_t pup(uint32_t x) {
  const uint32_t v = pdpp<0xA0>(x);
  return pair_h() ? v : 0u;
}
#endif
// pdown(x & M29) and pbcast<0>(x) & M29 as ONE v_and_b32 each: the DPP move folds into the and
// (GCNDPPCombine) when the mask is a register operand -- lmask = M29 on lane 0 and 0 on lane 1
// also does pdown's zeroing of lane 1, so the retire step loses an and and a cndmask and the m
// broadcast an and
#if LSG_LEAF_DPP_AND
LSG_PFN uint32_t pdown_and(uint32_t x, uint32_t lmask) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xF5, 0xf, 0xf, true) & lmask;
}
LSG_PFN uint32_t pbcast0_and(uint32_t x, uint32_t m29) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xA0, 0xf, 0xf, true) & m29;
}
#else
LSG_PFN uint32_t pdown_and(uint32_t x, uint32_t) { return pdown(x & LSG_M29); }
LSG_PFN uint32_t pbcast0_and(uint32_t x, uint32_t) { return pbcast<0>(x & LSG_M29); }
#endif
#else
#define LSG_PFN LSG_INL
#define LSG_PLEAF LSG_NOINL
LSG_PFN uint32_t pair_h() { return 0u; }
template <int S>
LSG_PFN uint32_t pbcast(uint32_t x) {
  return x;
}
LSG_PFN uint32_t pswap(uint32_t x) { return x; }
LSG_PFN uint32_t pdown(uint32_t) { return 0u; }
LSG_PFN uint32_t pup(uint32_t) { return 0u; }
LSG_PFN uint32_t pdown_and(uint32_t, uint32_t) { return 0u; }
LSG_PFN uint32_t pbcast0_and(uint32_t x, uint32_t m29) { return x & m29; }
#endif
LSG_PFN bool pair_top() { return pair_h() == (uint32_t)(LSG_GROUP - 1); }
// this lane's k-th limb of a 14-limb literal
LSG_PFN uint32_t pair_pick(const uint32_t* c, int k) {
  return (LSG_GROUP == 2 && pair_h()) ? c[LSG_PL + k] : c[k];
}

struct fp_t {
  uint32_t l[LSG_PL];  // two's-complement limbs
  fp_t() = default;
  LSG_PFN fp_t(const fpc_t& c) {
#pragma unroll
    for (int k = 0; k < LSG_PL; k++) l[k] = pair_pick(c.l, k);
  }
};
LSG_PFN fp_t fp_from_arr(const uint32_t* c) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) r.l[k] = pair_pick(c, k);
  return r;
}

// ---- carries
// One parallel carry round: limb k keeps its low 29 bits plus the (signed) carry of limb
// k-1; the top limb keeps everything above.  Value-preserving; inputs with |limb| < 2^31
// come out with limbs in [-4, 2^29 + 4).
LSG_PFN fp_t pair_carry(const fp_t& a) {
  const bool top = pair_top();
  int32_t c[LSG_PL];
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) c[k] = (int32_t)a.l[k] >> 29;
  const uint32_t cin = pup((uint32_t)c[LSG_PL - 1]);
  fp_t o;
  o.l[0] = (a.l[0] & LSG_M29) + cin;
#pragma unroll
  for (int k = 1; k < LSG_PL - 1; k++) o.l[k] = (a.l[k] & LSG_M29) + (uint32_t)c[k - 1];
  o.l[LSG_PL - 1] = (top ? a.l[LSG_PL - 1] : (a.l[LSG_PL - 1] & LSG_M29)) + (uint32_t)c[LSG_PL - 2];
  return o;
}
// Full normalisation: limbs 0..12 in [0, 2^29), the signed top limb holds the rest.
LSG_PFN fp_t pair_full_norm(const fp_t& a) {
  int32_t v[LSG_PL];
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) v[k] = (int32_t)a.l[k];
#pragma unroll
  for (int k = 0; k < LSG_PL - 1; k++) {
    v[k + 1] += v[k] >> 29;
    v[k] &= (int32_t)LSG_M29;
  }
#if LSG_PAIR_G == 2
  const uint32_t cin = pup((uint32_t)(v[LSG_PL - 1] >> 29));
  if (!pair_top()) v[LSG_PL - 1] &= (int32_t)LSG_M29;
  v[0] += (int32_t)cin;
#pragma unroll
  for (int k = 0; k < LSG_PL - 1; k++) {
    v[k + 1] += v[k] >> 29;
    v[k] &= (int32_t)LSG_M29;
  }
#endif
  fp_t o;
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) o.l[k] = (uint32_t)v[k];
  return o;
}
// sign of a fully normalised value (pair-uniform)
LSG_PFN bool pair_is_neg(const fp_t& n) {
  const uint32_t s = (int32_t)n.l[LSG_PL - 1] < 0 ? 1u : 0u;
  return pbcast<LSG_GROUP - 1>(s) != 0u;
}

#ifdef LSG_COUNT_MULS  // host build only: exact Fp-multiplication counts per stage
extern unsigned long long lsg_mul_count;
#define LSG_COUNT_MUL() (lsg_mul_count++)
#else
#define LSG_COUNT_MUL() ((void)0)
#endif

// The end of a CIOS reduction: the 14 accumulators (64-bit, value-preserving) -> limbs in
// [0, 2^29) and the signed top limb, the pair's cross-lane carry included.
LSG_PFN void pair_redc_tail(int64_t* t, fp_t& r, bool top) {
#pragma unroll
  for (int j = 0; j < LSG_PL - 1; j++) {
    t[j + 1] += t[j] >> 29;
    t[j] &= (int64_t)LSG_M29;
  }
#if LSG_PAIR_G == 2
  const int64_t ct = t[LSG_PL - 1] >> 29;
  const uint32_t clo = pup((uint32_t)ct), chi = pup((uint32_t)((uint64_t)ct >> 32));
  if (!top) t[LSG_PL - 1] &= (int64_t)LSG_M29;
  t[0] += (int64_t)(((uint64_t)chi << 32) | clo);
  // second pass: only limb 0 (lane 1's, plus lane 0's carry of < 2^35) can exceed 32 bits;
  // limbs 1.. are < 2^29 (the top limb small and signed) and the carries from limb 1 on are
  // a few units, so the rest runs on 32-bit words (same value, same unique limbs)
  int32_t c = (int32_t)(t[0] >> 29);
  r.l[0] = (uint32_t)t[0] & LSG_M29;
#pragma unroll
  for (int j = 1; j < LSG_PL; j++) {
    const int32_t v = (int32_t)(uint32_t)t[j] + c;
    if (j < LSG_PL - 1) {
      c = v >> 29;
      r.l[j] = (uint32_t)v & LSG_M29;
    } else {
      r.l[j] = (uint32_t)v;
    }
  }
#else
  (void)top;
#pragma unroll
  for (int j = 0; j < LSG_PL; j++) r.l[j] = (uint32_t)t[j];
#endif
}

// ---- Montgomery product (CIOS over the 14 radix-2^29 limbs, i-loop over time)
// N independent products advance step by step together: in-order issue stalls a lone
// product on its serial chain (t0 mad -> m -> DPP broadcast -> m*p mads -> retire) at the
// one or two waves per SIMD the per-set kernels run at; N chains fill those stalls.
template <int N>
LSG_PFN void pair_mont_mul_n(fp_t* r, const fp_t* a, const fp_t* b) {
  const bool top = pair_top();
  uint32_t p[LSG_PL];
#pragma unroll
  for (int j = 0; j < LSG_PL; j++) p[j] = pair_pick(LSG_P, j);
  int64_t t[N][LSG_PL];
#pragma unroll
  for (int n = 0; n < N; n++)
#pragma unroll
    for (int j = 0; j < LSG_PL; j++) t[n][j] = 0;
  uint32_t m29 = LSG_M29, lmask = top ? 0u : LSG_M29;
#if LSG_PAIR_G == 2
  asm volatile("" : "+v"(m29), "+v"(lmask));  // register operands: the DPP moves fold into the ands
#endif
#pragma unroll
  for (int i = 0; i < 14; i++) {
#pragma unroll
    for (int n = 0; n < N; n++) {
      const uint32_t bs = b[n].l[i % LSG_PL];
      const int32_t bi = (int32_t)(i / LSG_PL == 0 ? pbcast<0>(bs) : pbcast<LSG_GROUP - 1>(bs));
#pragma unroll
      for (int j = 0; j < LSG_PL; j++) t[n][j] += (int64_t)(int32_t)a[n].l[j] * bi;
    }
#pragma unroll
    for (int n = 0; n < N; n++) {
      const uint32_t m = pbcast0_and((uint32_t)t[n][0] * LSG_N0P, m29);
#pragma unroll
      for (int j = 0; j < LSG_PL; j++) t[n][j] += (int64_t)(int32_t)m * (int32_t)p[j];
    }
#pragma unroll
    for (int n = 0; n < N; n++) {
      // retire limb 0 (its low 29 bits are zero on lane 0): the high part carries into the
      // next accumulator of the same lane, lane 1's low 29 bits move down to lane 0's top
      const int64_t c = t[n][0] >> 29;
      const uint32_t mv = pdown_and((uint32_t)t[n][0], lmask);
#pragma unroll
      for (int j = 0; j < LSG_PL - 1; j++) t[n][j] = t[n][j + 1];
      t[n][0] += c;
      t[n][LSG_PL - 1] = (int64_t)mv;
    }
  }
#pragma unroll
  for (int n = 0; n < N; n++) pair_redc_tail(t[n], r[n], top);
}
#ifndef LSG_SOP_STEP_FENCE
#define LSG_SOP_STEP_FENCE 0
#endif
// ---- sums of two products with one Montgomery reduction (fp_sop)
//   r_n = REDC(xa_n ya_n + xb_n yb_n)
// ONE CIOS pass with two partial products per step.  The Fp2 product is two of them,
//   c0 = REDC(a0 b0 + (-a1) b1),  c1 = REDC(a0 b1 + a1 b0)        (u^2 = -1),
// the same 588 mads per lane as Karatsuba's three full products, without its third
// reduction's overhead, its two additions and three subtractions (~330 other instructions per
// lane instead of ~560).  Bounds: in the pair layout an accumulator lives at most 7 steps on
// each lane (lane 1 hands only its low 29 bits down, the carry stays behind), so it sums at
// most 7 x 3 terms of < 2^58.1: |t| < 2^62.6.  The one-lane host build (LSG_PAIR_G = 1) keeps
// a column for 14 steps and carries once at mid-loop instead.  For inputs |x|, |y| < 2^12.6 p
// the outputs satisfy |r| < 3p.
template <int N, bool NEG0 = false>  // NEG0: output 0 takes xa ya - xb yb
LSG_PFN void pair_sop2_n(fp_t* r, const fp_t* xa, const fp_t* ya, const fp_t* xb, const fp_t* yb) {
  const bool top = pair_top();
  uint32_t p[LSG_PL];
#pragma unroll
  for (int j = 0; j < LSG_PL; j++) p[j] = pair_pick(LSG_P, j);
  int64_t t[N][LSG_PL];
#pragma unroll
  for (int n = 0; n < N; n++)
#pragma unroll
    for (int j = 0; j < LSG_PL; j++) t[n][j] = 0;
  uint32_t m29 = LSG_M29, lmask = top ? 0u : LSG_M29;
#if LSG_PAIR_G == 2
  asm volatile("" : "+v"(m29), "+v"(lmask));  // register operands: the DPP moves fold into the ands
#endif
#pragma unroll
  for (int i = 0; i < 14; i++) {
#pragma unroll
    for (int n = 0; n < N; n++) {
      const uint32_t sa = ya[n].l[i % LSG_PL], sb = yb[n].l[i % LSG_PL];
      const int32_t ba = (int32_t)(i / LSG_PL == 0 ? pbcast<0>(sa) : pbcast<LSG_GROUP - 1>(sa));
      int32_t bb = (int32_t)(i / LSG_PL == 0 ? pbcast<0>(sb) : pbcast<LSG_GROUP - 1>(sb));
      if (NEG0 && n == 0) bb = -bb;
#pragma unroll
      for (int j = 0; j < LSG_PL; j++) {
        t[n][j] += (int64_t)(int32_t)xa[n].l[j] * ba;
        t[n][j] += (int64_t)(int32_t)xb[n].l[j] * bb;
      }
    }
#pragma unroll
    for (int n = 0; n < N; n++) {
      const uint32_t m = pbcast0_and((uint32_t)t[n][0] * LSG_N0P, m29);
#pragma unroll
      for (int j = 0; j < LSG_PL; j++) t[n][j] += (int64_t)(int32_t)m * (int32_t)p[j];
    }
#pragma unroll
    for (int n = 0; n < N; n++) {
      const int64_t c = t[n][0] >> 29;
      const uint32_t mv = pdown_and((uint32_t)t[n][0], lmask);
#pragma unroll
      for (int j = 0; j < LSG_PL - 1; j++) t[n][j] = t[n][j + 1];
      t[n][0] += c;
      t[n][LSG_PL - 1] = (int64_t)mv;
    }
#if LSG_PAIR_G == 2 && LSG_SOP_STEP_FENCE
    __builtin_amdgcn_sched_barrier(0);  // no step's broadcasts hoisted into an earlier one
#endif
#if LSG_PAIR_G == 1
    if (i == 6) {  // one lane holds every column for 14 steps: carry once (value-preserving)
#pragma unroll
      for (int n = 0; n < N; n++)
#pragma unroll
        for (int j = 0; j < LSG_PL - 1; j++) {
          t[n][j + 1] += t[n][j] >> 29;
          t[n][j] &= (int64_t)LSG_M29;
        }
    }
#endif
  }
#pragma unroll
  for (int n = 0; n < N; n++) pair_redc_tail(t[n], r[n], top);
}
LSG_PFN fp_t pair_neg_limbs(const fp_t& a) {  // -a limb by limb (no carry: SOP operands are signed)
  fp_t r;
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) r.l[k] = 0u - a.l[k];
  return r;
}
#ifndef LSG_SOP_INTERLEAVE  // A/B: 1 = the two outputs of an Fp2 product in one pass
#define LSG_SOP_INTERLEAVE 0
#endif
LSG_PFN void pair_fp2_mul_sop(fp_t& c0, fp_t& c1, const fp_t& a0, const fp_t& a1, const fp_t& b0, const fp_t& b1) {
#if LSG_SOP_INTERLEAVE
  const fp_t xa[2] = {a0, a0}, ya[2] = {b0, b1}, xb[2] = {a1, a1}, yb[2] = {b1, b0};
  fp_t r[2];
  pair_sop2_n<2, true>(r, xa, ya, xb, yb);
  c0 = r[0];
  c1 = r[1];
#else
  pair_sop2_n<1, true>(&c0, &a0, &b0, &a1, &b1);
#if LSG_PAIR_G == 2
  __builtin_amdgcn_sched_barrier(0);  // one pass after the other: half the live accumulators
#endif
  pair_sop2_n<1>(&c1, &a0, &b1, &a1, &b0);
#endif
}

LSG_PLEAF fp_t pair_mont_mul(fp_t a, fp_t b) {
  LSG_COUNT_MUL();
  fp_t r;
  pair_mont_mul_n<1>(&r, &a, &b);
  return r;
}
// Multi-product leaves.  Operands cross the call as 8-word vectors: the gfx950 call ABI
// passes vector arguments in VGPRs (up to 32), but only the first two 7-word structs; the
// rest went byval through scratch at every call site.
// LSG_LEAF_MODE (A/B builds): 0 = one product per call everywhere, 1 = the multi-product
// leaves below with their products one after another (default), 2 = interleaved
#ifndef LSG_LEAF_MODE
#define LSG_LEAF_MODE 1
#endif
#ifndef LSG_FP2_SOP  // A/B builds: 0 = the Karatsuba Fp2 leaf (three full products)
#define LSG_FP2_SOP 1
#endif
#if LSG_PAIR_G == 2 && LSG_LEAF_MODE == 1
#define LSG_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define LSG_SCHED_FENCE() ((void)0)
#endif
#if LSG_PAIR_G == 2
// (the call ABI keeps v31 for the work-item ids, so a fourth 8-word operand would put one
// word on the stack: the last operand of a four-operand leaf travels as 4 + 3 words)
typedef uint32_t fp_arg4_t __attribute__((ext_vector_type(4)));
typedef uint32_t fp_arg3_t __attribute__((ext_vector_type(3)));
struct fp_tail {
  fp_arg4_t lo;
  fp_arg3_t hi;
};
LSG_PFN fp_arg4_t fp_pack_lo(const fp_t& a) { return fp_arg4_t{a.l[0], a.l[1], a.l[2], a.l[3]}; }
LSG_PFN fp_arg3_t fp_pack_hi(const fp_t& a) { return fp_arg3_t{a.l[4], a.l[5], a.l[6]}; }
LSG_PFN fp_t fp_unpack2(const fp_arg4_t& lo, const fp_arg3_t& hi) {
  fp_t r;
  r.l[0] = lo[0];
  r.l[1] = lo[1];
  r.l[2] = lo[2];
  r.l[3] = lo[3];
  r.l[4] = hi[0];
  r.l[5] = hi[1];
  r.l[6] = hi[2];
  return r;
}
#define LSG_TAIL_PARAMS(x) fp_arg4_t x##_lo, fp_arg3_t x##_hi
#define LSG_TAIL_ARGS(v) fp_pack_lo(v), fp_pack_hi(v)
#define LSG_TAIL_UNPACK(x) fp_unpack2(x##_lo, x##_hi)
typedef uint32_t fp_arg_t __attribute__((ext_vector_type(8)));
LSG_PFN fp_arg_t fp_pack(const fp_t& a) {
  fp_arg_t v;  // word 7 is never read
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) v[k] = a.l[k];
  return v;
}
LSG_PFN fp_t fp_unpack(const fp_arg_t& v) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) r.l[k] = v[k];
  return r;
}
#else
#define LSG_TAIL_PARAMS(x) fp_t x
#define LSG_TAIL_ARGS(v) (v)
#define LSG_TAIL_UNPACK(x) (x)
typedef fp_t fp_arg_t;
LSG_PFN fp_arg_t fp_pack(const fp_t& a) { return a; }
LSG_PFN fp_t fp_unpack(const fp_arg_t& v) { return v; }
#endif
struct fp_duo {
  fp_t x, y;
};
LSG_PLEAF fp_duo pair_mont_mul2_v(fp_arg_t a0, fp_arg_t b0, fp_arg_t a1, LSG_TAIL_PARAMS(b1)) {
  LSG_COUNT_MUL();
  LSG_COUNT_MUL();
  const fp_t x[2] = {fp_unpack(a0), fp_unpack(a1)}, y[2] = {fp_unpack(b0), LSG_TAIL_UNPACK(b1)};
  fp_t r[2];
#if LSG_LEAF_MODE == 2
  pair_mont_mul_n<2>(r, x, y);
#else
  pair_mont_mul_n<1>(&r[0], &x[0], &y[0]);
  LSG_SCHED_FENCE();
  pair_mont_mul_n<1>(&r[1], &x[1], &y[1]);
#endif
  return fp_duo{r[0], r[1]};
}
LSG_PFN fp_duo pair_mont_mul2(const fp_t& a0, const fp_t& b0, const fp_t& a1, const fp_t& b1) {
  return pair_mont_mul2_v(fp_pack(a0), fp_pack(b0), fp_pack(a1), LSG_TAIL_ARGS(b1));
}
// Karatsuba Fp2 product (a0 + a1 u)(b0 + b1 u), u^2 = -1: its three Fp products in one call
LSG_PLEAF fp_duo pair_fp2_mul_v(fp_arg_t a0, fp_arg_t a1, fp_arg_t b0, LSG_TAIL_PARAMS(b1));
// Fp2 square (a0 + a1)(a0 - a1), 2 a0 a1: its two Fp products in one call
LSG_PLEAF fp_duo pair_fp2_sqr_v(fp_arg_t a0, fp_arg_t a1);
LSG_PFN fp_duo pair_fp2_mul(const fp_t& a0, const fp_t& a1, const fp_t& b0, const fp_t& b1) {
  return pair_fp2_mul_v(fp_pack(a0), fp_pack(a1), fp_pack(b0), LSG_TAIL_ARGS(b1));
}
LSG_PFN fp_duo pair_fp2_sqr(const fp_t& a0, const fp_t& a1) { return pair_fp2_sqr_v(fp_pack(a0), fp_pack(a1)); }
#if LSG_LEAF_MODE != 0
#define LSG_FP2_LEAF 1  // lsg_tower.hpp's fp2_mul / fp2_sqr call the two leaves above
#endif

// ------------------------------------------------------------------ Fp API
LSG_PFN fp_t fp_zero() {
  fp_t r;
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) r.l[k] = 0u;
  return r;
}
LSG_PFN fp_t fp_select(bool c, const fp_t& a, const fp_t& b) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) r.l[k] = c ? a.l[k] : b.l[k];
  return r;
}
LSG_PFN fp_t fp_add(const fp_t& a, const fp_t& b) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) r.l[k] = a.l[k] + b.l[k];
  return pair_carry(r);
}
LSG_PFN fp_t fp_sub(const fp_t& a, const fp_t& b) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) r.l[k] = a.l[k] - b.l[k];
  return pair_carry(r);
}
LSG_PFN fp_t fp_neg(const fp_t& a) { return fp_sub(fp_zero(), a); }
LSG_PFN fp_t fp_mul(const fp_t& a, const fp_t& b) { return pair_mont_mul(a, b); }
#if LSG_LEAF_MODE == 0
LSG_PFN void fp_mul2(fp_t& r0, fp_t& r1, const fp_t& a0, const fp_t& b0, const fp_t& a1, const fp_t& b1) {
  fp_t t = pair_mont_mul(a0, b0);
  r1 = pair_mont_mul(a1, b1);
  r0 = t;
}
LSG_PFN void fp_mul3(fp_t& r0, fp_t& r1, fp_t& r2, const fp_t& a0, const fp_t& b0, const fp_t& a1, const fp_t& b1,
                     const fp_t& a2, const fp_t& b2) {
  fp_t t0 = pair_mont_mul(a0, b0);
  fp_t t1 = pair_mont_mul(a1, b1);
  r2 = pair_mont_mul(a2, b2);
  r0 = t0;
  r1 = t1;
}
#else
LSG_PFN void fp_mul2(fp_t& r0, fp_t& r1, const fp_t& a0, const fp_t& b0, const fp_t& a1, const fp_t& b1) {
  const fp_duo d = pair_mont_mul2(a0, b0, a1, b1);
  r0 = d.x;
  r1 = d.y;
}
LSG_PFN void fp_mul3(fp_t& r0, fp_t& r1, fp_t& r2, const fp_t& a0, const fp_t& b0, const fp_t& a1, const fp_t& b1,
                     const fp_t& a2, const fp_t& b2) {
  const fp_duo d = pair_mont_mul2(a0, b0, a1, b1);
  r2 = pair_mont_mul(a2, b2);
  r0 = d.x;
  r1 = d.y;
}
#endif
LSG_PFN void fp_mul9(fp_t* r, const fp_t* a, const fp_t* b) {
#pragma unroll
  for (int g = 0; g < 9; g += 3) fp_mul3(r[g], r[g + 1], r[g + 2], a[g], b[g], a[g + 1], b[g + 1], a[g + 2], b[g + 2]);
}

// the Fp2 leaves declared above (they need fp_add / fp_sub)
LSG_PLEAF fp_duo pair_fp2_mul_v(fp_arg_t va0, fp_arg_t va1, fp_arg_t vb0, LSG_TAIL_PARAMS(vb1)) {
  LSG_COUNT_MUL();
  LSG_COUNT_MUL();
  LSG_COUNT_MUL();
  const fp_t a0 = fp_unpack(va0), a1 = fp_unpack(va1), b0 = fp_unpack(vb0), b1 = LSG_TAIL_UNPACK(vb1);
#if LSG_FP2_SOP
  fp_duo d;
  pair_fp2_mul_sop(d.x, d.y, a0, a1, b0, b1);
  return d;
#endif
  // the three products run one after another (sched_barrier): interleaved, the leaf needed
  // ~180 VGPRs, and every caller had to spill around it what the call clobbers
  fp_t t[3];
#if LSG_LEAF_MODE == 2
  const fp_t a[3] = {a0, a1, fp_add(a0, a1)}, b[3] = {b0, b1, fp_add(b0, b1)};
  pair_mont_mul_n<3>(t, a, b);
#else
  pair_mont_mul_n<1>(&t[0], &a0, &b0);
  LSG_SCHED_FENCE();
  pair_mont_mul_n<1>(&t[1], &a1, &b1);
  LSG_SCHED_FENCE();
  const fp_t s0 = fp_add(a0, a1), s1 = fp_add(b0, b1);
  pair_mont_mul_n<1>(&t[2], &s0, &s1);
#endif
  return fp_duo{fp_sub(t[0], t[1]), fp_sub(fp_sub(t[2], t[0]), t[1])};
}
LSG_PLEAF fp_duo pair_fp2_sqr_v(fp_arg_t va0, fp_arg_t va1) {
  LSG_COUNT_MUL();
  LSG_COUNT_MUL();
  const fp_t a0 = fp_unpack(va0), a1 = fp_unpack(va1);
  fp_t t[2];
#if LSG_LEAF_MODE == 2
  const fp_t a[2] = {fp_add(a0, a1), a0}, b[2] = {fp_sub(a0, a1), a1};
  pair_mont_mul_n<2>(t, a, b);
#else
  const fp_t s = fp_add(a0, a1), d = fp_sub(a0, a1);
  pair_mont_mul_n<1>(&t[0], &s, &d);
  LSG_SCHED_FENCE();
  pair_mont_mul_n<1>(&t[1], &a0, &a1);
#endif
  return fp_duo{t[0], fp_add(t[1], t[1])};
}

// a^e for a fixed public exponent e (12 little-endian words) in one call: the same sliding
// window of width 4 as lsg_tower.hpp's generic fp_pow_fixed, with its ~455 products inline
// (one call, one load of p, no per-product argument moves) -- the square roots of signature
// decompression and SSWU and the batched inversions' roots are chains of these
LSG_PLEAF fp_t pair_pow_fixed(fp_t a, const uint32_t* __restrict__ e) {
  auto mul = [](const fp_t& x, const fp_t& y) {
    LSG_COUNT_MUL();
    fp_t r;
    pair_mont_mul_n<1>(&r, &x, &y);
    return r;
  };
  // T[k] = a^(2k+1), written out: a table loop the compiler declines to unroll would put T
  // in scratch with indexed access
  fp_t T[8];
  const fp_t a2 = mul(a, a);
  T[0] = a;
  T[1] = mul(T[0], a2);
  T[2] = mul(T[1], a2);
  T[3] = mul(T[2], a2);
  T[4] = mul(T[3], a2);
  T[5] = mul(T[4], a2);
  T[6] = mul(T[5], a2);
  T[7] = mul(T[6], a2);
  int i = 383;
  while (i >= 0 && !((e[i >> 5] >> (i & 31)) & 1u)) i--;
  fp_t r = T[0];
  bool started = false;
  while (i >= 0) {
    if (!((e[i >> 5] >> (i & 31)) & 1u)) {
      r = mul(r, r);
      i--;
      continue;
    }
    int j = i - 3 < 0 ? 0 : i - 3;
    while (!((e[j >> 5] >> (j & 31)) & 1u)) j++;
    uint32_t v = 0;
    for (int t = i; t >= j; t--) v = (v << 1) | ((e[t >> 5] >> (t & 31)) & 1u);
    if (started)
      for (int t = i; t >= j; t--) r = mul(r, r);
    fp_t tv = T[0];
#pragma unroll
    for (int k = 1; k < 8; k++) tv = fp_select(v == (uint32_t)(2 * k + 1), T[k], tv);
    r = started ? mul(r, tv) : tv;
    started = true;
    i = j - 1;
  }
  return r;
}
#if LSG_LEAF_MODE != 0 && !defined(LSG_NO_POW_LEAF)  // (A/B builds: -DLSG_NO_POW_LEAF)
#define LSG_POW_LEAF 1  // lsg_tower.hpp's fp_pow_fixed calls pair_pow_fixed
#endif

// The same sliding window, planned at compile time.  pair_pow_fixed walks the exponent bit by
// bit through a pointer argument: every bit test is a vector load and a wait (the pointer is
// not known to be uniform inside the leaf), ~7 dependent loads per window against ~5
// products.  Here the plan of each of the three fixed exponents is a constant table read with
// scalar loads at a wave-uniform index, and the control flow is scalar.
//   step[0] = k:             r = a^(2k+1)
//   step[w] = (s << 8) | k:  r = r^(2^s) * a^(2k+1)
//   then `tail` squarings
enum lsg_pow_id { LSG_POW_INV = 0, LSG_POW_SQRT = 1, LSG_POW_SQRT34 = 2 };  // p-2, (p+1)/4, (p-3)/4
#define LSG_POW_IDS 1
struct pow_plan_t {
  int n, tail;
  uint32_t step[128];
};
constexpr pow_plan_t make_pow_plan(const uint32_t (&e)[12]) {
  pow_plan_t P{};
  int i = 383;
  while (i >= 0 && !((e[i >> 5] >> (i & 31)) & 1u)) i--;
  int sq = 0;
  while (i >= 0) {
    if (!((e[i >> 5] >> (i & 31)) & 1u)) {
      sq++;
      i--;
      continue;
    }
    int j = i - 3 < 0 ? 0 : i - 3;  // window e[i..j] ends in a set bit
    while (!((e[j >> 5] >> (j & 31)) & 1u)) j++;
    uint32_t v = 0;
    for (int t = i; t >= j; t--) v = (v << 1) | ((e[t >> 5] >> (t & 31)) & 1u);
    if (P.n > 0) sq += i - j + 1;
    P.step[P.n++] = ((uint32_t)sq << 8) | (v >> 1);
    sq = 0;
    i = j - 1;
  }
  P.tail = sq;
  return P;
}
// the plan's exponent, rebuilt step by step, is e (checked at compile time below)
constexpr bool pow_plan_is(const pow_plan_t& P, const uint32_t (&e)[12]) {
  uint32_t x[13] = {};
  for (int w = 0; w <= P.n; w++) {
    const int s = w == P.n ? P.tail : (int)(P.step[w] >> 8);
    for (int b = 0; b < s; b++) {  // x <<= 1
      if (x[12] >> 31) return false;
      for (int k = 12; k > 0; k--) x[k] = (x[k] << 1) | (x[k - 1] >> 31);
      x[0] <<= 1;
    }
    if (w < P.n) {  // x += 2k + 1 (x is even here but for w = 0, where it is 0)
      uint64_t c = 2 * (P.step[w] & 0xffu) + 1;
      for (int k = 0; k < 13; k++) {
        c += x[k];
        x[k] = (uint32_t)c;
        c >>= 32;
      }
    }
  }
  for (int k = 0; k < 12; k++)
    if (x[k] != e[k]) return false;
  return x[12] == 0 && P.n > 0;
}
LSG_CONST pow_plan_t LSG_POW_PLANS[3] = {make_pow_plan(LSG_EXP_P_MINUS_2), make_pow_plan(LSG_EXP_P_PLUS_1_DIV_4),
                                        make_pow_plan(LSG_EXP_P_MINUS_3_DIV_4)};
static_assert(pow_plan_is(LSG_POW_PLANS[LSG_POW_INV], LSG_EXP_P_MINUS_2), "p-2 plan");
static_assert(pow_plan_is(LSG_POW_PLANS[LSG_POW_SQRT], LSG_EXP_P_PLUS_1_DIV_4), "(p+1)/4 plan");
static_assert(pow_plan_is(LSG_POW_PLANS[LSG_POW_SQRT34], LSG_EXP_P_MINUS_3_DIV_4), "(p-3)/4 plan");

LSG_PLEAF fp_t pair_pow_plan(fp_t a, int id) {
#if LSG_PAIR_G == 2
  id = __builtin_amdgcn_readfirstlane(id);  // a literal at every call site
#endif
  const pow_plan_t& P = LSG_POW_PLANS[id];
  auto mul = [](const fp_t& x, const fp_t& y) {
    LSG_COUNT_MUL();
    fp_t r;
    pair_mont_mul_n<1>(&r, &x, &y);
    return r;
  };
  auto pick = [](const fp_t* T, uint32_t k) {
    fp_t tv = T[0];
#pragma unroll
    for (uint32_t q = 1; q < 8; q++) tv = fp_select(k == q, T[q], tv);
    return tv;
  };
  fp_t T[8];  // T[k] = a^(2k+1), written out as in pair_pow_fixed
  const fp_t a2 = mul(a, a);
  T[0] = a;
  T[1] = mul(T[0], a2);
  T[2] = mul(T[1], a2);
  T[3] = mul(T[2], a2);
  T[4] = mul(T[3], a2);
  T[5] = mul(T[4], a2);
  T[6] = mul(T[5], a2);
  T[7] = mul(T[6], a2);
  // the operands made opaque at each product: known non-negative limbs (a product's masked
  // output) would turn the mads into v_mad_u64_u32 plus accumulator moves
  auto hide = [](fp_t x) {
#if LSG_PAIR_G == 2
#pragma unroll
    for (int k = 0; k < LSG_PL; k++) asm volatile("" : "+v"(x.l[k]));
#endif
    return x;
  };
  auto sqr = [&](const fp_t& x) {
    const fp_t y = hide(x);
    return mul(y, y);
  };
  fp_t r = pick(T, P.step[0] & 0xffu);
  const int n = P.n;
#pragma unroll 1
  for (int w = 1; w < n; w++) {
    const uint32_t s = P.step[w];
#pragma unroll 1
    for (uint32_t b = s >> 8; b; b--) r = sqr(r);
    r = mul(hide(r), hide(pick(T, s & 0xffu)));
  }
#pragma unroll 1
  for (int b = P.tail; b; b--) r = sqr(r);
  return r;
}
#if defined(LSG_POW_LEAF) && !defined(LSG_NO_POW_PLAN)  // (A/B builds: -DLSG_NO_POW_PLAN)
#define LSG_POW_PLAN 1  // lsg_tower.hpp's fp_pow_id calls pair_pow_plan
#endif

// ---- canonical values
// v in (-p, 2p) -> the representative in [0, p), fully normalised
LSG_PFN fp_t pair_canon_small(const fp_t& v0) {
  const fp_t p = fp_from_arr(LSG_P);
  fp_t v = pair_full_norm(v0);
  v = fp_select(pair_is_neg(v), pair_full_norm(fp_add(v, p)), v);
  fp_t d = pair_full_norm(fp_sub(v, p));
  return fp_select(pair_is_neg(d), v, d);
}
// any lazy value -> [0, p): one product by mont(1) lands it in (-p, 2p)
LSG_PFN fp_t pair_canon(const fp_t& a) { return pair_canon_small(pair_mont_mul(a, fp_t(FP_ONE))); }
// fp_from_mont's result (lsg_tower.hpp) is made canonical here, so serialisation and the
// canonical predicates below see plain integers in [0, p)
LSG_PFN fp_t fp_canonical(const fp_t& a) { return pair_canon_small(a); }

// |result| < 2p for any lazy value (for loop-carried values that are not products)
LSG_PFN fp_t fp_tame(const fp_t& a) { return pair_mont_mul(a, fp_t(FP_ONE)); }

LSG_PFN bool fp_is_zero(const fp_t& a) {
  const fp_t c = pair_canon(a);
  uint32_t nz = 0;
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) nz |= c.l[k];
  nz |= pswap(nz);
  return nz == 0u;
}
LSG_PFN bool fp_eq(const fp_t& a, const fp_t& b) { return fp_is_zero(fp_sub(a, b)); }

// predicates on canonical (non-Montgomery) values
LSG_PFN bool fp_canon_gt_half(const fp_t& c) {
  return pair_is_neg(pair_full_norm(fp_sub(fp_from_arr(LSG_HALF_P_CANON), pair_canon_small(c))));
}
// c = a raw decoded integer (not reduced): c < p
LSG_PFN bool fp_canon_lt_p(const fp_t& c) { return pair_is_neg(pair_full_norm(fp_sub(c, fp_from_arr(LSG_P)))); }
LSG_PFN uint32_t fp_canon_parity(const fp_t& c) { return pbcast<0>(pair_canon_small(c).l[0] & 1u); }

// ---- bytes
LSG_PFN uint32_t pair_be32(const uint8_t* q) {
  return ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
}
// the number formed by the 4*nwords big-endian bytes at b (nwords <= 12)
LSG_PFN fp_t fp_from_be_bytes(const uint8_t* b, int nwords) {
  uint32_t w[12];
#pragma unroll
  for (int k = 0; k < 12; k++) w[k] = k < nwords ? pair_be32(b + 4 * (nwords - 1 - k)) : 0u;
  uint32_t L[14];
#pragma unroll
  for (int k = 0; k < 14; k++) {
    const int bit = 29 * k, wi = bit / 32, off = bit % 32;
    uint32_t x = w[wi] >> off;
    if (off > 3 && wi + 1 < 12) x |= w[wi + 1] << (32 - off);
    L[k] = x & LSG_M29;
  }
  return fp_from_arr(L);
}
// all 14 limbs of a value in every lane of its pair
LSG_PFN void pair_gather(uint32_t* L, const fp_t& a) {
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) {
    const uint32_t o = pswap(a.l[k]);
    if (LSG_GROUP == 2) {
      L[k] = pair_h() ? o : a.l[k];
      L[LSG_PL + k] = pair_h() ? a.l[k] : o;
    } else {
      L[k] = a.l[k];
    }
  }
}
LSG_PFN void pair_put_be32(uint8_t* q, uint32_t v) {
  q[0] = (uint8_t)(v >> 24);
  q[1] = (uint8_t)(v >> 16);
  q[2] = (uint8_t)(v >> 8);
  q[3] = (uint8_t)v;
}
// 48 big-endian bytes of a canonical (or flag-carrying raw) value; lane h writes 24 of them
LSG_PFN void fp_to_be48(uint8_t* b, const fp_t& a) {
  uint32_t L[14];
  pair_gather(L, pair_full_norm(a));
  uint32_t w[12];
#pragma unroll
  for (int k = 0; k < 12; k++) {
    const int bit = 32 * k, li = bit / 29, off = bit % 29;
    uint64_t x = (uint64_t)L[li] >> off;
    int got = 29 - off;
    if (li + 1 < 14) x |= (uint64_t)L[li + 1] << got;
    got += 29;
    if (got < 32 && li + 2 < 14) x |= (uint64_t)L[li + 2] << got;
    w[k] = (uint32_t)x;
  }
  constexpr int PW = 12 / LSG_GROUP;
#pragma unroll
  for (int j = 0; j < PW; j++) {
    const int k = PW * (int)pair_h() + j;
    const uint32_t v = (LSG_GROUP == 2 && pair_h()) ? w[(PW + j) % 12] : w[j];
    pair_put_be32(b + 44 - 4 * k, v);
  }
}
// the 3 ZCash flag bits are bits 381..383 = bits 4..6 of limb 13 (top lane, last register)
LSG_PFN fp_t fp_mask_flags(const fp_t& a) {
  fp_t r = a;
  if (pair_top()) r.l[LSG_PL - 1] &= 0xfu;
  return r;
}
// flags: the ZCash flag byte (bits 5..7), placed at bits 381..383 of a canonical value
LSG_PFN fp_t fp_or_flags(const fp_t& a, uint32_t flags) {
  fp_t r = pair_full_norm(a);
  if (pair_top()) r.l[LSG_PL - 1] |= flags >> 1;
  return r;
}

// kernels call this once (the quad backend stages p in LDS; here p is a literal)
LSG_PFN void lsg_lane_setup() {}

// ---- item-major global storage: a value of type T (a struct of W words per lane) for item
// i lives at mem[(i*W + k)*G + h], k = 0..W-1 (one 8-byte segment per pair and word)
template <class T>
LSG_PFN T lane_load(const uint32_t* __restrict__ mem, size_t item) {
  constexpr int W = sizeof(T) / 4;
  uint32_t w[W];
  const uint32_t* p = mem + item * W * LSG_GROUP + pair_h();
#pragma unroll
  for (int k = 0; k < W; k++) w[k] = p[k * LSG_GROUP];
  T v;
  __builtin_memcpy(&v, w, sizeof(T));
  return v;
}
template <class T>
LSG_PFN void lane_store(uint32_t* __restrict__ mem, size_t item, const T& v) {
  constexpr int W = sizeof(T) / 4;
  uint32_t w[W];
  __builtin_memcpy(w, &v, sizeof(T));
  uint32_t* p = mem + item * W * LSG_GROUP + pair_h();
#pragma unroll
  for (int k = 0; k < W; k++) p[k * LSG_GROUP] = w[k];
}
template <class T>
constexpr size_t lane_words() {
  return sizeof(T) / 4 * LSG_GROUP;  // u32 words per item in global memory
}
