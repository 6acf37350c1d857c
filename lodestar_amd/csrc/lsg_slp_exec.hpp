// lsg_slp_exec.hpp -- one operation of a straight-line program (tools/gen_slp.py), shared
// by the gfx950 interpreter kernel (lsg_slp.hip, LSG_PAIR_G = 2: a lane pair per operation)
// and the host build of the pair backend (tests/native/hostcheck.hip, LSG_PAIR_G = 1: all 14
// limbs in one "lane"), so the exact device arithmetic -- gathers, carry round, lazy bounds,
// LDS layout -- is checked against the oracle without a GPU.  Include after lsg_fp_pair.hpp.
#pragma once
#include "lsg_inv.hpp"

// LDS slot s: LSG_SLP_STRIDE words; lane h of a pair holds its LSG_PL limbs at words
// s*STRIDE + h*8 ..  (a stride that is not a multiple of the bank count spreads the lane
// pairs of a step, which read unrelated slots, over the LDS banks)
#ifndef LSG_SLP_STRIDE
#define LSG_SLP_STRIDE 16
#endif
LSG_PFN fp_t slot_load(const uint32_t* lds, uint32_t s, uint32_t h) {
  fp_t r;
#if LSG_PAIR_G == 2
  // two aligned 16-byte reads (word 7 is padding)
  const uint4* p = reinterpret_cast<const uint4*>(lds) + s * (LSG_SLP_STRIDE / 4) + h * 2;
  const uint4 a = p[0], b = p[1];
  r.l[0] = a.x;
  r.l[1] = a.y;
  r.l[2] = a.z;
  r.l[3] = a.w;
  r.l[4] = b.x;
  r.l[5] = b.y;
  r.l[6] = b.z;
#else
  const uint32_t* p = lds + s * LSG_SLP_STRIDE + h * 8;
  for (int k = 0; k < LSG_PL; k++) r.l[k] = p[k];
#endif
  return r;
}
LSG_PFN void slot_store(uint32_t* lds, uint32_t s, uint32_t h, const fp_t& v) {
#if LSG_PAIR_G == 2
  uint4* p = reinterpret_cast<uint4*>(lds) + s * (LSG_SLP_STRIDE / 4) + h * 2;
  p[0] = make_uint4(v.l[0], v.l[1], v.l[2], v.l[3]);
  p[1] = make_uint4(v.l[4], v.l[5], v.l[6], 0u);
#else
  uint32_t* p = lds + s * LSG_SLP_STRIDE + h * 8;
  for (int k = 0; k < LSG_PL; k++) p[k] = v.l[k];
#endif
}

// acc += coef * slot over the first N terms of a 7-term half (t: slot | coef << 10, 16
// bits): straight-line code, every load issued before the first multiply-add
template <int N>
LSG_PFN void slp_gather_n(int64_t* acc, const uint32_t* lds, const uint32_t* t, uint32_t h) {
  fp_t v[N];
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = slot_load(lds, t[k] & 1023u, h);
#pragma unroll
  for (int k = 0; k < N; k++) {
    const int32_t c = (int32_t)(t[k] << 16) >> 26;  // bits 10..15, signed
#pragma unroll
    for (int j = 0; j < LSG_PL; j++) acc[j] += (int64_t)c * (int64_t)(int32_t)v[k].l[j];
  }
}
// n: the step's maximum term count (uniform, from the step descriptor); lanes with fewer
// terms hold zero terms (slot 0, coefficient 0), so nothing diverges
LSG_PFN void slp_gather(int64_t* acc, const uint32_t* lds, const uint32_t* t, uint32_t n, uint32_t h) {
  switch (n) {
    case 1: slp_gather_n<1>(acc, lds, t, h); break;
    case 2: slp_gather_n<2>(acc, lds, t, h); break;
    case 3: slp_gather_n<3>(acc, lds, t, h); break;
    case 4: slp_gather_n<4>(acc, lds, t, h); break;
    case 5: slp_gather_n<5>(acc, lds, t, h); break;
    case 6: slp_gather_n<6>(acc, lds, t, h); break;
    case 7: slp_gather_n<7>(acc, lds, t, h); break;
    default: break;
  }
}

// one parallel carry round over the 14 accumulators (|acc| < 2^45): limbs in
// [-2^16, 2^29 + 2^16), the signed top limb keeps everything above
LSG_PFN fp_t slp_carry(const int64_t* acc) {
  const bool top = pair_top();
  int32_t c[LSG_PL];
#pragma unroll
  for (int j = 0; j < LSG_PL; j++) c[j] = (int32_t)(acc[j] >> 29);
  const uint32_t cin = pup((uint32_t)c[LSG_PL - 1]);
  fp_t o;
  o.l[0] = ((uint32_t)acc[0] & LSG_M29) + cin;
#pragma unroll
  for (int j = 1; j < LSG_PL - 1; j++) o.l[j] = ((uint32_t)acc[j] & LSG_M29) + (uint32_t)c[j - 1];
  o.l[LSG_PL - 1] = (top ? (uint32_t)acc[LSG_PL - 1] : ((uint32_t)acc[LSG_PL - 1] & LSG_M29)) + (uint32_t)c[LSG_PL - 2];
  return o;
}

// operation entry e (8 words): w0 = dst | kind << 10 (0 LIN, 1 MUL, 2 LOADMUL, 3 INV) | nA << 12 | nB << 16 | input << 20,
// then 14 16-bit terms (A at 0..6, B at 7..13).  d: the step descriptor (uniform: the term
// counts to gather, whether any LIN / any product is in the step).  inp: the item's input
// blob (LOADMUL).
LSG_PFN void slp_exec(uint32_t* lds, const uint32_t* e, const uint8_t* inp, uint32_t h, uint32_t d) {
  const uint32_t w0 = e[0];
  const uint32_t kind = (w0 >> 10) & 3u, na = (d >> 8) & 7u, nb = (d >> 11) & 7u;
  uint32_t ta[7], tb[7];
#pragma unroll
  for (int k = 0; k < 7; k++) {
    const uint32_t lo = e[1 + k] & 0xffffu, hi = e[1 + k] >> 16;
    if (2 * k < 7) ta[2 * k] = lo; else tb[2 * k - 7] = lo;
    if (2 * k + 1 < 7) ta[2 * k + 1] = hi; else tb[2 * k + 1 - 7] = hi;
  }
  int64_t acc[LSG_PL], bcc[LSG_PL];
#pragma unroll
  for (int j = 0; j < LSG_PL; j++) acc[j] = bcc[j] = 0;
  slp_gather(acc, lds, ta, na, h);
  slp_gather(bcc, lds, tb, nb, h);
  fp_t r;
  if ((d >> 14) & 1u) {  // the step has LIN ops (a product lane overwrites r below)
    int64_t s[LSG_PL];
#pragma unroll
    for (int j = 0; j < LSG_PL; j++) s[j] = acc[j] + bcc[j];
    r = slp_carry(s);
  }
  if (((d >> 15) & 1u) && kind != 0u) {
    fp_t a = kind == 2u ? fp_from_be_bytes(inp + 48 * (w0 >> 20), 12) : slp_carry(acc);
    if (kind == 3u) a = pair_inv_gcd(pair_canon_small(a));  // INV: the GCD inverse, then * R^3
    const fp_t b = slp_carry(bcc);
    pair_mont_mul_n<1>(&r, &a, &b);
  }
  slot_store(lds, w0 & 1023u, h, r);
}

// canonical value of an output slot (|v| < 2p after the program's final product with 1)
LSG_PFN fp_t slp_output(const uint32_t* lds, uint32_t s, uint32_t h) { return pair_canon_small(slot_load(lds, s, h)); }
