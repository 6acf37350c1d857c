// lsg_slp_exec.hpp -- one operation of a straight-line program (tools/gen_slp.py), shared
// by the gfx950 interpreter kernel (lsg_slp.hip, LSG_PAIR_G = 2: a lane pair per operation)
// and the host build of the pair backend (tests/native/hostcheck.hip, LSG_PAIR_G = 1: all 14
// limbs in one "lane"), so the exact device arithmetic -- gathers, carry round, lazy bounds,
// LDS layout -- is checked against the oracle without a GPU.  Include after lsg_fp_pair.hpp.
#pragma once

// LDS slot s: 16 words; lane h of a pair holds its LSG_PL limbs at words s*16 + h*8 ..
LSG_PFN fp_t slot_load(const uint32_t* lds, uint32_t s, uint32_t h) {
  const uint32_t* p = lds + s * 16 + h * 8;
  fp_t r;
#if LSG_PAIR_G == 2
  const uint4 a = *(const uint4*)p;
  const uint3 b = *(const uint3*)(p + 4);
  r.l[0] = a.x;
  r.l[1] = a.y;
  r.l[2] = a.z;
  r.l[3] = a.w;
  r.l[4] = b.x;
  r.l[5] = b.y;
  r.l[6] = b.z;
#else
  for (int k = 0; k < LSG_PL; k++) r.l[k] = p[k];
#endif
  return r;
}
LSG_PFN void slot_store(uint32_t* lds, uint32_t s, uint32_t h, const fp_t& v) {
  uint32_t* p = lds + s * 16 + h * 8;
#if LSG_PAIR_G == 2
  *(uint4*)p = make_uint4(v.l[0], v.l[1], v.l[2], v.l[3]);
  *(uint3*)(p + 4) = make_uint3(v.l[4], v.l[5], v.l[6]);
#else
  for (int k = 0; k < LSG_PL; k++) p[k] = v.l[k];
#endif
}

// acc += coef * slot for the terms [0, n) of a 7-term half (t: slot | coef << 10, 16 bits)
LSG_PFN void slp_gather(int64_t* acc, const uint32_t* lds, const uint32_t* t, uint32_t n, uint32_t h) {
#pragma unroll
  for (int k = 0; k < 7; k++) {
    if ((uint32_t)k < n) {
      const uint32_t w = t[k];
      const fp_t v = slot_load(lds, w & 1023u, h);
      const int32_t c = (int32_t)(w << 16) >> 26;  // bits 10..15, signed
#pragma unroll
      for (int j = 0; j < LSG_PL; j++) acc[j] += (int64_t)c * (int64_t)(int32_t)v.l[j];
    }
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

// operation entry e (8 words): w0 = dst | kind << 10 | nA << 12 | nB << 16 | input << 20,
// then 14 16-bit terms (A at 0..6, B at 7..13).  inp: the item's input blob (LOADMUL).
LSG_PFN void slp_exec(uint32_t* lds, const uint32_t* e, const uint8_t* inp, uint32_t h) {
  const uint32_t w0 = e[0];
  const uint32_t kind = (w0 >> 10) & 3u, nA = (w0 >> 12) & 15u, nB = (w0 >> 16) & 15u;
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
  slp_gather(acc, lds, ta, nA, h);
  slp_gather(bcc, lds, tb, nB, h);
  fp_t r;
  if (kind == 0u) {
#pragma unroll
    for (int j = 0; j < LSG_PL; j++) acc[j] += bcc[j];
    r = slp_carry(acc);
  } else {
    fp_t a = kind == 2u ? fp_from_be_bytes(inp + 48 * (w0 >> 20), 12) : slp_carry(acc);
    const fp_t b = slp_carry(bcc);
    pair_mont_mul_n<1>(&r, &a, &b);
  }
  slot_store(lds, w0 & 1023u, h, r);
}

// canonical value of an output slot (|v| < 2p after the program's final product with 1)
LSG_PFN fp_t slp_output(const uint32_t* lds, uint32_t s, uint32_t h) { return pair_canon_small(slot_load(lds, s, h)); }
