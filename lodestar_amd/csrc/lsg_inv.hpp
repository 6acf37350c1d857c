// Fp inversion by Bernstein-Yang divsteps, variable time (every input of the verifier is
// public), for the straight-line programs (lsg_slp_exec.hpp INV operations).
//
// A Fermat inversion a^(p-2) is ~460 dependent products; here one lane pair runs the
// extended binary GCD instead: batches of 30 divsteps computed on the low 32 bits of f and g
// (the first 30 divsteps depend on nothing else), each batch's 2x2 transition matrix applied
// to f, g and to the cofactors d, e held as 13 signed 30-bit limbs (one v_mad_i64_i32 per
// limb product), d and e kept divisible by 2^30 modulo p with p^-1 mod 2^30.  Invariants:
// f = d x, g = e x (mod p), f = p and g = x initially; when g reaches 0, f = +-gcd = +-1 and
// x^-1 = +-d.  Both lanes of a pair run the same code (the result is split back into the
// pair's two halves).  Include after lsg_fp_pair.hpp.
#pragma once

struct s30_t {
  int32_t v[13];  // value = sum v[i] 2^(30 i); v[0..11] in [0, 2^30) after normalisation, v[12] signed
};
constexpr uint32_t LSG_M30 = (1u << 30) - 1;

// 30 divsteps on the low bits: returns delta; t = [u v; q r] with
// (f', g') = (u f + v g, q f + r g) / 2^30 after the batch
LSG_PFN int32_t by_divsteps30(int32_t delta, uint32_t f, uint32_t g, int32_t* t) {
  int32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll 1
  for (int i = 0; i < 30; i++) {
    const bool godd = (g & 1u) != 0;
    if (delta > 0 && godd) {  // (f, g) <- (g, (g - f) / 2)
      delta = 1 - delta;
      const uint32_t nf = g;
      g = (g - f) >> 1;
      f = nf;
      const int32_t nq = q - u, nr = r - v;
      u = 2 * q;
      v = 2 * r;
      q = nq;
      r = nr;
    } else if (godd) {  // g <- (g + f) / 2
      delta = 1 + delta;
      g = (g + f) >> 1;
      q += u;
      r += v;
      u *= 2;
      v *= 2;
    } else {  // g <- g / 2
      delta = 1 + delta;
      g >>= 1;
      u *= 2;
      v *= 2;
    }
  }
  t[0] = u;
  t[1] = v;
  t[2] = q;
  t[3] = r;
  return delta;
}

// (f, g) <- (u f + v g, q f + r g) / 2^30 (exact)
LSG_PFN void by_update_fg(s30_t& f, s30_t& g, const int32_t* t) {
  int64_t cf = (int64_t)t[0] * f.v[0] + (int64_t)t[1] * g.v[0];
  int64_t cg = (int64_t)t[2] * f.v[0] + (int64_t)t[3] * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 13; i++) {
    cf += (int64_t)t[0] * f.v[i] + (int64_t)t[1] * g.v[i];
    cg += (int64_t)t[2] * f.v[i] + (int64_t)t[3] * g.v[i];
    f.v[i - 1] = (int32_t)((uint32_t)cf & LSG_M30);
    g.v[i - 1] = (int32_t)((uint32_t)cg & LSG_M30);
    cf >>= 30;
    cg >>= 30;
  }
  f.v[12] = (int32_t)cf;
  g.v[12] = (int32_t)cg;
}

// (d, e) <- (u d + v e + md p, q d + r e + me p) / 2^30 with md, me making the sums divisible
// (|md|, |me| <= 2^29: |d'| <= max(|d|, |e|) + p / 2)
LSG_PFN void by_update_de(s30_t& d, s30_t& e, const int32_t* t, const s30_t& p, uint32_t pinv30) {
  int64_t cd = (int64_t)t[0] * d.v[0] + (int64_t)t[1] * e.v[0];
  int64_t ce = (int64_t)t[2] * d.v[0] + (int64_t)t[3] * e.v[0];
  int32_t md = (int32_t)((0u - (uint32_t)cd * pinv30) & LSG_M30);
  int32_t me = (int32_t)((0u - (uint32_t)ce * pinv30) & LSG_M30);
  if (md >= (1 << 29)) md -= 1 << 30;
  if (me >= (1 << 29)) me -= 1 << 30;
  cd += (int64_t)md * p.v[0];
  ce += (int64_t)me * p.v[0];
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 13; i++) {
    cd += (int64_t)t[0] * d.v[i] + (int64_t)t[1] * e.v[i] + (int64_t)md * p.v[i];
    ce += (int64_t)t[2] * d.v[i] + (int64_t)t[3] * e.v[i] + (int64_t)me * p.v[i];
    d.v[i - 1] = (int32_t)((uint32_t)cd & LSG_M30);
    e.v[i - 1] = (int32_t)((uint32_t)ce & LSG_M30);
    cd >>= 30;
    ce >>= 30;
  }
  d.v[12] = (int32_t)cd;
  e.v[12] = (int32_t)ce;
}

// 14 radix-2^29 limbs (non-negative, normalised) -> 13 radix-2^30 limbs
LSG_PFN s30_t s30_from_l29(const uint32_t* L) {
  s30_t r;
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const int bit = 30 * i, k = bit / 29, s = bit % 29;
    uint64_t x = (uint64_t)L[k] >> s;
    if (k + 1 < 14) x |= (uint64_t)L[k + 1] << (29 - s);
    if (k + 2 < 14 && 58 - s < 30) x |= (uint64_t)L[k + 2] << (58 - s);
    r.v[i] = (int32_t)((uint32_t)x & LSG_M30);
  }
  return r;
}

// the pair half of a signed 13 x 30-bit value (v[0..11] normalised): limbs 7h .. 7h + 6 of its
// radix-2^29 form, limb 13 signed
LSG_PFN fp_t s30_to_pair(const s30_t& a) {
  uint32_t L[14];
#pragma unroll
  for (int k = 0; k < 14; k++) {
    const int bit = 29 * k, i = bit / 30, s = bit % 30;
    if (k == 13) {
      L[k] = (uint32_t)(a.v[12] >> 17);  // bits 377.. (limb 12 holds bits 360..), signed
    } else {
      uint64_t x = (uint64_t)(uint32_t)a.v[i] >> s;
      if (i + 1 < 13) x |= (uint64_t)(uint32_t)a.v[i + 1] << (30 - s);
      L[k] = (uint32_t)x & LSG_M29;
    }
  }
  return fp_from_arr(L);
}

// x^-1 mod p as a lazy integer (|result| < 2^387) for a canonical x in [0, p) (0 -> 0)
LSG_PFN fp_t pair_inv_gcd(const fp_t& x) {
  uint32_t L[14], PL_[14];
  pair_gather(L, x);
#pragma unroll
  for (int k = 0; k < 14; k++) PL_[k] = LSG_P[k];
  const s30_t p = s30_from_l29(PL_);
  uint32_t pinv = p.v[0];  // Newton: p^-1 mod 2^32 from p (odd)
#pragma unroll
  for (int i = 0; i < 5; i++) pinv *= 2u - (uint32_t)p.v[0] * pinv;
  pinv &= LSG_M30;
  s30_t f = p, g = s30_from_l29(L), d, e;
#pragma unroll
  for (int i = 0; i < 13; i++) d.v[i] = e.v[i] = 0;
  e.v[0] = 1;
  int32_t delta = 1;
#pragma unroll 1
  for (int it = 0; it < 48; it++) {  // 1440 divsteps > the 1103 any 381-bit input needs
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 13; i++) nz |= (uint32_t)g.v[i];
    if (nz == 0u) break;
    int32_t t[4];
    delta = by_divsteps30(delta, (uint32_t)f.v[0] | ((uint32_t)f.v[1] << 30), (uint32_t)g.v[0] | ((uint32_t)g.v[1] << 30), t);
    by_update_fg(f, g, t);
    by_update_de(d, e, t, p, pinv);
  }
  if (f.v[12] < 0) {  // f = -1: x^-1 = -d, renormalised
#pragma unroll
    for (int i = 0; i < 13; i++) d.v[i] = -d.v[i];
#pragma unroll
    for (int i = 0; i < 12; i++) {
      const int32_t c = d.v[i] >> 30;
      d.v[i] &= (int32_t)LSG_M30;
      d.v[i + 1] += c;
    }
  }
  return s30_to_pair(d);
}
