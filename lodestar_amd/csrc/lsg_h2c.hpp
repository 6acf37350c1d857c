// hash_to_G2 for gfx950: RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_ as used by blst's
// Pairing(hash_or_encode = true, DST) inside @chainsafe/blst verifyMultipleAggregateSignatures
// (reached from packages/beacon-node/src/chain/bls/maybeBatch.ts:18,37).
//   expand_message_xmd (SHA-256) -> hash_to_field (4 Fp) -> simplified SWU on E2'
//   -> 3-isogeny -> Q0 + Q1 -> clear_cofactor (psi form) .
// Mirrors oracle/hash_to_curve.py step for step.
#pragma once
#include "lsg_curve.hpp"

// ------------------------------------------------------------------ SHA-256
LSG_CONST uint32_t SHA_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

LSG_INL uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

LSG_BIGFN void sha256_compress(uint32_t* st, const uint32_t* blk) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + SHA_K[i] + wi;
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

// Streaming SHA-256 over bytes (messages here are < 2^32 bits).
struct sha256_ctx {
  uint32_t st[8];
  uint32_t blk[16];
  uint32_t n;      // bytes in current block
  uint32_t total;  // total bytes
};

LSG_INL void sha256_init(sha256_ctx& c) {
  c.st[0] = 0x6a09e667u;
  c.st[1] = 0xbb67ae85u;
  c.st[2] = 0x3c6ef372u;
  c.st[3] = 0xa54ff53au;
  c.st[4] = 0x510e527fu;
  c.st[5] = 0x9b05688cu;
  c.st[6] = 0x1f83d9abu;
  c.st[7] = 0x5be0cd19u;
  for (int i = 0; i < 16; i++) c.blk[i] = 0;
  c.n = 0;
  c.total = 0;
}

LSG_INL void sha256_byte(sha256_ctx& c, uint8_t v) {
  uint32_t wi = c.n >> 2, sh = 24 - 8 * (c.n & 3);
  c.blk[wi] |= (uint32_t)v << sh;
  c.n++;
  c.total++;
  if (c.n == 64) {
    sha256_compress(c.st, c.blk);
    for (int i = 0; i < 16; i++) c.blk[i] = 0;
    c.n = 0;
  }
}

LSG_INL void sha256_bytes(sha256_ctx& c, const uint8_t* p, uint32_t len) {
  for (uint32_t i = 0; i < len; i++) sha256_byte(c, p[i]);
}

LSG_INL void sha256_final(sha256_ctx& c, uint32_t* out8) {
  uint32_t bits = c.total * 8;
  sha256_byte(c, 0x80);
  while (c.n != 56) sha256_byte(c, 0);
  c.blk[14] = 0;
  c.blk[15] = bits;
  sha256_compress(c.st, c.blk);
  for (int i = 0; i < 8; i++) out8[i] = c.st[i];
}

LSG_INL void be_words_to_bytes(uint8_t* out, const uint32_t* w, int nw) {
  for (int i = 0; i < nw; i++) {
    out[4 * i] = (uint8_t)(w[i] >> 24);
    out[4 * i + 1] = (uint8_t)(w[i] >> 16);
    out[4 * i + 2] = (uint8_t)(w[i] >> 8);
    out[4 * i + 3] = (uint8_t)w[i];
  }
}

// expand_message_xmd(msg, DST, 256) -> 256 bytes   (RFC 9380 section 5.3.1)
LSG_INL void expand_message_xmd_256(uint8_t* out, const uint8_t* msg, uint32_t msg_len, const uint8_t* dst,
                                    uint32_t dst_len) {
  sha256_ctx c;
  uint32_t b0[8], bi[8];
  sha256_init(c);
  for (int i = 0; i < 64; i++) sha256_byte(c, 0);  // Z_pad
  sha256_bytes(c, msg, msg_len);
  sha256_byte(c, 1);  // l_i_b_str = 256 (2 bytes, big endian)
  sha256_byte(c, 0);
  sha256_byte(c, 0);  // I2OSP(0, 1)
  sha256_bytes(c, dst, dst_len);
  sha256_byte(c, (uint8_t)dst_len);
  sha256_final(c, b0);
  for (int i = 1; i <= 8; i++) {
    sha256_init(c);
    for (int k = 0; k < 8; k++) {
      uint32_t v = (i == 1) ? b0[k] : (b0[k] ^ bi[k]);
      sha256_byte(c, (uint8_t)(v >> 24));
      sha256_byte(c, (uint8_t)(v >> 16));
      sha256_byte(c, (uint8_t)(v >> 8));
      sha256_byte(c, (uint8_t)v);
    }
    sha256_byte(c, (uint8_t)i);
    sha256_bytes(c, dst, dst_len);
    sha256_byte(c, (uint8_t)dst_len);
    sha256_final(c, bi);
    be_words_to_bytes(out + 32 * (i - 1), bi, 8);
  }
}

// 64 big-endian bytes -> element mod p, Montgomery form.  Split N into three pieces that
// are each < p (a Montgomery product needs both inputs < p):
//   N = hi * 2^384 + mid * 2^256 + lo,  hi, mid < 2^128, lo < 2^256
//   mont(N) = mont_mul(lo, R^2) + mont_mul(mid, 2^256 R^2) + mont_mul(hi, R^3)
LSG_INL fp_t fp_from_be64_mod(const uint8_t* b) {
  fp_t lo = fp_from_be_bytes(b + 32, 8);
  fp_t mid = fp_from_be_bytes(b + 16, 4);
  fp_t hi = fp_from_be_bytes(b, 4);
  return fp_add(fp_add(fp_mul(lo, fp_t(FP_R2)), fp_mul(mid, fp_t(FP_R2_SHL256))), fp_mul(hi, fp_t(FP_R3)));
}

// ------------------------------------------------------------------ SSWU on E2' (RFC 9380 6.6.2)
// One exponentiation decides between x1 and x2 for every row of the wave at once (no
// divergent second square root): with gx2 = (Z u^2)^3 gx1 and N(Z) = 5 a non-square in Fp,
// if N(gx1) is a non-square then
//   sqrt(N(gx2)) = N(Z u^2) N(u) (N(Z) N(gx1))^((p+1)/4) = N(Z u^2) N(u) 5^((p+1)/4) s1,
// where s1 = N(gx1)^((p+1)/4) is the candidate already computed.  The root of gx (x1 or
// x2) then costs one more exponentiation.  The result equals RFC 9380's: the square root
// is unique up to sign and the sign is fixed by sgn0 below.
//
// The one inversion, 1/tv1 = conj(tv1) / N(tv1), is split out so that a batch of sets can
// share one field inversion for all its N(tv1) (Montgomery's trick, done by the caller):
// sswu_tv1(u) gives tv1, and map_to_curve_sswu_ni(u, ni) finishes with ni = 1/N(tv1)
// (ni = 0 when tv1 = 0, the exceptional case, as fp_inv(0) = 0 gives).
LSG_INL fp2_t sswu_tv1(const fp2_t& u) {
  fp2_t zu2 = fp2_mul(SSWU_Z, fp2_sqr(u));
  return fp2_add(fp2_sqr(zu2), zu2);
}
LSG_INL fp2_t fp2_inv_with_norm_inv(const fp2_t& a, const fp_t& ni) {
  return fp2_t(fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni)));
}
LSG_BIGFN g2a_t map_to_curve_sswu_ni(fp2_t u, fp_t ni) {
  fp2_t u2 = fp2_sqr(u);
  fp2_t zu2 = fp2_mul(SSWU_Z, u2);
  fp2_t tv1 = fp2_add(fp2_sqr(zu2), zu2);
  bool exc = fp2_is_zero(tv1);
  fp2_t x1 = fp2_mul(SSWU_MINUS_B_OVER_A, fp2_add(fp2_one(), fp2_inv_with_norm_inv(tv1, ni)));
  x1 = fp2_select(exc, SSWU_B_OVER_ZA, x1);
  fp2_t gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), SSWU_A), x1), SSWU_B);
  fp2_t x2 = fp2_mul(zu2, x1);
  fp2_t gx2 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x2), SSWU_A), x2), SSWU_B);
  bool sq1;
  fp_t s1 = fp2_norm_sqrt_candidate(gx1, &sq1);
  fp_t s2 = fp_mul(fp_mul(fp2_norm(zu2), fp2_norm(u)), fp_mul(s1, fp_t(SSWU_NZ_POW_P1D4)));
  g2a_t r;
  r.x = fp2_select(sq1, x1, x2);
  fp2_t y;
  (void)fp2_sqrt_with_norm_root(y, fp2_select(sq1, gx1, gx2), fp_select(sq1, s1, s2));
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  r.y = y;
  return r;
}
LSG_BIGFN g2a_t map_to_curve_sswu(fp2_t u) { return map_to_curve_sswu_ni(u, fp_inv(fp2_norm(sswu_tv1(u)))); }

// 3-isogeny E2' -> E2, projective output (X, Y, Z) = (xn yd, y yn xd, xd yd)
LSG_BIGFN g2p_t iso_map3(g2a_t p) {
  const fp2_t& x = p.x;
  fp2_t xn = fp2_add(fp2_mul(fp2_add(fp2_mul(fp2_add(fp2_mul(ISO_XNUM_3, x), ISO_XNUM_2), x), ISO_XNUM_1), x),
                     ISO_XNUM_0);
  fp2_t xd = fp2_add(fp2_mul(fp2_add(x, ISO_XDEN_1), x), ISO_XDEN_0);
  fp2_t yn = fp2_add(fp2_mul(fp2_add(fp2_mul(fp2_add(fp2_mul(ISO_YNUM_3, x), ISO_YNUM_2), x), ISO_YNUM_1), x),
                     ISO_YNUM_0);
  fp2_t yd = fp2_add(fp2_mul(fp2_add(fp2_mul(fp2_add(x, ISO_YDEN_2), x), ISO_YDEN_1), x), ISO_YDEN_0);
  g2p_t r;
  r.X = fp2_mul(xn, yd);
  r.Y = fp2_mul(fp2_mul(p.y, yn), xd);
  r.Z = fp2_mul(xd, yd);
  if (fp2_is_zero(r.Z)) r = proj_inf<fp2_t>();
  return r;
}

// h_eff * P = [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P)   (RFC 9380 appendix G.3), as
// c + [x]([x]P + psi(P)) with c = psi^2(2P) - psi(P) - P - [x]P: the terms are folded into c
// as soon as they exist, so each [x] chain runs with one other point live (registers, not
// scratch).
LSG_BIGFN g2p_t clear_cofactor_g2(g2p_t p) {
  const g2p_t u = g2_psi(p);
  g2p_t c = g2_add(g2_psi2(g2_dbl(p)), proj_neg(u));
  c = g2_add(c, proj_neg(p));
  const g2p_t t1 = proj_neg(proj_mul_xabs(p));  // [x]P
  c = g2_add(c, proj_neg(t1));
  const g2p_t t2 = proj_neg(proj_mul_xabs(g2_add(t1, u)));  // [x]([x]P + psi(P))
  return g2_add(c, t2);
}
// The same sum for a per-set kernel with one parked point (get/put: a per-lane LDS slot
// holding P on entry) and one point parked in the caller's global slot (cput/cget): the [x]
// chains run with their base in LDS and only the accumulator in registers, and no step in
// between holds more than two points.
template <class G, class P, class CP, class CG>
LSG_INL g2p_t clear_cofactor_g2_parked(const G& get, const P& put, const CP& cput, const CG& cget) {
  cput(proj_neg(proj_mul_xabs_get<fp2_t>(get)));  // t1 = [x]P
  g2p_t c;
  {
    const g2p_t p = get();
    c = g2_add(g2_psi2(g2_dbl(p)), proj_neg(p));
    put(g2_psi(p));  // u = psi(P)
  }
  c = g2_add(c, proj_neg(get()));
  const g2p_t t1 = cget();
  cput(g2_add(c, proj_neg(t1)));  // c = psi^2(2P) - P - psi(P) - [x]P
  put(g2_add(t1, get()));         // [x]P + psi(P)
  const g2p_t t2 = proj_neg(proj_mul_xabs_get<fp2_t>(get));  // [x]([x]P + psi(P))
  return g2_add(cget(), t2);
}
