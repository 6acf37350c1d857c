// Canonical (big-endian, non-Montgomery) byte forms of tower and curve values, shared by the
// translation units of the two Fp backends (lsg_bls.hip: quad, lsg_serial.hip: row).  These
// 576/288-byte blobs are the hand-off format between backends and across GPUs (the Fp12
// Miller partial of SURVEY.md 8e).
#pragma once
#include "lsg_pairing.hpp"

// The conversions to and from Montgomery form are issued as one batch of independent
// products (fp_mul_list): the row backend splits a batch over the rows that share an item.
template <int N>
LSG_DEVI void fps_from_canon_bytes(fp_t* v, const uint8_t* b) {
  fp_t x[N], r2[N];
#pragma unroll
  for (int k = 0; k < N; k++) {
    x[k] = fp_from_be48(b + 48 * k);
    r2[k] = fp_t(FP_R2);
  }
  fp_mul_list<N>(v, x, r2);
}
template <int N>
LSG_DEVI void fps_to_canon_bytes(uint8_t* o, const fp_t* v) {
  fp_t one[N], c[N];
#pragma unroll
  for (int k = 0; k < N; k++) one[k] = fp_t(FP_ONE_CANON);
  fp_mul_list<N>(c, v, one);
#pragma unroll
  for (int k = 0; k < N; k++) fp_to_be48(o + 48 * k, fp_canonical(c[k]));
}

// Fp12 as 12 canonical 48-byte Fp in tower order (c0.c0.c0, c0.c0.c1, c0.c1.c0, ...)
LSG_DEVI fp12_t fp12_from_canon_bytes(const uint8_t* b) {
  fp_t v[12];
  fps_from_canon_bytes<12>(v, b);
  fp12_t f;
  fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
#pragma unroll
  for (int j = 0; j < 6; j++) *c[j] = fp2_t(v[2 * j], v[2 * j + 1]);
  return f;
}
LSG_DEVI void fp12_to_canon_bytes(uint8_t* o, const fp12_t& f) {
  const fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  fp_t v[12];
#pragma unroll
  for (int j = 0; j < 6; j++) {
    v[2 * j] = c[j]->c0;
    v[2 * j + 1] = c[j]->c1;
  }
  fps_to_canon_bytes<12>(o, v);
}
// homogeneous projective G2 point as 6 canonical Fp (X.c0, X.c1, Y.c0, Y.c1, Z.c0, Z.c1)
LSG_DEVI g2p_t g2p_from_canon_bytes(const uint8_t* b) {
  fp_t v[6];
  fps_from_canon_bytes<6>(v, b);
  g2p_t p;
  p.X = fp2_t(v[0], v[1]);
  p.Y = fp2_t(v[2], v[3]);
  p.Z = fp2_t(v[4], v[5]);
  return p;
}
LSG_DEVI void g2p_to_canon_bytes(uint8_t* o, const g2p_t& p) {
  const fp_t v[6] = {p.X.c0, p.X.c1, p.Y.c0, p.Y.c1, p.Z.c0, p.Z.c1};
  fps_to_canon_bytes<6>(o, v);
}
