// Canonical (big-endian, non-Montgomery) byte forms of tower and curve values, shared by the
// translation units of the two Fp backends (lsg_bls.hip: quad, lsg_serial.hip: row).  These
// 576/288-byte blobs are the hand-off format between backends and across GPUs (the Fp12
// Miller partial of SURVEY.md 8e).
#pragma once
#include "lsg_pairing.hpp"

// Fp12 as 12 canonical 48-byte Fp in tower order (c0.c0.c0, c0.c0.c1, c0.c1.c0, ...)
LSG_DEVI fp12_t fp12_from_canon_bytes(const uint8_t* b) {
  fp12_t f;
  fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int j = 0; j < 6; j++) {
    c[j]->c0 = fp_to_mont(fp_from_be48(b + 96 * j));
    c[j]->c1 = fp_to_mont(fp_from_be48(b + 96 * j + 48));
  }
  return f;
}
LSG_DEVI void fp12_to_canon_bytes(uint8_t* o, const fp12_t& f) {
  const fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int j = 0; j < 6; j++) {
    fp_to_be48(o + 96 * j, fp_from_mont(c[j]->c0));
    fp_to_be48(o + 96 * j + 48, fp_from_mont(c[j]->c1));
  }
}
// homogeneous projective G2 point as 6 canonical Fp (X.c0, X.c1, Y.c0, Y.c1, Z.c0, Z.c1)
LSG_DEVI g2p_t g2p_from_canon_bytes(const uint8_t* b) {
  g2p_t p;
  fp2_t* c[3] = {&p.X, &p.Y, &p.Z};
  for (int j = 0; j < 3; j++) {
    c[j]->c0 = fp_to_mont(fp_from_be48(b + 96 * j));
    c[j]->c1 = fp_to_mont(fp_from_be48(b + 96 * j + 48));
  }
  return p;
}
LSG_DEVI void g2p_to_canon_bytes(uint8_t* o, const g2p_t& p) {
  const fp2_t* c[3] = {&p.X, &p.Y, &p.Z};
  for (int j = 0; j < 3; j++) {
    fp_to_be48(o + 96 * j, fp_from_mont(c[j]->c0));
    fp_to_be48(o + 96 * j + 48, fp_from_mont(c[j]->c1));
  }
}
