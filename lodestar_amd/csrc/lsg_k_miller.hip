// lsg_k_miller.hip -- the per-set half of the RLC multi-Miller loop (blst miller_loop_n under
// Pairing.commit(), packages/beacon-node/src/chain/bls/maybeBatch.ts:18),
// split into its G2 side and its Fp12 side (lsg_pairing.hpp miller_lines /
// miller_accum_multi, host-checked equal to the product of single loops):
//   k_miller_lines   the 68 unevaluated lines of Q_i = H(m_i) for every set
//   k_miller_accum   f_item = prod over the item's <= K sets of their lines at P_i, K pairs
//                    sharing one f and its squarings
#include "lsg_kcommon.hpp"

// Line storage is word-major over sets: word k (of the W per lane of a line_t) of step st of
// set i lives at lines[((st * W + k) * n + i) * G + h], so one store or load instruction of a
// wave touches one contiguous 256-byte run.  ML_STEPS lines = 68 x 6 Fp per set (~22.8 KB).
constexpr int W_LINE_LANE = (int)(sizeof(line_t) / 4);
LSG_DEVI void line_store(uint32_t* __restrict__ lines, size_t n, size_t i, int st, const line_t& L) {
  uint32_t w[W_LINE_LANE];
  __builtin_memcpy(w, &L, sizeof(line_t));
  uint32_t* p = lines + (((size_t)st * W_LINE_LANE) * n + i) * LSG_GROUP + (threadIdx.x % LSG_GROUP);
#pragma unroll
  for (int k = 0; k < W_LINE_LANE; k++) p[(size_t)k * n * LSG_GROUP] = w[k];
}
LSG_DEVI line_t line_load(const uint32_t* __restrict__ lines, size_t n, size_t i, int st) {
  uint32_t w[W_LINE_LANE];
  const uint32_t* p = lines + (((size_t)st * W_LINE_LANE) * n + i) * LSG_GROUP + (threadIdx.x % LSG_GROUP);
#pragma unroll
  for (int k = 0; k < W_LINE_LANE; k++) w[k] = p[(size_t)k * n * LSG_GROUP];
  line_t L;
  __builtin_memcpy(&L, w, sizeof(line_t));
  return L;
}

// the G2 half: the 68 unevaluated lines of Q_i = H(m_i) for every set (no dependency on the
// pubkey side, so it runs as soon as hash_to_G2 is done).  Sets whose point is unusable still
// run the chain on whatever Q holds: every lane pair follows one control path.
__global__ void LSG_KERNEL_ATTR k_miller_lines(int n, const uint32_t* __restrict__ H, uint32_t* __restrict__ lines) {
  LANE_ITEM(n);
  (void)lead;
  const g2a_t Q = lane_load<g2a_t>(H, item);
  miller_lines(Q, [&](int st, const line_t& L) { line_store(lines, (size_t)n, item, st, L); });
}

// the Fp12 half: f_item = prod over the item's <= K sets of their lines evaluated at P_i,
// with shared squarings.  Sets with errors or an infinite point contribute 1.
#ifndef LSG_ACCUM_WAVES
#define LSG_ACCUM_WAVES 1  // 512 registers: f, the line and the products stay out of scratch (1.33M -> 1.43M sets/s)
#endif
template <int K>
__global__ void LSG_KERNEL_ATTR_W(LSG_ACCUM_WAVES)
    k_miller_accum(int n_items, const int32_t* __restrict__ item_first, const int32_t* __restrict__ item_cnt,
                   const uint32_t* __restrict__ P, const uint8_t* __restrict__ pinf, const uint8_t* __restrict__ hinf,
                   const int32_t* __restrict__ err, int n_sets, const uint32_t* __restrict__ lines,
                   uint32_t* __restrict__ f) {
  LANE_ITEM(n_items);
  (void)lead;
  const int first = item_first[item], cnt = item_cnt[item];
  g1a_t Pk[K];
  bool use[K];
  int idx[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int i = first + (k < cnt ? k : cnt - 1);
    idx[k] = i;
    use[k] = k < cnt && err[i] == 0 && !pinf[i] && !hinf[i];
    Pk[k] = lane_load<g1a_t>(P, i);
  }
  lane_store(f, item, miller_accum_multi<K>(Pk, use, [&](int k, int st) {
               return line_load(lines, (size_t)n_sets, (size_t)idx[k], st);
             }));
}

// ---- list form (fallback phases of single-set jobs): item k is the one pair of set list[k];
// its lines are stored at position k (a fallback phase touches a few thousand of a package's
// sets), then accumulated alone -- the fused kernel would spend four waves on one pair
__global__ void LSG_KERNEL_ATTR k_miller_lines_list(int n, const int32_t* __restrict__ list, const uint32_t* __restrict__ H,
                                                    uint32_t* __restrict__ lines) {
  LANE_ITEM(n);
  (void)lead;
  const g2a_t Q = lane_load<g2a_t>(H, (size_t)list[item]);
  miller_lines(Q, [&](int st, const line_t& L) { line_store(lines, (size_t)n, item, st, L); });
}
__global__ void LSG_KERNEL_ATTR_W(LSG_ACCUM_WAVES)
    k_miller_accum_list(int n, const int32_t* __restrict__ list, const uint32_t* __restrict__ P,
                        const uint8_t* __restrict__ pinf, const uint8_t* __restrict__ hinf, const int32_t* __restrict__ err,
                        const uint32_t* __restrict__ lines, uint32_t* __restrict__ f) {
  LANE_ITEM(n);
  (void)lead;
  const int i = list[item];
  g1a_t Pk[1] = {lane_load<g1a_t>(P, (size_t)i)};
  bool use[1] = {err[i] == 0 && !pinf[i] && !hinf[i]};
  lane_store(f, item, miller_accum_multi<1>(Pk, use, [&](int, int st) { return line_load(lines, (size_t)n, item, st); }));
}

// ---- Fused Miller kernel: lines computed and consumed in LDS (north_star: "line coefficients
// staged in LDS"), the Fp12 accumulator of each item shared by four waves.
//
// A workgroup is 4 waves and owns 32 items of <= 4 sets (MF_ITEMS).  Lane pair q of every
// wave works on item q; wave w is "pair w" of its item and keeps that pair's G2 point T in
// LDS:
//   L phase   wave w advances T (doubling or addition step), evaluates the line at its P and
//             writes it to LDS (the identity line (1, 0, 0) for a set that does not
//             contribute) -- the four lines of an item come out in parallel;
//   P phase   the lines are multiplied in pairs, M01 = l0 l1 and M23 = l2 l3 (sparse x sparse:
//             6 Fp2 products each, three per wave), into the slots of the lines;
//   S phase   f <- f^2: the 12 Fp2 products of (a + b w)^2 = (u - t - v t) + 2t w,
//             t = a b, u = (a + b)(a + v b), three per wave, then the six output
//             coefficients combined by the waves in parallel;
//   M phase   f <- f * M for M = M01, M23: 17 Fp2 products (Karatsuba over Fp6 with the
//             second half of M sparse) split 5/4/4/4, then the six output coefficients.
// Per doubling that is 12 + 12 + 34 Fp2 products in phases of 3, 3, 5 and 5 per wave, where
// four line multiplications (13 products each, split 4/3/3/3) were 12 + 52 in phases of 3 and
// 4 x 4.  f, the lines, the products and the points live in LDS only (158 KB per workgroup), so a set's
// HBM traffic is its inputs (Q, P, flags) and 1/4 of its item's f: no line round trip.  The
// operation order differs from miller_accum_multi, the field element is the same: the
// host-checked split loop and the GPU parity tests pin it.
constexpr int MF_ITEMS = 32;
// LDS components (one Fp of 32 items each): f, the four lines (then M01, M23), the products,
// the four G2 points T.  Products V15 and V16 of the M phase use the third coefficient slots of
// lines 1 and 3, which M01 and M23 leave free, so that everything fits 160 KB.
constexpr int MF_F = 0, MF_L = 12, MF_V = 36, MF_T = 66, MF_COMPS = 90;
constexpr size_t MF_LDS_BYTES = (size_t)MF_COMPS * 7 * 64 * 4;  // 161,280 B: one workgroup per CU

LSG_DEVI uint32_t* mf_slot(uint32_t* lds, int c) { return lds + (size_t)c * 7 * 64 + (threadIdx.x & 63); }
LSG_DEVI void mf_put(uint32_t* lds, int c, const fp_t& v) {
  uint32_t* p = mf_slot(lds, c);
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) p[k * 64] = v.l[k];
}
LSG_DEVI fp_t mf_get(uint32_t* lds, int c) {
  const uint32_t* p = mf_slot(lds, c);
  fp_t v;
#pragma unroll
  for (int k = 0; k < LSG_PL; k++) v.l[k] = p[k * 64];
  return v;
}
LSG_DEVI void mf_put2(uint32_t* lds, int c, const fp2_t& v) {
  mf_put(lds, c, v.c0);
  mf_put(lds, c + 1, v.c1);
}
LSG_DEVI fp2_t mf_get2(uint32_t* lds, int c) { return fp2_t(mf_get(lds, c), mf_get(lds, c + 1)); }
// Fp2 coefficient j (0..5: c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2) of f, product p, line k
#define MF_FC(j) (MF_F + 2 * (j))
#define MF_LC(k, j) (MF_L + 6 * (k) + 2 * (j))
#define MF_VC(p) ((p) < 15 ? MF_V + 2 * (p) : ((p) == 15 ? MF_LC(1, 2) : MF_LC(3, 2)))

// f <- f^2 (S phase).  V0..5: t = a b (v0, v1, v2, m0, m1, m2 of the Karatsuba Fp6 product),
// V6..11: u = (a + b)(a + v b).
LSG_DEVI void mf_sqr(uint32_t* lds, int w) {
  {
    fp6_t x, y;
    const fp6_t a = fp6_make(mf_get2(lds, MF_FC(0)), mf_get2(lds, MF_FC(1)), mf_get2(lds, MF_FC(2)));
    const fp6_t b = fp6_make(mf_get2(lds, MF_FC(3)), mf_get2(lds, MF_FC(4)), mf_get2(lds, MF_FC(5)));
    if (w < 2) {
      x = a;
      y = b;
    } else {
      x = fp6_add(a, b);
      y = fp6_add(a, fp6_mul_v(b));
    }
    fp2_t p0, p1, p2;
    if ((w & 1) == 0) {  // v0, v1, v2
      p0 = fp2_mul(x.c0, y.c0);
      p1 = fp2_mul(x.c1, y.c1);
      p2 = fp2_mul(x.c2, y.c2);
    } else {  // m0 = (x1 + x2)(y1 + y2), m1 = (x0 + x1)(y0 + y1), m2 = (x0 + x2)(y0 + y2)
      p0 = fp2_mul(fp2_add(x.c1, x.c2), fp2_add(y.c1, y.c2));
      p1 = fp2_mul(fp2_add(x.c0, x.c1), fp2_add(y.c0, y.c1));
      p2 = fp2_mul(fp2_add(x.c0, x.c2), fp2_add(y.c0, y.c2));
    }
    mf_put2(lds, MF_VC(3 * w), p0);
    mf_put2(lds, MF_VC(3 * w + 1), p1);
    mf_put2(lds, MF_VC(3 * w + 2), p2);
  }
  __syncthreads();
  // Karatsuba Fp6 combination of t (V0..5): c0 = v0 + xi (m0 - v1 - v2), c1 = m1 - v0 - v1 + xi v2,
  // c2 = m2 - v0 - v2 + v1; likewise u (V6..11).  New f: c0 = u - t - v t, c1 = 2t.
  auto fin = [&](int base, int j) {
    const fp2_t v0 = mf_get2(lds, MF_VC(base)), v1 = mf_get2(lds, MF_VC(base + 1)), v2 = mf_get2(lds, MF_VC(base + 2));
    if (j == 0) return fp2_add(v0, fp2_mul_xi(fp2_sub(fp2_sub(mf_get2(lds, MF_VC(base + 3)), v1), v2)));
    if (j == 1) return fp2_add(fp2_sub(fp2_sub(mf_get2(lds, MF_VC(base + 4)), v0), v1), fp2_mul_xi(v2));
    return fp2_add(fp2_sub(fp2_sub(mf_get2(lds, MF_VC(base + 5)), v0), v2), v1);
  };
  fp2_t o0, o1, o2;
  if (w == 0) {  // c1 = 2t
    o0 = fin(0, 0);
    o1 = fin(0, 1);
    o2 = fin(0, 2);
  } else if (w == 1) {  // c0.c0 = u0 - t0 - xi t2
    o0 = fp2_sub(fp2_sub(fin(6, 0), fin(0, 0)), fp2_mul_xi(fin(0, 2)));
  } else if (w == 2) {  // c0.c1 = u1 - t1 - t0
    o0 = fp2_sub(fp2_sub(fin(6, 1), fin(0, 1)), fin(0, 0));
  } else {  // c0.c2 = u2 - t2 - t1
    o0 = fp2_sub(fp2_sub(fin(6, 2), fin(0, 2)), fin(0, 1));
  }
  // No barrier before or after the writes: f was last read in the product half (before the
  // barrier above) and the combination reads only the products; the next reader of f (the M
  // phase) and the next writer of the product slots (the P phase) both come after the L
  // phase's barrier.  (Round 4 kept two more barriers here.)
  if (w == 0) {
    mf_put2(lds, MF_FC(3), fp2_add(o0, o0));
    mf_put2(lds, MF_FC(4), fp2_add(o1, o1));
    mf_put2(lds, MF_FC(5), fp2_add(o2, o2));
  } else {
    mf_put2(lds, MF_FC(w - 1), o0);
  }
}

// P phase: M01 = l0 l1 into the slots of lines 0 and 1, M23 = l2 l3 into those of 2 and 3.
// For lines l = (l00 + l01 v) + (l11 v) w:  l l' = (m0 + m1 v + m2 v^2) + (m4 v + m5 v^2) w,
//   m0 = P0 + xi P1, m1 = P3 - P0 - P2, m2 = P2, m4 = P4 - P0 - P1, m5 = P5 - P2 - P1, with
//   P0 = l00 l00', P1 = l11 l11', P2 = l01 l01', P3 = (l00 + l01)(l00' + l01'),
//   P4 = (l00 + l11)(l00' + l11'), P5 = (l01 + l11)(l01' + l11').
// Waves 2pi and 2pi + 1 work on pair pi: three products each, then m0..m2 / m4, m5.
LSG_DEVI void mf_pair_lines(uint32_t* lds, int w) {
  const int pi = w >> 1, h = w & 1;
  {
    const fp2_t a0 = mf_get2(lds, MF_LC(2 * pi, 0)), a1 = mf_get2(lds, MF_LC(2 * pi, 1)),
                a2 = mf_get2(lds, MF_LC(2 * pi, 2));
    const fp2_t b0 = mf_get2(lds, MF_LC(2 * pi + 1, 0)), b1 = mf_get2(lds, MF_LC(2 * pi + 1, 1)),
                b2 = mf_get2(lds, MF_LC(2 * pi + 1, 2));
    if (h == 0) {
      mf_put2(lds, MF_VC(6 * pi), fp2_mul(a0, b0));
      mf_put2(lds, MF_VC(6 * pi + 1), fp2_mul(a2, b2));
      mf_put2(lds, MF_VC(6 * pi + 2), fp2_mul(a1, b1));
    } else {
      mf_put2(lds, MF_VC(6 * pi + 3), fp2_mul(fp2_add(a0, a1), fp2_add(b0, b1)));
      mf_put2(lds, MF_VC(6 * pi + 4), fp2_mul(fp2_add(a0, a2), fp2_add(b0, b2)));
      mf_put2(lds, MF_VC(6 * pi + 5), fp2_mul(fp2_add(a1, a2), fp2_add(b1, b2)));
    }
  }
  __syncthreads();
  // the lines of pair pi were read before the barrier: their slots take M
  const fp2_t P0 = mf_get2(lds, MF_VC(6 * pi)), P1 = mf_get2(lds, MF_VC(6 * pi + 1)), P2 = mf_get2(lds, MF_VC(6 * pi + 2));
  if (h == 0) {
    mf_put2(lds, MF_LC(2 * pi, 0), fp2_add(P0, fp2_mul_xi(P1)));
    mf_put2(lds, MF_LC(2 * pi, 1), fp2_sub(fp2_sub(mf_get2(lds, MF_VC(6 * pi + 3)), P0), P2));
    mf_put2(lds, MF_LC(2 * pi, 2), P2);
  } else {
    mf_put2(lds, MF_LC(2 * pi + 1, 0), fp2_sub(fp2_sub(mf_get2(lds, MF_VC(6 * pi + 4)), P0), P1));
    mf_put2(lds, MF_LC(2 * pi + 1, 1), fp2_sub(fp2_sub(mf_get2(lds, MF_VC(6 * pi + 5)), P2), P1));
  }
  __syncthreads();
}

// M phase: f <- f * M for M = (m0, m1, m2) + (0, m4, m5) w in the slots of lines 2k, 2k + 1.
// f = a + b w:  t0 = a M0 (6 products), t1 = b M1 = v n with n = b (m4 + m5 v) (5),
// t2 = (a + b)(M0 + M1) (6);  f' = (t0 + v t1) + (t2 - t0 - t1) w.
//   V0 a0 m0   V1 a1 m1   V2 a2 m2   V3 (a0+a1)(m0+m1)   V4 (a1+a2)(m1+m2)   V5 (a0+a2)(m0+m2)
//   V6 b0 m4   V7 b1 m5   V8 (b0+b1)(m4+m5)   V9 b2 m4   V10 b2 m5
//   V11 s0 q0  V12 s1 q1  V13 s2 q2  V14 (s0+s1)(q0+q1)  V15 (s1+s2)(q1+q2)  V16 (s0+s2)(q0+q2)
//   with s = a + b, q = (m0, m1 + m4, m2 + m5); split 5/4/4/4 over the waves.
LSG_DEVI void mf_mul_pair(uint32_t* lds, int w, int k) {
  {
    const fp2_t m0 = mf_get2(lds, MF_LC(2 * k, 0)), m1 = mf_get2(lds, MF_LC(2 * k, 1)), m2 = mf_get2(lds, MF_LC(2 * k, 2));
    if (w == 0) {
      const fp2_t a0 = mf_get2(lds, MF_FC(0)), a1 = mf_get2(lds, MF_FC(1)), a2 = mf_get2(lds, MF_FC(2));
      mf_put2(lds, MF_VC(0), fp2_mul(a0, m0));
      mf_put2(lds, MF_VC(1), fp2_mul(a1, m1));
      mf_put2(lds, MF_VC(2), fp2_mul(a2, m2));
      mf_put2(lds, MF_VC(3), fp2_mul(fp2_add(a0, a1), fp2_add(m0, m1)));
      mf_put2(lds, MF_VC(4), fp2_mul(fp2_add(a1, a2), fp2_add(m1, m2)));
    } else if (w == 1) {
      const fp2_t m4 = mf_get2(lds, MF_LC(2 * k + 1, 0)), m5 = mf_get2(lds, MF_LC(2 * k + 1, 1));
      const fp2_t b0 = mf_get2(lds, MF_FC(3)), b1 = mf_get2(lds, MF_FC(4));
      mf_put2(lds, MF_VC(5), fp2_mul(fp2_add(mf_get2(lds, MF_FC(0)), mf_get2(lds, MF_FC(2))), fp2_add(m0, m2)));
      mf_put2(lds, MF_VC(6), fp2_mul(b0, m4));
      mf_put2(lds, MF_VC(7), fp2_mul(b1, m5));
      mf_put2(lds, MF_VC(8), fp2_mul(fp2_add(b0, b1), fp2_add(m4, m5)));
    } else if (w == 2) {
      const fp2_t m4 = mf_get2(lds, MF_LC(2 * k + 1, 0)), m5 = mf_get2(lds, MF_LC(2 * k + 1, 1));
      const fp2_t b2 = mf_get2(lds, MF_FC(5));
      mf_put2(lds, MF_VC(9), fp2_mul(b2, m4));
      mf_put2(lds, MF_VC(10), fp2_mul(b2, m5));
      const fp2_t s0 = fp2_add(mf_get2(lds, MF_FC(0)), mf_get2(lds, MF_FC(3)));
      const fp2_t s1 = fp2_add(mf_get2(lds, MF_FC(1)), mf_get2(lds, MF_FC(4)));
      mf_put2(lds, MF_VC(11), fp2_mul(s0, m0));
      mf_put2(lds, MF_VC(12), fp2_mul(s1, fp2_add(m1, m4)));
    } else {
      const fp2_t m4 = mf_get2(lds, MF_LC(2 * k + 1, 0)), m5 = mf_get2(lds, MF_LC(2 * k + 1, 1));
      const fp2_t s0 = fp2_add(mf_get2(lds, MF_FC(0)), mf_get2(lds, MF_FC(3)));
      const fp2_t s1 = fp2_add(mf_get2(lds, MF_FC(1)), mf_get2(lds, MF_FC(4)));
      const fp2_t s2 = fp2_add(mf_get2(lds, MF_FC(2)), mf_get2(lds, MF_FC(5)));
      const fp2_t q1 = fp2_add(m1, m4), q2 = fp2_add(m2, m5);
      mf_put2(lds, MF_VC(13), fp2_mul(s2, q2));
      mf_put2(lds, MF_VC(14), fp2_mul(fp2_add(s0, s1), fp2_add(m0, q1)));
      mf_put2(lds, MF_VC(15), fp2_mul(fp2_add(s1, s2), fp2_add(q1, q2)));
      mf_put2(lds, MF_VC(16), fp2_mul(fp2_add(s0, s2), fp2_add(m0, q2)));
    }
  }
  __syncthreads();
  auto V = [&](int p) { return mf_get2(lds, MF_VC(p)); };
  // t0 = a M0, n = b (m4 + m5 v), t2 = s q (Karatsuba over Fp6, as in mf_sqr)
  auto t0c = [&](int j) {
    if (j == 0) return fp2_add(V(0), fp2_mul_xi(fp2_sub(fp2_sub(V(4), V(1)), V(2))));
    if (j == 1) return fp2_add(fp2_sub(fp2_sub(V(3), V(0)), V(1)), fp2_mul_xi(V(2)));
    return fp2_add(fp2_sub(fp2_sub(V(5), V(0)), V(2)), V(1));
  };
  auto t2c = [&](int j) {
    if (j == 0) return fp2_add(V(11), fp2_mul_xi(fp2_sub(fp2_sub(V(15), V(12)), V(13))));
    if (j == 1) return fp2_add(fp2_sub(fp2_sub(V(14), V(11)), V(12)), fp2_mul_xi(V(13)));
    return fp2_add(fp2_sub(fp2_sub(V(16), V(11)), V(13)), V(12));
  };
  auto nc = [&](int j) {
    if (j == 0) return fp2_add(V(6), fp2_mul_xi(V(10)));
    if (j == 1) return fp2_sub(fp2_sub(V(8), V(6)), V(7));
    return fp2_add(V(7), V(9));
  };
  // f'.c0 = t0 + v t1 = t0 + (xi n1, xi n2, n0);  f'.c1 = t2 - t0 - t1 = t2 - t0 - (xi n2, n0, n1)
  fp2_t o0, o1;
  int j0, j1 = -1;
  if (w == 0) {  // c0.0, c0.1
    o0 = fp2_add(t0c(0), fp2_mul_xi(nc(1)));
    o1 = fp2_add(t0c(1), fp2_mul_xi(nc(2)));
    j0 = 0;
    j1 = 1;
  } else if (w == 1) {  // c0.2, c1.0
    o0 = fp2_add(t0c(2), nc(0));
    o1 = fp2_sub(fp2_sub(t2c(0), t0c(0)), fp2_mul_xi(nc(2)));
    j0 = 2;
    j1 = 3;
  } else if (w == 2) {  // c1.1
    o0 = fp2_sub(fp2_sub(t2c(1), t0c(1)), nc(0));
    j0 = 4;
  } else {  // c1.2
    o0 = fp2_sub(fp2_sub(t2c(2), t0c(2)), nc(1));
    j0 = 5;
  }
  // f's coefficients are not read in this half: write them at once
  mf_put2(lds, MF_FC(j0), o0);
  if (j1 >= 0) mf_put2(lds, MF_FC(j1), o1);
  __syncthreads();
}

// L phase steps with their values staged through LDS: ml_dbl_step_raw / ml_add_step_raw +
// line_eval (lsg_pairing.hpp), the same formulas in the same order, but each line
// coefficient is evaluated at P and written to its slot as soon as it exists, and T's
// coordinates go back to their slots as soon as they are final.  Computed first and written
// last (the generic step), the line's three Fp2 values were live across the remaining point
// products and went to scratch (176 B per lane).
#ifndef LSG_MF_STAGED
#define LSG_MF_STAGED 1
#endif
LSG_DEVI void mf_put_line(uint32_t* lds, int wl, bool use, const fp2_t& l00, const fp2_t& l01P, const fp2_t& l11P) {
  mf_put2(lds, MF_LC(wl, 0), fp2_select(use, l00, fp2_one()));
  mf_put2(lds, MF_LC(wl, 1), fp2_select(use, l01P, fp2_zero()));
  mf_put2(lds, MF_LC(wl, 2), fp2_select(use, l11P, fp2_zero()));
}
LSG_DEVI void mf_dbl_line(uint32_t* lds, int wl, bool use, const uint32_t* __restrict__ P, size_t sl) {
  const int tb = MF_T + 6 * wl;
  fp2_t t0, t1, t2, v1;
  {
    const fp2_t X = mf_get2(lds, tb), Y = mf_get2(lds, tb + 2), Z = mf_get2(lds, tb + 4);
    t0 = fp2_sqr(Y);
    t1 = fp2_mul(Y, Z);
    t2 = fp2_mul_b3(fp2_sqr(Z));
    const fp2_t XX = fp2_sqr(X);
    v1 = fp2_mul(X, Y);
    const g1a_t Pk = lane_load<g1a_t>(P, sl);
    mf_put_line(lds, wl, use, fp2_sub(t2, t0), fp2_mul_fp(fp2_add(fp2_add(XX, XX), XX), Pk.x),
                fp2_mul_fp(fp2_neg(fp2_add(t1, t1)), Pk.y));
  }
  fp2_t Z3 = fp2_add(t0, t0);
  Z3 = fp2_add(Z3, Z3);
  Z3 = fp2_add(Z3, Z3);
  fp2_t X3 = fp2_mul(t2, Z3);
  fp2_t Y3 = fp2_add(t0, t2);
  mf_put2(lds, tb + 4, fp2_mul(t1, Z3));
  const fp2_t u2 = fp2_add(fp2_add(t2, t2), t2);
  const fp2_t s0 = fp2_sub(t0, u2);
  Y3 = fp2_mul(s0, Y3);
  mf_put2(lds, tb + 2, fp2_add(X3, Y3));
  X3 = fp2_mul(s0, v1);
  mf_put2(lds, tb, fp2_add(X3, X3));
}
LSG_DEVI void mf_add_line(uint32_t* lds, int wl, bool use, const uint32_t* __restrict__ P, const uint32_t* __restrict__ H,
                          size_t sl) {
  const int tb = MF_T + 6 * wl;
  fp2_t theta, delta;
  {
    const g2a_t Q = lane_load<g2a_t>(H, sl);
    const fp2_t Z = mf_get2(lds, tb + 4);
    theta = fp2_sub(mf_get2(lds, tb + 2), fp2_mul(Q.y, Z));
    delta = fp2_sub(mf_get2(lds, tb), fp2_mul(Q.x, Z));
    const fp2_t l00 = fp2_sub(fp2_mul(delta, Q.y), fp2_mul(theta, Q.x));
    const g1a_t Pk = lane_load<g1a_t>(P, sl);
    mf_put_line(lds, wl, use, l00, fp2_mul_fp(theta, Pk.x), fp2_mul_fp(fp2_neg(delta), Pk.y));
  }
  const fp2_t C = fp2_sqr(theta);
  const fp2_t D = fp2_sqr(delta);
  const fp2_t E = fp2_mul(D, delta);
  const fp2_t F = fp2_mul(mf_get2(lds, tb + 4), C);
  const fp2_t G = fp2_mul(mf_get2(lds, tb), D);
  const fp2_t Hs = fp2_sub(fp2_add(E, F), fp2_add(G, G));
  mf_put2(lds, tb, fp2_mul(delta, Hs));
  const fp2_t Y3 = fp2_sub(fp2_mul(theta, fp2_sub(G, Hs)), fp2_mul(E, mf_get2(lds, tb + 2)));
  mf_put2(lds, tb + 2, Y3);
  mf_put2(lds, tb + 4, fp2_mul(E, mf_get2(lds, tb + 4)));
}

// Issue priority of the fused kernel's waves (s_setprio; 0 = the default of every wave).  Its
// four waves meet at eight barriers per doubling while the per-set kernels of other packages
// share their SIMDs: ahead of those, a workgroup's slowest wave reaches each barrier sooner
// and the other waves fill the SIMD while it waits.  Firehose +0.9 % (8 of 8 pairs) and
// +1.7 % (5 rounds) on one MI355X, `profiles/r06_mf_prio_ab.txt`.  (A/B: -DLSG_MF_PRIO=0.)
#ifndef LSG_MF_PRIO
#define LSG_MF_PRIO 2
#endif
#ifndef LSG_MF_WAVES
#define LSG_MF_WAVES 2  // waves per SIMD the register budget is sized for (256 VGPR + AGPR)
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LSG_MF_WAVES)))
k_miller_fused(int n_items, const int32_t* __restrict__ item_first, const int32_t* __restrict__ item_cnt,
               const uint32_t* __restrict__ P, const uint8_t* __restrict__ pinf, const uint8_t* __restrict__ hinf,
               const int32_t* __restrict__ err, const uint32_t* __restrict__ H, uint32_t* __restrict__ f_out) {
  // dynamic LDS (MF_LDS_BYTES at launch): the compiler then sizes registers for
  // LSG_MF_WAVES waves per SIMD instead of the one workgroup per CU the LDS allows, so the
  // other kernels of the pipeline can share the SIMDs while this one waits at its barriers
  extern __shared__ uint32_t lds[];
#if LSG_MF_PRIO
  __builtin_amdgcn_s_setprio(LSG_MF_PRIO);
#endif
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform: an SGPR
  const size_t it = (size_t)blockIdx.x * MF_ITEMS + ((threadIdx.x & 63) >> 1);
  const bool live = it < (size_t)n_items;  // lanes past the end run item 0's data and store nothing
  const size_t itc = live ? it : 0;
  const int first = item_first[itc], cnt = item_cnt[itc];
  const int si = first + (w < cnt ? w : cnt - 1);
  // the lanes whose pair contributes, as a wave mask (SGPRs) rather than a live VGPR
  const uint64_t use_mask = __ballot(live && w < cnt && err[si] == 0 && !pinf[si] && !hinf[si]);
  // nothing stays in registers across the loop: T lives in LDS, Q (addition steps) and P are
  // re-read from global memory (L2 hits)
  {
    const g2p_t T = proj_from_aff(lane_load<g2a_t>(H, (size_t)si));
    mf_put2(lds, MF_T + 6 * w, T.X);
    mf_put2(lds, MF_T + 6 * w + 2, T.Y);
    mf_put2(lds, MF_T + 6 * w + 4, T.Z);
  }
  auto line_phase = [&](bool add) {
    // w and si re-materialised per phase: hoisted out of the loop, the wave-dependent LDS
    // slot addresses and point pointers were spilled to scratch and reloaded every step
    int wl = w, sl = si;
    asm volatile("" : "+s"(wl), "+v"(sl));
#if LSG_MF_STAGED
    const bool use = (use_mask >> __lane_id()) & 1u;
    if (add)
      mf_add_line(lds, wl, use, P, H, (size_t)sl);
    else
      mf_dbl_line(lds, wl, use, P, (size_t)sl);
#else
    g2p_t T;  // this wave's own slots: no other wave touches them
    T.X = mf_get2(lds, MF_T + 6 * wl);
    T.Y = mf_get2(lds, MF_T + 6 * wl + 2);
    T.Z = mf_get2(lds, MF_T + 6 * wl + 4);
    line_t L = add ? ml_add_step_raw(T, lane_load<g2a_t>(H, (size_t)sl)) : ml_dbl_step_raw(T);
    mf_put2(lds, MF_T + 6 * wl, T.X);
    mf_put2(lds, MF_T + 6 * wl + 2, T.Y);
    mf_put2(lds, MF_T + 6 * wl + 4, T.Z);
    const g1a_t Pk = lane_load<g1a_t>(P, (size_t)sl);
    L = line_eval(L, Pk.x, Pk.y);
    const bool use = (use_mask >> __lane_id()) & 1u;
    mf_put2(lds, MF_LC(wl, 0), fp2_select(use, L.l00, fp2_one()));
    mf_put2(lds, MF_LC(wl, 1), fp2_select(use, L.l01, fp2_zero()));
    mf_put2(lds, MF_LC(wl, 2), fp2_select(use, L.l11, fp2_zero()));
#endif
    __syncthreads();
    mf_pair_lines(lds, wl);
#pragma unroll 1
    for (int k = 0; k < 2; k++) mf_mul_pair(lds, wl, k);
  };
  // f = 1 (each wave writes a third of the coefficients' limbs: c0.c0 = 1, the rest 0)
  if (w < 2) {
    mf_put2(lds, MF_FC(3 * w), w == 0 ? fp2_one() : fp2_zero());
    mf_put2(lds, MF_FC(3 * w + 1), fp2_zero());
    mf_put2(lds, MF_FC(3 * w + 2), fp2_zero());
  }
  const uint64_t xa = ((uint64_t)LSG_X_ABS_HI << 32) | LSG_X_ABS_LO;
  line_phase(false);  // the first doubling
  line_phase(true);   // bit 62 of |x|
#pragma unroll 1
  for (int b = 61; b >= 0; b--) {
    mf_sqr(lds, w);
    line_phase(false);
    if ((xa >> b) & 1u) line_phase(true);
  }
  // f_item = conj(f): wave w stores Fp components 3w..3w+2 (components 6..11 negated)
  if (live) {
    uint32_t* o = f_out + it * (size_t)lsgl::W_F12 + pair_h();  // W_F12: words per item (both lanes)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const int c = 3 * w + j;
      fp_t v = mf_get(lds, MF_F + c);
      if (c >= 6) v = fp_neg(v);
#pragma unroll
      for (int k = 0; k < LSG_PL; k++) o[(7 * c + k) * LSG_GROUP] = v.l[k];
    }
  }
}

namespace lsgk {
hipError_t miller_fused(hipStream_t st, int n_items, const int32_t* item_first, const int32_t* item_cnt,
                        const uint32_t* P, const uint8_t* pinf, const uint8_t* hinf, const int32_t* err,
                        const uint32_t* H, uint32_t* f) {
  if (n_items <= 0) return hipSuccess;
  static const hipError_t attr = hipFuncSetAttribute((const void*)k_miller_fused,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)MF_LDS_BYTES);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(k_miller_fused, dim3((n_items + MF_ITEMS - 1) / MF_ITEMS), dim3(256), MF_LDS_BYTES, st, n_items, item_first,
                     item_cnt, P, pinf, hinf, err, H, f);
  return hipGetLastError();
}
hipError_t miller_lines_list(hipStream_t st, int n, const int32_t* list, const uint32_t* H, uint32_t* lines) {
  LSG_LAUNCH_ITEMS(k_miller_lines_list, n, st, n, list, H, lines);
}
hipError_t miller_accum_list(hipStream_t st, int n, const int32_t* list, const uint32_t* P, const uint8_t* pinf,
                             const uint8_t* hinf, const int32_t* err, const uint32_t* lines, uint32_t* f) {
  LSG_LAUNCH_ITEMS(k_miller_accum_list, n, st, n, list, P, pinf, hinf, err, lines, f);
}
hipError_t miller_lines(hipStream_t st, int n, const uint32_t* H, uint32_t* lines) {
  LSG_LAUNCH_ITEMS(k_miller_lines, n, st, n, H, lines);
}
hipError_t miller_accum(hipStream_t st, int K, int n_items, const int32_t* item_first, const int32_t* item_cnt,
                        const uint32_t* P, const uint8_t* pinf, const uint8_t* hinf, const int32_t* err, int n_sets,
                        const uint32_t* lines, uint32_t* f) {
  if (K == 1) LSG_LAUNCH_ITEMS(k_miller_accum<1>, n_items, st, n_items, item_first, item_cnt, P, pinf, hinf, err, n_sets, lines, f);
  if (K == 2) LSG_LAUNCH_ITEMS(k_miller_accum<2>, n_items, st, n_items, item_first, item_cnt, P, pinf, hinf, err, n_sets, lines, f);
  LSG_LAUNCH_ITEMS(k_miller_accum<4>, n_items, st, n_items, item_first, item_cnt, P, pinf, hinf, err, n_sets, lines, f);
}
}  // namespace lsgk
