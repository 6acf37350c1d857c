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

namespace lsgk {
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
