// lsg_k_pk.hip -- public-key kernels: deserializeSet's PublicKey.fromBytes (multithread/
// worker.ts:108-114) and the resident pubkey table gather (8f(1)), batched
// KeyValidate (8f(2), block/processDeposit.ts:57-65), the RLC scaling [r_i] aggPK_i of blst
// mul_n_aggregate (8a M4) and G1 serialisation.
#include "lsg_kcommon.hpp"
namespace {
#include "lsg_inv.hpp"
}  // namespace

// Key `item` of a staged key list as an affine point: is_inf for the point at infinity and for
// a key that does not decode (err != 0).  A key given by index (len == LSG_PK_INDEX: the slot's
// first 4 bytes) is read from the resident table: affine rows, tab_ok 1 = a finite key, 2 = the
// infinity key, 0 = no key (lsg_pubkey_table_set; tab_n rows).
LSG_DEVI int pk_fetch_aff(size_t item, const uint8_t* __restrict__ pk, uint32_t stride, const uint32_t* __restrict__ pk_len,
                          const uint32_t* __restrict__ tab, const uint8_t* __restrict__ tab_ok, uint32_t tab_n,
                          g1a_t& a, bool& is_inf) {
  const uint32_t len = pk_len[item];
  is_inf = true;
  if (len == LSG_PK_INDEX) {
    const uint8_t* b = pk + (size_t)stride * item;
    const uint32_t idx = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    const uint8_t ok = idx < tab_n ? tab_ok[idx] : 0;
    a = lane_load<g1a_t>(tab, ok == 1 ? idx : 0);  // (row 0 for an infinite or missing key: unused)
    is_inf = ok != 1;
    return ok ? 0 : LSG_ERR_BAD_INDEX;
  }
  a.x = fp_zero();
  a.y = fp_zero();
  bool inf = false;
  const int e = (len == 48 || len == 96) ? g1_deserialize(a, inf, pk + (size_t)stride * item, (int)len) : LSG_BLST_INVALID_SIZE;
  is_inf = e != 0 || inf;
  return e;
}

// pubkey -> projective G1 (infinity and undecodable keys become (0:1:0))
__global__ void LSG_KERNEL_ATTR k_pk_decode(int n, const uint8_t* __restrict__ pk, uint32_t stride,
                                            const uint32_t* __restrict__ pk_len,
                                            uint32_t* __restrict__ pkp, int32_t* __restrict__ err,
                                            const uint32_t* __restrict__ tab, const uint8_t* __restrict__ tab_ok,
                                            uint32_t tab_n) {
  LANE_ITEM(n);
  g1a_t a;
  bool is_inf;
  const int e = pk_fetch_aff(item, pk, stride, pk_len, tab, tab_ok, tab_n, a, is_inf);
  lane_store(pkp, item, is_inf ? proj_inf<fp_t>() : proj_from_aff(a));
  if (lead) err[item] = e;
}

// pubkey -> affine G1 + infinity flag (the first level of the aggregation tree below; the
// table rows of lsg_pubkey_table_set)
__global__ void LSG_KERNEL_ATTR k_pk_gather_aff(int n, const uint8_t* __restrict__ pk, uint32_t stride,
                                                const uint32_t* __restrict__ pk_len, uint32_t* __restrict__ pts,
                                                uint8_t* __restrict__ inf, int32_t* __restrict__ err,
                                                const uint32_t* __restrict__ tab, const uint8_t* __restrict__ tab_ok,
                                                uint32_t tab_n) {
  LANE_ITEM(n);
  g1a_t a;
  bool is_inf;
  const int e = pk_fetch_aff(item, pk, stride, pk_len, tab, tab_ok, tab_n, a, is_inf);
  lane_store(pts, item, a);
  if (lead) {
    err[item] = e;
    inf[item] = is_inf ? 1 : 0;
  }
}

// ---- PublicKey.aggregate of the many keys of aggregate sets (utils.ts:11)
// as a pairwise tree of AFFINE additions with simultaneous inversion.  Level t holds every
// set's points (affine + infinity flag), segment s = one set; item q adds the pair (2p, 2p+1)
// of its segment (p = q - cum[s]; a lone last point is copied) into level t+1.  An affine
// addition is lambda = dy / dx, x3 = lambda^2 - x1 - x2, y3 = lambda (x1 - x3) - y1: three
// products plus one shared inversion, against twelve for a complete projective addition.  The
// inversions of a whole level are ONE inversion (Montgomery's trick): k_agg_fold multiplies
// each chunk of AGG_T items' denominators (prefix products kept), lsg_host.hip's batched
// inversion inverts the chunk products, k_agg_unfold walks each chunk back and adds.  Per
// addition ~6.3 products instead of 12.  Exceptional pairs (equal x: P + P or P - P) make
// their chunk's product zero, which the batched inversion returns as zero; such a chunk is
// redone in k_agg_unfold with doubling / infinity denominators and its own divstep inversion.
// Segments shorter than AGG_FINAL_MAX points skip the levels: k_agg_final sums each set's
// remaining points with complete mixed additions.
enum { AGG_ADD = 0, AGG_DBL = 1, AGG_INF = 2, AGG_COPY_A = 3, AGG_COPY_B = 4 };

// level plan (lsg_host.hip agg_plan): cum[0..n_seg] item prefix counts, then in_off, len,
// out_off per participating segment
struct AggLevel {
  const int32_t* cum;
  const int32_t* in_off;
  const int32_t* len;
  const int32_t* out_off;
  int n_seg;
};
LSG_DEVI AggLevel agg_level(const int32_t* plan, int n_seg) {
  AggLevel L;
  L.cum = plan;
  L.in_off = plan + n_seg + 1;
  L.len = L.in_off + n_seg;
  L.out_off = L.len + n_seg;
  L.n_seg = n_seg;
  return L;
}
// segment of item q: the last s with cum[s] <= q
LSG_DEVI int agg_seg(const AggLevel& L, int32_t q) {
  int lo = 0, hi = L.n_seg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L.cum[mid] <= q) lo = mid; else hi = mid - 1;
  }
  return lo;
}
// the pair of item q: input positions a (and b = a + 1 unless a is its segment's last point)
LSG_DEVI void agg_pair(const AggLevel& L, int s, int32_t q, int32_t& a, bool& has_b, int32_t& out) {
  const int32_t p = q - L.cum[s];
  a = L.in_off[s] + 2 * p;
  has_b = 2 * p + 1 < L.len[s];
  out = L.out_off[s] + p;
}
// the type of item q from the infinity flags alone (equal-x pairs are found by the inversion)
LSG_DEVI int agg_type(bool has_b, bool ia, bool ib) {
  if (!has_b || ib) return ia ? AGG_INF : AGG_COPY_A;
  return ia ? AGG_COPY_B : AGG_ADD;
}

__global__ void LSG_KERNEL_ATTR k_agg_fold(int n_items, int T, const int32_t* __restrict__ plan, int n_seg,
                                           const uint32_t* __restrict__ pts, const uint8_t* __restrict__ inf,
                                           uint32_t* __restrict__ pre, uint32_t* __restrict__ tot) {
  LANE_ITEM((n_items + T - 1) / T);
  (void)lead;
  const AggLevel L = agg_level(plan, n_seg);
  const int32_t first = (int32_t)item * T, last = min(n_items, first + T);
  int s = agg_seg(L, first);
  const fp_t one = fp_one();
  fp_t acc = one;
#pragma unroll 1
  for (int32_t q = first; q < last; q++) {
    while (L.cum[s + 1] <= q) s++;
    int32_t a, out;
    bool has_b;
    agg_pair(L, s, q, a, has_b, out);
    const int ty = agg_type(has_b, inf[a] != 0, has_b && inf[a + 1] != 0);
    fp_t den = one;
    if (ty == AGG_ADD) den = fp_sub(lane_load<fp_t>(pts, (size_t)(a + 1) * 2), lane_load<fp_t>(pts, (size_t)a * 2));
    acc = q == first ? den : fp_mul(acc, den);
    lane_store(pre, q, acc);
  }
  lane_store(tot, item, acc);
}

// the denominators of items first..last-1 with the equal-x pairs resolved (doubling: 2 y1;
// P - P: 1), their prefix products rewritten into pre, and the chunk inverse by divsteps
LSG_DEVI fp_t agg_chunk_redo(const AggLevel& L, int32_t first, int32_t last, const uint32_t* __restrict__ pts,
                             const uint8_t* __restrict__ inf, uint32_t* __restrict__ pre) {
  int s = agg_seg(L, first);
  const fp_t one = fp_one();
  fp_t acc = one;
#pragma unroll 1
  for (int32_t q = first; q < last; q++) {
    while (L.cum[s + 1] <= q) s++;
    int32_t a, out;
    bool has_b;
    agg_pair(L, s, q, a, has_b, out);
    const int ty = agg_type(has_b, inf[a] != 0, has_b && inf[a + 1] != 0);
    fp_t den = one;
    if (ty == AGG_ADD) {
      const g1a_t A = lane_load<g1a_t>(pts, a), B = lane_load<g1a_t>(pts, a + 1);
      den = fp_sub(B.x, A.x);
      if (fp_is_zero(den)) den = fp_eq(A.y, B.y) ? fp_add(A.y, A.y) : one;
    }
    acc = q == first ? den : fp_mul(acc, den);
    lane_store(pre, q, acc);
  }
  const fp_t d = pair_inv_gcd(pair_canon(acc));  // (acc R)^-1 as an integer
  return pair_mont_mul(d, fp_t(FP_RCUBE));        // acc^-1 R
}

__global__ void LSG_KERNEL_ATTR k_agg_unfold(int n_items, int T, const int32_t* __restrict__ plan, int n_seg,
                                             const uint32_t* __restrict__ pts, const uint8_t* __restrict__ inf,
                                             uint32_t* __restrict__ pre, const uint32_t* __restrict__ tinv,
                                             uint32_t* __restrict__ out_pts, uint8_t* __restrict__ out_inf) {
  LANE_ITEM((n_items + T - 1) / T);
  const AggLevel L = agg_level(plan, n_seg);
  const int32_t first = (int32_t)item * T, last = min(n_items, first + T);
  fp_t acc = lane_load<fp_t>(tinv, item);  // 1 / (product of the chunk's denominators)
  // a zero chunk inverse: an equal-x pair in the chunk (rare): resolve it and invert alone
  const bool redo = fp_is_zero(acc);
  if (redo) acc = agg_chunk_redo(L, first, last, pts, inf, pre);
  int s = agg_seg(L, last - 1);
  const fp_t one = fp_one();
#pragma unroll 1
  for (int32_t q = last - 1; q >= first; q--) {
    while (L.cum[s] > q) s--;
    int32_t a, o;
    bool has_b;
    agg_pair(L, s, q, a, has_b, o);
    const bool ia = inf[a] != 0, ib = has_b && inf[a + 1] != 0;
    int ty = agg_type(has_b, ia, ib);
    const g1a_t A = lane_load<g1a_t>(pts, a);
    g1a_t B = A;
    if (has_b) B = lane_load<g1a_t>(pts, a + 1);
    fp_t den = fp_sub(B.x, A.x), num = fp_sub(B.y, A.y);
    if (redo && ty == AGG_ADD && fp_is_zero(den)) {  // equal x: P + P or P + (-P)
      if (fp_is_zero(num)) {
        ty = AGG_DBL;
        den = fp_add(A.y, A.y);
        const fp_t x2 = fp_mul(A.x, A.x);
        num = fp_add(fp_add(x2, x2), x2);
      } else {
        ty = AGG_INF;
      }
    }
    if (ty != AGG_ADD && ty != AGG_DBL) den = one;
    const fp_t inv = q > first ? fp_mul(acc, lane_load<fp_t>(pre, q - 1)) : acc;
    if (q > first) acc = fp_mul(acc, den);
    const fp_t lam = fp_mul(num, inv);
    const fp_t x3 = fp_sub(fp_sub(fp_mul(lam, lam), A.x), B.x);
    g1a_t R;
    R.x = x3;
    R.y = fp_sub(fp_mul(lam, fp_sub(A.x, x3)), A.y);
    bool rinf = false;
    if (ty == AGG_COPY_A) R = A;
    if (ty == AGG_COPY_B) R = B;
    if (ty == AGG_INF) rinf = true;
    if (ty == AGG_COPY_A) rinf = ia;
    lane_store(out_pts, o, R);
    if (lead) out_inf[o] = rinf ? 1 : 0;
  }
}

// each set's remaining points (segment [off, off + len) of its last level) summed with
// complete mixed additions -> projective aggregate (the identity for none / all infinite)
__global__ void LSG_KERNEL_ATTR k_agg_final(int n_sets, const int32_t* __restrict__ src, const uint32_t* __restrict__ arena,
                                            const uint8_t* __restrict__ inf_arena, uint32_t* __restrict__ agg) {
  LANE_ITEM(n_sets);
  (void)lead;
  const int32_t base = src[3 * item], off = src[3 * item + 1], len = src[3 * item + 2];
  const uint32_t* pts = arena + (size_t)base * lsgl::W_G1A;
  const uint8_t* inf = inf_arena + base;
  g1p_t acc = proj_inf<fp_t>();
#pragma unroll 1
  for (int32_t k = 0; k < len; k++) {
    if (inf[off + k]) continue;
    const g1a_t a = lane_load<g1a_t>(pts, off + k);
    acc = proj_is_inf(acc) ? proj_from_aff(a) : g1_add_mixed(acc, a);
  }
  lane_store(agg, item, acc);
}

// KeyValidate: decode, reject infinity and points outside G1; pts receives the key as a
// projective point (the identity for rejected keys); keys sit in 96-byte slots
__global__ void LSG_KERNEL_ATTR k_pk_validate(int n, const uint8_t* __restrict__ pk, uint32_t len,
                                              uint32_t* __restrict__ pts, int32_t* __restrict__ err) {
  LANE_ITEM(n);
  g1a_t a;
  a.x = fp_zero();
  a.y = fp_zero();
  bool is_inf = false;
  int e = g1_deserialize(a, is_inf, pk + 96 * item, (int)len);
  if (e == 0 && is_inf) e = LSG_BLST_PK_IS_INFINITY;
  const g1p_t p = e == 0 ? proj_from_aff(a) : proj_inf<fp_t>();
  if (e == 0 && !g1_in_group(p)) e = LSG_BLST_POINT_NOT_IN_GROUP;
  lane_store(pts, item, e == 0 ? p : proj_inf<fp_t>());
  if (lead) err[item] = e;
}

// P_i = [r_i] agg_i, projective (r_i == 0: no scaling); zP_i = its Z (0 at infinity) for the
// batched inversion; pinf = aggregate is infinity
__global__ void LSG_KERNEL_ATTR k_pk_scale(int n, const uint32_t* __restrict__ agg, const uint64_t* __restrict__ rnd,
                                           uint32_t* __restrict__ Pp, uint32_t* __restrict__ zP,
                                           uint8_t* __restrict__ pinf) {
  LANE_ITEM(n);
  g1p_t acc = lane_load<g1p_t>(agg, item);
  uint64_t r = rnd[item];
  bool is_inf = proj_is_inf(acc);
  if (r != 0 && !is_inf) acc = proj_mul_u64_s3(acc, r);
  lane_store(Pp, item, acc);
  lane_store(zP, item, is_inf ? fp_zero() : acc.Z);
  if (lead) pinf[item] = is_inf ? 1 : 0;
}

// P_i affine = (X / Z, Y / Z) with 1/Z from the batched inversion
__global__ void LSG_KERNEL_ATTR k_pk_affine(int n, const uint32_t* __restrict__ Pp, const uint32_t* __restrict__ zinv,
                                            uint32_t* __restrict__ P) {
  LANE_ITEM(n);
  (void)lead;
  g1p_t p = lane_load<g1p_t>(Pp, item);
  fp_t zi = lane_load<fp_t>(zinv, item);
  g1a_t a;
  fp_mul2(a.x, a.y, p.X, zi, p.Y, zi);
  lane_store(P, item, a);
}

// One Miller pair per distinct message (lsg_host.hip msg_agg): the package group's scaled keys
// r_i pk_i, each masked to the identity when its set cannot contribute (the rule of the Miller
// kernels: a decode error or an infinite key), are summed per message by the segmented
// reduction; the sums go affine with one divstep inversion each (a few dozen messages).
__global__ void LSG_KERNEL_ATTR k_pk_mask(int n, const uint32_t* __restrict__ Pp, const int32_t* __restrict__ err,
                                          const uint8_t* __restrict__ pinf, uint32_t* __restrict__ out) {
  LANE_ITEM(n);
  (void)lead;
  g1p_t p = proj_inf<fp_t>();
  if (err[item] == 0 && !pinf[item]) p = lane_load<g1p_t>(Pp, item);
  lane_store(out, item, p);
}
__global__ void LSG_KERNEL_ATTR k_g1p_affine_inv(int n, const uint32_t* __restrict__ Pp, uint32_t* __restrict__ P,
                                                 uint8_t* __restrict__ pinf) {
  LANE_ITEM(n);
  const g1p_t p = lane_load<g1p_t>(Pp, item);
  const bool is_inf = proj_is_inf(p);
  const fp_t d = pair_inv_gcd(pair_canon(is_inf ? fp_one() : p.Z));  // (Z R)^-1 as an integer
  const fp_t zi = pair_mont_mul(d, fp_t(FP_RCUBE));                   // Z^-1 R
  g1a_t a;
  fp_mul2(a.x, a.y, p.X, zi, p.Y, zi);
  lane_store(P, item, a);
  if (lead) pinf[item] = is_inf ? 1 : 0;
}

__global__ void LSG_KERNEL_ATTR k_g1p_to_bytes(int n, const uint32_t* __restrict__ pts, uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  (void)lead;
  g1p_t p = lane_load<g1p_t>(pts, item);
  bool is_inf = proj_is_inf(p);
  g1a_t a;
  if (is_inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    a = proj_to_aff(p);
  }
  g1_serialize(out + 96 * item, a, is_inf);
}

// pk_i = [sk_i] G1, uncompressed 96 bytes (bench/test input generation; double-and-add)
__global__ void LSG_KERNEL_ATTR k_sk_to_pk(int n, const uint8_t* __restrict__ sks, uint8_t* __restrict__ out96) {
  LANE_ITEM(n);
  (void)lead;
  g1a_t g;
  g.x = fp_t(G1_GEN_X);
  g.y = fp_t(G1_GEN_Y);
  const g1p_t base = proj_from_aff(g);
  g1p_t acc = proj_inf<fp_t>();
  const uint8_t* k = sks + 32 * item;
  for (int byte = 0; byte < 32; byte++) {
    uint32_t v = k[byte];
    for (int b = 7; b >= 0; b--) {
      acc = g1_dbl(acc);
      g1p_t s = g1_add(acc, base);
      bool bit = (v >> b) & 1u;
      acc.X = fp_select(bit, s.X, acc.X);
      acc.Y = fp_select(bit, s.Y, acc.Y);
      acc.Z = fp_select(bit, s.Z, acc.Z);
    }
  }
  bool is_inf = proj_is_inf(acc);
  g1a_t a;
  if (is_inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    a = proj_to_aff(acc);
  }
  g1_serialize(out96 + 96 * item, a, is_inf);
}

namespace lsgk {
hipError_t pk_decode(hipStream_t st, int n, const uint8_t* pk, uint32_t stride, const uint32_t* pk_len, uint32_t* pts,
                     int32_t* err, const uint32_t* tab, const uint8_t* tab_ok, uint32_t tab_n) {
  LSG_LAUNCH_ITEMS(k_pk_decode, n, st, n, pk, stride, pk_len, pts, err, tab, tab_ok, tab_n);
}
hipError_t pk_gather_aff(hipStream_t st, int n, const uint8_t* pk, uint32_t stride, const uint32_t* pk_len, uint32_t* pts,
                         uint8_t* inf, int32_t* err, const uint32_t* tab, const uint8_t* tab_ok, uint32_t tab_n) {
  LSG_LAUNCH_ITEMS(k_pk_gather_aff, n, st, n, pk, stride, pk_len, pts, inf, err, tab, tab_ok, tab_n);
}
hipError_t agg_fold(hipStream_t st, int n_items, int T, const int32_t* plan, int n_seg, const uint32_t* pts,
                    const uint8_t* inf, uint32_t* pre, uint32_t* tot) {
  LSG_LAUNCH_ITEMS(k_agg_fold, (n_items + T - 1) / T, st, n_items, T, plan, n_seg, pts, inf, pre, tot);
}
hipError_t agg_unfold(hipStream_t st, int n_items, int T, const int32_t* plan, int n_seg, const uint32_t* pts,
                      const uint8_t* inf, uint32_t* pre, const uint32_t* tinv, uint32_t* out_pts, uint8_t* out_inf) {
  LSG_LAUNCH_ITEMS(k_agg_unfold, (n_items + T - 1) / T, st, n_items, T, plan, n_seg, pts, inf, pre, tinv, out_pts, out_inf);
}
hipError_t agg_final(hipStream_t st, int n_sets, const int32_t* src, const uint32_t* arena, const uint8_t* inf_arena,
                     uint32_t* agg) {
  LSG_LAUNCH_ITEMS(k_agg_final, n_sets, st, n_sets, src, arena, inf_arena, agg);
}
hipError_t pk_validate(hipStream_t st, int n, const uint8_t* pk, uint32_t len, uint32_t* pts, int32_t* err) {
  LSG_LAUNCH_ITEMS(k_pk_validate, n, st, n, pk, len, pts, err);
}
hipError_t pk_scale(hipStream_t st, int n, const uint32_t* agg, const uint64_t* rnd, uint32_t* Pp, uint32_t* zP,
                    uint8_t* pinf) {
  LSG_LAUNCH_ITEMS(k_pk_scale, n, st, n, agg, rnd, Pp, zP, pinf);
}
hipError_t pk_affine(hipStream_t st, int n, const uint32_t* Pp, const uint32_t* zinv, uint32_t* P) {
  LSG_LAUNCH_ITEMS(k_pk_affine, n, st, n, Pp, zinv, P);
}
hipError_t pk_mask(hipStream_t st, int n, const uint32_t* Pp, const int32_t* err, const uint8_t* pinf, uint32_t* out) {
  LSG_LAUNCH_ITEMS(k_pk_mask, n, st, n, Pp, err, pinf, out);
}
hipError_t g1p_affine_inv(hipStream_t st, int n, const uint32_t* Pp, uint32_t* P, uint8_t* pinf) {
  LSG_LAUNCH_ITEMS(k_g1p_affine_inv, n, st, n, Pp, P, pinf);
}
hipError_t g1p_to_bytes(hipStream_t st, int n, const uint32_t* pts, uint8_t* out96) {
  LSG_LAUNCH_ITEMS(k_g1p_to_bytes, n, st, n, pts, out96);
}
hipError_t sk_to_pk(hipStream_t st, int n, const uint8_t* sks, uint8_t* out96) {
  LSG_LAUNCH_ITEMS(k_sk_to_pk, n, st, n, sks, out96);
}
}  // namespace lsgk
