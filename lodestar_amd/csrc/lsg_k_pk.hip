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
    // one 128-byte row per key (row 0 for an infinite or missing key: unused)
    a = lane_load<g1a_t>(tab + (size_t)(ok == 1 ? idx : 0) * lsgl::W_TAB, 0);
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

// PublicKey.aggregate of many sets' keys straight from the staged keys (utils.ts:11; SURVEY.md
// 8a M1): one pass of the segmented reduction (lsg_k_reduce.hip k_seg_reduce, plan_seg) whose
// elements are fetched as affine points (table row or decoded bytes) and folded with complete
// mixed additions -- no projective copy of every key written and read back -- then the
// chunk's lane pairs combined by a butterfly.  Chunk = (first key, count, output: >= 0 into
// dst, < 0 into tmp for a second pass).
__global__ void LSG_KERNEL_ATTR k_pk_agg_seg(int n_chunks, int ips_log2, const int32_t* __restrict__ chunks,
                                             const uint8_t* __restrict__ pk, uint32_t stride,
                                             const uint32_t* __restrict__ pk_len, int32_t* __restrict__ err,
                                             const uint32_t* __restrict__ tab, const uint8_t* __restrict__ tab_ok,
                                             uint32_t tab_n, uint32_t* __restrict__ dst, uint32_t* __restrict__ tmp) {
  lsg_lane_setup();
  const size_t item = gtid() / LSG_GROUP;
  const bool lead = (threadIdx.x % LSG_GROUP) == 0;
  const size_t c = item >> ips_log2;
  const int ips = 1 << ips_log2, j = (int)(item & (size_t)(ips - 1));
  const bool active = c < (size_t)n_chunks;
  g1p_t acc = proj_inf<fp_t>();
  int out = 0;
  if (active) {
    const int off = chunks[3 * c], len = chunks[3 * c + 1];
    out = chunks[3 * c + 2];
    // software-pipelined: the next key's row is in flight while this one is added (the
    // gathers are scattered over the table; unhidden, their latency bounds the fold)
    g1a_t a;
    bool is_inf = true;
    int e = 0;
    if (j < len) e = pk_fetch_aff((size_t)(off + j), pk, stride, pk_len, tab, tab_ok, tab_n, a, is_inf);
#pragma unroll 1
    for (int k = j; k < len; k += ips) {
      const g1a_t cur = a;
      const bool cur_inf = is_inf;
      if (lead) err[off + k] = e;
      if (k + ips < len) e = pk_fetch_aff((size_t)(off + k + ips), pk, stride, pk_len, tab, tab_ok, tab_n, a, is_inf);
      if (!cur_inf) acc = proj_is_inf(acc) ? proj_from_aff(cur) : g1_add_mixed(acc, cur);
    }
  }
  // every lane runs the butterfly: a chunk never straddles a wave (ips <= 32 pairs)
#pragma unroll 1
  for (int o = ips >> 1; o >= 1; o >>= 1) acc = g1_add(acc, shfl_xor_t(acc, LSG_GROUP * o));
  if (active && j == 0) {
    if (out >= 0)
      lane_store(dst, (size_t)out, acc);
    else
      lane_store(tmp, (size_t)(-out - 1), acc);
  }
}

// pubkey -> affine G1 + infinity flag: the rows (lsgl::W_TAB words each) of lsg_pubkey_table_set
__global__ void LSG_KERNEL_ATTR k_pk_gather_aff(int n, const uint8_t* __restrict__ pk, uint32_t stride,
                                                const uint32_t* __restrict__ pk_len, uint32_t* __restrict__ pts,
                                                uint8_t* __restrict__ inf, int32_t* __restrict__ err,
                                                const uint32_t* __restrict__ tab, const uint8_t* __restrict__ tab_ok,
                                                uint32_t tab_n) {
  LANE_ITEM(n);
  g1a_t a;
  bool is_inf;
  const int e = pk_fetch_aff(item, pk, stride, pk_len, tab, tab_ok, tab_n, a, is_inf);
  lane_store(pts + item * lsgl::W_TAB, 0, a);
  if (lead) {
    err[item] = e;
    inf[item] = is_inf ? 1 : 0;
  }
}

// ---- PublicKey.aggregate of the keys of large packages (utils.ts:11) as a
// pairwise tree of AFFINE additions with simultaneous inversion.  An affine addition is
// lambda = dy / dx, x3 = lambda^2 - x1 - x2, y3 = lambda (x1 - x3) - y1: three products plus
// a share of one inversion, against eleven for a complete mixed addition.
//
// Layout (lsg_launch.h AggTreeArgs): level 0 holds each tree set's keys at an offset aligned
// to 2^L, padded with infinity; level t + 1 point q = level t points 2q + 2q + 1, so no pair
// ever straddles two sets and no segment lookup is needed above level 0.  Lane pair c owns
// the items q = c + j n_c(t), j < T: consecutive lane pairs touch consecutive points.
//
// The inversions of a level are one inversion per block (Montgomery's trick in two tiers):
// each lane pair folds its T denominators (prefix products kept), the block multiplies its
// chunk products in an LDS heap, inverts the root with one divstep inversion and runs the heap
// back down, leaving every chunk's inverse (cinv).  k_agg_step(t) walks each chunk back adding
// its pairs and -- fused -- folds level t + 1's denominators: the pair partner of output q is
// output q ^ 1, held by the adjacent lane pair at the same step (a lane shuffle); its block
// then inverts them the same way.  One launch per level, no global reduction between levels.
// Equal x (P + P or P - P) gives a zero denominator, which zeroes its chunk product: the fold
// tests each chunk product once and redoes such a chunk with the pairs resolved (doubling
// denominator 2y, or 1 for P - P), flagging it so that the step resolves its pairs again.
enum { AGG_ADD = 0, AGG_DBL = 1, AGG_INF = 2, AGG_COPY_A = 3, AGG_COPY_B = 4 };

LSG_DEVI int64_t agg_base(const lsgk::AggTreeArgs& a, int t) { return t == 0 ? 0 : 2 * a.N0 - (a.N0 >> (t - 1)); }

// the addition type of (A, B) with its denominator and numerator; exact: equal x resolved,
// else such a pair gives den == 0 (found by the chunk test)
LSG_DEVI int agg_den(const g1a_t& A, bool ia, const g1a_t& B, bool ib, bool exact, fp_t& den, fp_t& num) {
  den = fp_one();
  num = den;
  if (ia) return ib ? AGG_INF : AGG_COPY_B;
  if (ib) return AGG_COPY_A;
  den = fp_sub(B.x, A.x);
  num = fp_sub(B.y, A.y);
  if (exact && fp_is_zero(den)) {
    if (fp_is_zero(num)) {
      den = fp_add(A.y, A.y);
      const fp_t x2 = fp_mul(A.x, A.x);
      num = fp_add(fp_add(x2, x2), x2);
      return AGG_DBL;
    }
    den = fp_one();
    return AGG_INF;
  }
  return AGG_ADD;
}

// level-0 point p: key p - o of its set, or infinity in the padding
LSG_DEVI void agg_fetch0(const lsgk::AggTreeArgs& a, int64_t p, g1a_t& P, bool& pinf, bool lead) {
  const int s = a.blk_set[p >> a.L];
  const int64_t k = p - a.set_o0[s];
  pinf = true;
  P.x = fp_zero();
  P.y = P.x;
  if (k < a.set_len[s]) {
    const size_t key = (size_t)a.set_pk0[s] + (size_t)k;
    const int e = pk_fetch_aff(key, a.pk, a.stride, a.pk_len, a.tab, a.tab_ok, a.tab_n, P, pinf);
    if (lead) a.pk_err[key] = e;
  }
}

// a chunk's fold again with its equal-x pairs resolved (the points are in memory): prefix
// products rewritten, the chunk product returned.  asc: the level's fold order is j = 0..T-1.
LSG_DEVI fp_t agg_redo(const uint32_t* __restrict__ pts, const uint8_t* __restrict__ inf, uint32_t* __restrict__ pre,
                       int64_t c, int64_t nc, int64_t n_items, int T, bool asc) {
  fp_t acc = fp_one();
#pragma unroll 1
  for (int k = 0; k < T; k++) {
    const int64_t q = c + (int64_t)(asc ? k : T - 1 - k) * nc;
    fp_t den = fp_one(), num;
    if (q < n_items)
      agg_den(lane_load<g1a_t>(pts, 2 * q), inf[2 * q] != 0, lane_load<g1a_t>(pts, 2 * q + 1), inf[2 * q + 1] != 0,
              true, den, num);
    acc = k == 0 ? den : fp_mul(acc, den);
    lane_store(pre, q, acc);
  }
  return acc;
}

// level 0: gather each item's two keys, fold the chunk, invert the block's chunk products
__global__ void LSG_KERNEL_ATTR k_agg_leaf(lsgk::AggTreeArgs a) {
  __shared__ uint32_t H[2 * LSG_ITEMS_PER_BLOCK * lsgl::W_FP], I[2 * LSG_ITEMS_PER_BLOCK * lsgl::W_FP];
  lsg_lane_setup();
  const int l = (int)(threadIdx.x / LSG_GROUP);
  const bool lead = (threadIdx.x % LSG_GROUP) == 0;
  const int64_t c = (int64_t)blockIdx.x * LSG_ITEMS_PER_BLOCK + l, nc = a.n_c0, n_items = a.N0 >> 1;
  fp_t acc = fp_one();
#pragma unroll 1
  for (int j = 0; j < a.T; j++) {
    const int64_t q = c + (int64_t)j * nc;
    fp_t den = fp_one(), num;
    if (q < n_items) {
      g1a_t A, B;
      bool ia, ib;
      agg_fetch0(a, 2 * q, A, ia, lead);
      agg_fetch0(a, 2 * q + 1, B, ib, lead);
      lane_store(a.pts, 2 * q, A);
      lane_store(a.pts, 2 * q + 1, B);
      if (lead) {
        a.inf[2 * q] = ia ? 1 : 0;
        a.inf[2 * q + 1] = ib ? 1 : 0;
      }
      agg_den(A, ia, B, ib, false, den, num);
    }
    acc = j == 0 ? den : fp_mul(acc, den);
    lane_store(a.pre[0], q, acc);
  }
  const bool redo = fp_is_zero(acc);  // an equal-x pair (rare)
  if (redo) acc = agg_redo(a.pts, a.inf, a.pre[0], c, nc, n_items, a.T, true);
  if (lead) a.flag[0][c] = redo ? 1 : 0;
  lane_store(a.cinv[0], c, block_inv<LSG_ITEMS_PER_BLOCK>(H, I, l, acc));
}

// level t: chunks walked back (each pair added into level t + 1), level t + 1's denominators
// folded on the way (even lane pairs: its item q / 2 = outputs q, q + 1) and inverted
__global__ void LSG_KERNEL_ATTR k_agg_step(lsgk::AggTreeArgs a, int t) {
  constexpr int G = LSG_ITEMS_PER_BLOCK / 2;
  __shared__ uint32_t H[2 * G * lsgl::W_FP], I[2 * G * lsgl::W_FP];
  lsg_lane_setup();
  const int l = (int)(threadIdx.x / LSG_GROUP);
  const bool lead = (threadIdx.x % LSG_GROUP) == 0;
  const int64_t nc = a.n_c0 >> t, c = (int64_t)blockIdx.x * LSG_ITEMS_PER_BLOCK + l, n_items = a.N0 >> (t + 1);
  const int T = a.T;
  fp_t acc = lane_load<fp_t>(a.cinv[t & 1], c);  // 1 / (this chunk's product)

  const bool asc = (t & 1) == 0;  // level t's fold order: j ascending for even t
  const bool exact = a.flag[t & 1][c] != 0;
  const bool next = t + 1 < a.L, even = (l & 1) == 0;
  const uint32_t* pin = a.pts + lsgl::W_G1A * agg_base(a, t);
  const uint8_t* iin = a.inf + agg_base(a, t);
  uint32_t* pout = a.pts + lsgl::W_G1A * agg_base(a, t + 1);
  uint8_t* iout = a.inf + agg_base(a, t + 1);
  const uint32_t* pre = a.pre[t & 1];
  uint32_t* pre2 = a.pre[(t + 1) & 1];
  fp_t acc2 = fp_one();
#pragma unroll 1
  for (int k = T - 1; k >= 0; k--) {
    const int64_t q = c + (int64_t)(asc ? k : T - 1 - k) * nc;
    g1a_t A, B;
    bool ia = true, ib = true;
    fp_t den = fp_one(), num = den;
    int ty = AGG_INF;
    if (q < n_items) {
      A = lane_load<g1a_t>(pin, 2 * q);
      B = lane_load<g1a_t>(pin, 2 * q + 1);
      ia = iin[2 * q] != 0;
      ib = iin[2 * q + 1] != 0;
      ty = agg_den(A, ia, B, ib, exact, den, num);
    } else {
      A.x = fp_zero();
      A.y = A.x;
      B = A;
    }
    fp_t inv = acc;
    if (k > 0) {
      inv = fp_mul(acc, lane_load<fp_t>(pre, c + (int64_t)(asc ? k - 1 : T - k) * nc));
      acc = fp_mul(acc, den);
    }
    const fp_t lam = fp_mul(num, inv);
    g1a_t R;
    R.x = fp_sub(fp_sub(fp_mul(lam, lam), A.x), B.x);
    R.y = fp_sub(fp_mul(lam, fp_sub(A.x, R.x)), A.y);
    bool rinf = ty == AGG_INF;
    if (ty == AGG_COPY_A) R = A;
    if (ty == AGG_COPY_B) R = B;
    if (q < n_items) {
      lane_store(pout, q, R);
      if (lead) iout[q] = rinf ? 1 : 0;
    }
    if (next) {  // level t + 1 item q / 2 (even lane pairs): (R, the partner's output q + 1)
      const g1a_t Rp = shfl_xor_t(R, LSG_GROUP);
      const bool rpinf = __shfl_xor(rinf ? 1 : 0, LSG_GROUP, 64) != 0;
      fp_t den2, num2;
      agg_den(R, rinf, Rp, rpinf, false, den2, num2);
      acc2 = k == T - 1 ? den2 : fp_mul(acc2, den2);
      if (even) lane_store(pre2, q >> 1, acc2);
    }
  }
  if (!next) return;  // (uniform: no barrier follows)
  __threadfence_block();  // level t + 1's points, for a redo by the even lane pair
  const int64_t c2 = c >> 1, nc2 = nc >> 1, n2 = n_items >> 1;
  const bool redo = even && fp_is_zero(acc2);
  if (redo) acc2 = agg_redo(pout, iout, pre2, c2, nc2, n2, T, !asc);
  if (even && lead) a.flag[(t + 1) & 1][c2] = redo ? 1 : 0;
  const fp_t inv2 = block_inv<G>(H, I, even ? l / 2 : -1, acc2);
  if (even) lane_store(a.cinv[(t + 1) & 1], c2, inv2);
}

// each set's points summed with complete mixed additions -> projective aggregate (the
// identity for none / all infinite): (0, off, n) level-L points, (1, key, n) staged keys
__global__ void LSG_KERNEL_ATTR k_agg_final(lsgk::AggTreeArgs a, int n_sets, const int32_t* __restrict__ src,
                                            uint32_t* __restrict__ agg) {
  LANE_ITEM(n_sets);
  const int32_t mode = src[3 * item], off = src[3 * item + 1], len = src[3 * item + 2];
  g1p_t acc = proj_inf<fp_t>();
  if (mode == 0) {
    const uint32_t* pts = a.pts + lsgl::W_G1A * agg_base(a, a.L);
    const uint8_t* inf = a.inf + agg_base(a, a.L);
#pragma unroll 1
    for (int32_t k = 0; k < len; k++) {
      if (inf[off + k]) continue;
      const g1a_t p = lane_load<g1a_t>(pts, off + k);
      acc = proj_is_inf(acc) ? proj_from_aff(p) : g1_add_mixed(acc, p);
    }
  } else {
#pragma unroll 1
    for (int32_t k = 0; k < len; k++) {
      g1a_t p;
      bool pinf;
      const int e = pk_fetch_aff((size_t)off + k, a.pk, a.stride, a.pk_len, a.tab, a.tab_ok, a.tab_n, p, pinf);
      if (lead) a.pk_err[off + k] = e;
      if (pinf) continue;
      acc = proj_is_inf(acc) ? proj_from_aff(p) : g1_add_mixed(acc, p);
    }
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
hipError_t pk_agg_seg(hipStream_t st, int n_chunks, int ips_log2, const int32_t* chunks, const uint8_t* pk, uint32_t stride,
                      const uint32_t* pk_len, int32_t* err, const uint32_t* tab, const uint8_t* tab_ok, uint32_t tab_n,
                      uint32_t* dst, uint32_t* tmp) {
  LSG_LAUNCH_ITEMS(k_pk_agg_seg, (size_t)n_chunks << ips_log2, st, n_chunks, ips_log2, chunks, pk, stride, pk_len, err,
                   tab, tab_ok, tab_n, dst, tmp);
}
hipError_t agg_leaf(hipStream_t st, const AggTreeArgs& a) {
  if (a.L <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_agg_leaf, dim3((unsigned)(a.n_c0 / LSG_ITEMS_PER_BLOCK)), dim3(LSG_TPB), 0, st, a);
  return hipGetLastError();
}
hipError_t agg_step(hipStream_t st, const AggTreeArgs& a, int t) {
  hipLaunchKernelGGL(k_agg_step, dim3((unsigned)((a.n_c0 >> t) / LSG_ITEMS_PER_BLOCK)), dim3(LSG_TPB), 0, st, a, t);
  return hipGetLastError();
}
hipError_t agg_final(hipStream_t st, const AggTreeArgs& a, int n_sets, const int32_t* src, uint32_t* agg) {
  LSG_LAUNCH_ITEMS(k_agg_final, n_sets, st, a, n_sets, src, agg);
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
