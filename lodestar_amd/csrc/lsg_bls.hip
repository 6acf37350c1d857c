// lsg_bls.hip -- gfx950 kernels and the C ABI (include/lodestar_bls.h) of the MI355X
// BLS12-381 signature-set verifier.
//
// Reference path replaced (file:line under /root/reference):
//   packages/beacon-node/src/chain/bls/multithread/worker.ts:30-114  (verifyManySignatureSets,
//       deserializeSet: batch-of-jobs verification with the per-job retry fallback)
//   packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39         (RLC batch vs single verify)
//   packages/beacon-node/src/chain/bls/utils.ts:5-26               (pubkey aggregation)
//   + the un-vendored @chainsafe/blst@0.2.8 arithmetic underneath.
//
// Execution model: every field element is limb-parallel over a 16-lane DPP row
// (lsg_fp_lane.hpp), so one work item (a set, a pubkey, a group) is one row and a wave64
// carries four items.  Per work package:
//   k_expand_msg      expand_message_xmd (SHA-256), one thread per set          [M3]
//   k_sig_decode      96/192-byte signature -> affine G2                         [M2]
//   k_sig_subgroup    psi(P) == [x]P                                             [M2]
//   k_pk_decode       48/96-byte pubkey -> projective G1 (on-curve only)         [H8]
//   tree(G1 add)      per-set pubkey aggregation, pairwise over levels           [M1]
//   k_pk_scale        P_i = [r_i] agg_i (affine)                                 [M4]
//   k_hash_map        SSWU x2 -> 3-isogeny -> add -> clear_cofactor -> affine     [M3]
//   k_sig_scale       [r_i] sig_i                                                [M4]
//   k_miller_sets     f_i = ML(P_i, H(m_i))                                      [M5]
// then per group (an RLC batch = a chunk of batchable jobs, or one job):
//   tree(G2 add)      S_g = sum [r_i] sig_i
//   k_miller_groups   f_g = ML(-G1, S_g)
//   tree(Fp12 mul)    F_g = f_g prod f_i
//   k_final_exp_check FE(F_g) == 1                                               [M6]
// Per-set values stay resident between the batch attempt and the per-job retry.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/lodestar_bls.h"
#include "lsg_fp_lane.hpp"
#include "lsg_h2c.hpp"
#include "lsg_pairing.hpp"

#define LSG_TPB 256          // threads per block (16 lane-items)
#define LSG_ITEMS_PER_BLOCK 16

static __device__ __forceinline__ size_t gtid() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }
#define LANE_ITEM(n)                        \
  lsg_lane_setup();                         \
  const size_t item = gtid() >> 4;          \
  if (item >= (size_t)(n)) return;          \
  const bool lead = (threadIdx.x & 15) == 0

// ---------------------------------------------------------------------------- kernels
// expand_message_xmd(msg_i, DST, 256): one thread per set (byte-serial SHA-256)
__global__ void __launch_bounds__(64) k_expand_msg(int n, const uint8_t* __restrict__ msg,
                                                    const uint32_t* __restrict__ msg_off,
                                                    const uint32_t* __restrict__ msg_len,
                                                    const uint8_t* __restrict__ dst, uint32_t dst_len,
                                                    uint8_t* __restrict__ ub) {
  size_t i = gtid();
  if (i >= (size_t)n) return;
  uint8_t out[256];
  expand_message_xmd_256(out, msg + msg_off[i], msg_len[i], dst, dst_len);
  uint32_t* o = (uint32_t*)(ub + 256 * i);
  for (int k = 0; k < 64; k++) {
    uint32_t w;
    __builtin_memcpy(&w, out + 4 * k, 4);
    o[k] = w;
  }
}

__global__ void __launch_bounds__(LSG_TPB) k_sig_decode(int n, const uint8_t* __restrict__ sig,
                                                         const uint32_t* __restrict__ sig_len,
                                                         uint32_t* __restrict__ sig_aff, uint8_t* __restrict__ inf,
                                                         int32_t* __restrict__ err) {
  LANE_ITEM(n);
  uint32_t len = sig_len[item];
  g2a_t p;
  p.x = fp2_zero();
  p.y = fp2_zero();
  bool is_inf = false;
  int e;
  if (len == 96)
    e = g2_uncompress(p, is_inf, sig + 192 * item);
  else if (len == 192)
    e = g2_deserialize_uncompressed(p, is_inf, sig + 192 * item);
  else
    e = LSG_BLST_INVALID_SIZE;
  lane_store(sig_aff, item, p);
  if (lead) {
    inf[item] = is_inf ? 1 : 0;
    err[item] = e;
  }
}

__global__ void __launch_bounds__(LSG_TPB) k_sig_subgroup(int n, const uint32_t* __restrict__ sig_aff,
                                                           const uint8_t* __restrict__ inf, int32_t* __restrict__ err) {
  LANE_ITEM(n);
  if (err[item] != 0 || inf[item]) return;
  bool ok = g2_in_group(proj_from_aff(lane_load<g2a_t>(sig_aff, item)));
  if (lead && !ok) err[item] = LSG_BLST_POINT_NOT_IN_GROUP;
}

// pubkey -> projective G1 (infinity and undecodable keys become (0:1:0))
__global__ void __launch_bounds__(LSG_TPB) k_pk_decode(int n, const uint8_t* __restrict__ pk,
                                                        const uint32_t* __restrict__ pk_len, uint32_t* __restrict__ pkp,
                                                        int32_t* __restrict__ err) {
  LANE_ITEM(n);
  uint32_t len = pk_len[item];
  g1a_t a;
  a.x = fp_zero();
  a.y = fp_zero();
  bool is_inf = false;
  int e = (len == 48 || len == 96) ? g1_deserialize(a, is_inf, pk + 96 * item, (int)len) : LSG_BLST_INVALID_SIZE;
  g1p_t p = (e == 0 && !is_inf) ? proj_from_aff(a) : proj_inf<fp_t>();
  lane_store(pkp, item, p);
  if (lead) err[item] = e;
}

// P_i = [r_i] agg_i in affine (r_i == 0: no scaling); pinf = aggregate is infinity
__global__ void __launch_bounds__(LSG_TPB) k_pk_scale(int n, const uint32_t* __restrict__ agg,
                                                       const uint64_t* __restrict__ rnd, uint32_t* __restrict__ P,
                                                       uint8_t* __restrict__ pinf) {
  LANE_ITEM(n);
  g1p_t acc = lane_load<g1p_t>(agg, item);
  uint64_t r = rnd[item];
  bool is_inf = proj_is_inf(acc);
  if (r != 0 && !is_inf) acc = proj_mul_u64(acc, r);
  g1a_t a;
  if (is_inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    a = proj_to_aff(acc);
  }
  lane_store(P, item, a);
  if (lead) pinf[item] = is_inf ? 1 : 0;
}

__global__ void __launch_bounds__(LSG_TPB) k_hash_map(int n, const uint8_t* __restrict__ ub, uint32_t* __restrict__ H,
                                                       uint8_t* __restrict__ hinf) {
  LANE_ITEM(n);
  const uint8_t* b = ub + 256 * item;
  fp2_t u0 = fp2_make(fp_from_be64_mod(b), fp_from_be64_mod(b + 64));
  fp2_t u1 = fp2_make(fp_from_be64_mod(b + 128), fp_from_be64_mod(b + 192));
  g2p_t q = g2_add(iso_map3(map_to_curve_sswu(u0)), iso_map3(map_to_curve_sswu(u1)));
  q = clear_cofactor_g2(q);
  bool is_inf = proj_is_inf(q);
  g2a_t a;
  if (is_inf) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    a = proj_to_aff(q);
  }
  lane_store(H, item, a);
  if (lead) hinf[item] = is_inf ? 1 : 0;
}

__global__ void __launch_bounds__(LSG_TPB) k_sig_scale(int n, const uint32_t* __restrict__ sig_aff,
                                                        const uint8_t* __restrict__ inf, const int32_t* __restrict__ err,
                                                        const uint64_t* __restrict__ rnd, uint32_t* __restrict__ rs) {
  LANE_ITEM(n);
  g2p_t r = proj_inf<fp2_t>();
  if (err[item] == 0 && !inf[item]) r = proj_mul_u64(proj_from_aff(lane_load<g2a_t>(sig_aff, item)), rnd[item]);
  lane_store(rs, item, r);
}

__global__ void __launch_bounds__(LSG_TPB) k_miller_sets(int n, const uint32_t* __restrict__ P,
                                                          const uint8_t* __restrict__ pinf, const uint32_t* __restrict__ H,
                                                          const uint8_t* __restrict__ hinf,
                                                          const int32_t* __restrict__ err, uint32_t* __restrict__ f) {
  LANE_ITEM(n);
  fp12_t r = fp12_one();
  if (err[item] == 0 && !pinf[item] && !hinf[item])
    r = miller_loop(lane_load<g1a_t>(P, item), lane_load<g2a_t>(H, item));
  lane_store(f, item, r);
}

// f_g = ML(-G1, S_g) = conj(ML(G1, S_g)) written at slot n_sets + g
__global__ void __launch_bounds__(LSG_TPB) k_miller_groups(int ng, const uint32_t* __restrict__ S, size_t slot0,
                                                            uint32_t* __restrict__ f) {
  LANE_ITEM(ng);
  g2p_t s = lane_load<g2p_t>(S, item);
  fp12_t r = fp12_one();
  if (!proj_is_inf(s)) {
    g1a_t ng1;
    ng1.x = fp_t(G1_GEN_X);
    ng1.y = fp_t(G1_GEN_NEG_Y);
    r = miller_loop(ng1, proj_to_aff(s));
  }
  lane_store(f, slot0 + item, r);
}

// one level of a segmented pairwise reduction: dst[k] = src[ia[k]] (+) src[ib[k]]  (ib < 0: copy)
template <int OP>
__global__ void __launch_bounds__(LSG_TPB) k_tree_level(int n, const int32_t* __restrict__ ia,
                                                         const int32_t* __restrict__ ib, const uint32_t* __restrict__ src,
                                                         uint32_t* __restrict__ dst) {
  LANE_ITEM(n);
  int32_t a = ia[item], b = ib[item];
  if (OP == 0) {
    g1p_t x = lane_load<g1p_t>(src, a);
    if (b >= 0) x = g1_add(x, lane_load<g1p_t>(src, b));
    lane_store(dst, item, x);
  } else if (OP == 1) {
    g2p_t x = lane_load<g2p_t>(src, a);
    if (b >= 0) x = g2_add(x, lane_load<g2p_t>(src, b));
    lane_store(dst, item, x);
  } else {
    fp12_t x = lane_load<fp12_t>(src, a);
    if (b >= 0) x = fp12_mul(x, lane_load<fp12_t>(src, b));
    lane_store(dst, item, x);
  }
}

__global__ void __launch_bounds__(LSG_TPB) k_final_exp_check(int ng, const uint32_t* __restrict__ F,
                                                              int32_t* __restrict__ verdict) {
  LANE_ITEM(ng);
  bool one = fp12_is_one(final_exp(lane_load<fp12_t>(F, item)));
  if (lead) verdict[item] = one ? 1 : 0;
}

LSG_DEVI fp12_t fp12_from_canon_bytes(const uint8_t* b) {
  fp12_t f;
  fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int j = 0; j < 6; j++) {
    c[j]->c0 = fp_to_mont(fp_from_be48(b + 96 * j));
    c[j]->c1 = fp_to_mont(fp_from_be48(b + 96 * j + 48));
  }
  return f;
}

// partials: canonical big-endian 576-byte Fp12 blobs -> lane form (one item each)
__global__ void __launch_bounds__(LSG_TPB) k_blobs_to_fp12(int n, const uint8_t* __restrict__ blobs,
                                                            uint32_t* __restrict__ out) {
  LANE_ITEM(n);
  lane_store(out, item, fp12_from_canon_bytes(blobs + 576 * item));
}

__global__ void __launch_bounds__(LSG_TPB) k_fp12_to_canon(int n, const uint32_t* __restrict__ in,
                                                            uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  const fp12_t f = lane_load<fp12_t>(in, item);
  const fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  uint8_t* o = out + 576 * item;
  for (int j = 0; j < 6; j++) {
    fp_to_be48(o + 96 * j, fp_from_mont(c[j]->c0));
    fp_to_be48(o + 96 * j + 48, fp_from_mont(c[j]->c1));
  }
}

__global__ void __launch_bounds__(LSG_TPB) k_g1p_to_bytes(int n, const uint32_t* __restrict__ pts,
                                                           uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  g1p_t p = lane_load<g1p_t>(pts, item);
  bool inf = proj_is_inf(p);
  g1a_t a;
  if (inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    a = proj_to_aff(p);
  }
  g1_serialize(out + 96 * item, a, inf);
}

__global__ void __launch_bounds__(LSG_TPB) k_g2a_to_bytes(int n, const uint32_t* __restrict__ pts,
                                                           const uint8_t* __restrict__ inf, uint8_t* __restrict__ out) {
  LANE_ITEM(n);
  g2_serialize(out + 192 * item, lane_load<g2a_t>(pts, item), inf[item] != 0);
}

// [k]P for a 256-bit big-endian scalar (test-data utilities only: signing, keygen)
template <class F>
__device__ proj_t<F> proj_mul_be256(const proj_t<F>& p, const uint8_t* k) {
  proj_t<F> acc = proj_inf<F>();
  for (int byte = 0; byte < 32; byte++) {
    uint32_t v = k[byte];
    for (int b = 7; b >= 0; b--) {
      acc = gdbl(acc);
      proj_t<F> s = gadd(acc, p);
      bool bit = (v >> b) & 1u;
      acc.X = fselect(bit, s.X, acc.X);
      acc.Y = fselect(bit, s.Y, acc.Y);
      acc.Z = fselect(bit, s.Z, acc.Z);
    }
  }
  return acc;
}

// sig_i = [sk_i] H(m_i), ZCash-compressed (bench/test input generation; not on the verify path)
__global__ void __launch_bounds__(LSG_TPB) k_sign(int n, const uint8_t* __restrict__ sks, const uint32_t* __restrict__ H,
                                                   uint8_t* __restrict__ out96) {
  LANE_ITEM(n);
  g2p_t s = proj_mul_be256(proj_from_aff(lane_load<g2a_t>(H, item)), sks + 32 * item);
  bool inf = proj_is_inf(s);
  g2a_t a;
  if (inf) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    a = proj_to_aff(s);
  }
  g2_compress(out96 + 96 * item, a, inf);
}

// pk_i = [sk_i] G1, uncompressed 96 bytes (bench/test input generation)
__global__ void __launch_bounds__(LSG_TPB) k_sk_to_pk(int n, const uint8_t* __restrict__ sks,
                                                       uint8_t* __restrict__ out96) {
  LANE_ITEM(n);
  g1a_t g;
  g.x = fp_t(G1_GEN_X);
  g.y = fp_t(G1_GEN_Y);
  g1p_t s = proj_mul_be256(proj_from_aff(g), sks + 32 * item);
  bool inf = proj_is_inf(s);
  g1a_t a;
  if (inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    a = proj_to_aff(s);
  }
  g1_serialize(out96 + 96 * item, a, inf);
}

// roofline probe: 4 independent limb-parallel Montgomery chains per row
__global__ void __launch_bounds__(LSG_TPB) k_probe_fp_mul(int n, int iters, uint32_t* __restrict__ io) {
  LANE_ITEM(n);
  fp_t a = lane_load<fp_t>(io, item), b = fp_t(FP_R2), c = fp_t(FP_R3), d = fp_t(FP_HALF);
  for (int k = 0; k < iters; k++) {
    a = fp_mul(a, b);
    b = fp_mul(b, c);
    c = fp_mul(c, d);
    d = fp_mul(d, a);
  }
  lane_store(io, item, fp_add(fp_add(a, b), fp_add(c, d)));
}

// ---------------------------------------------------------------------------- host side
namespace {

const uint8_t DST_POP[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
const uint32_t DST_POP_LEN = 43;

// u32 words per item for each lane-form type
constexpr size_t W_G1A = lane_words<g1a_t>();
constexpr size_t W_G1P = lane_words<g1p_t>();
constexpr size_t W_G2A = lane_words<g2a_t>();
constexpr size_t W_G2P = lane_words<g2p_t>();
constexpr size_t W_F12 = lane_words<fp12_t>();
constexpr size_t W_MAX = W_F12;

uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

struct Timer {
  const char* name;
  hipEvent_t a, b;
};

}  // namespace

struct TreeSlot {
  DevBuf idx, tA, tB;
  std::vector<int32_t> host;  // index pairs of the last reduction (alive until the call syncs)
};

// Three streams: S0 = hash_to_G2 -> Miller loops -> products -> FE, S1 = pubkeys,
// S2 = signatures (decode, subgroup, RLC scaling, sums, sig Miller loop).  Stage order is
// encoded with events; one synchronisation per phase.
struct lsg_ctx {
  int device = 0;
  hipStream_t st[3] = {nullptr, nullptr, nullptr};
  int cur = 0;
  hipEvent_t ev_pk = nullptr, ev_sig = nullptr, ev_grp = nullptr;
  std::mutex mu;
  std::string err;
  // inputs
  DevBuf d_sig, d_siglen, d_msg, d_msgoff, d_msglen, d_pk, d_pklen, d_rnd, d_dst;
  // per-set / per-pk state
  DevBuf d_ub, d_sigaff, d_siginf, d_seterr, d_pkp, d_pkerr, d_agg, d_P, d_pinf, d_H, d_hinf, d_rs, d_fall;
  // groups and reductions
  DevBuf d_S, d_F, d_verdict, d_blob, d_aux;
  TreeSlot tree[3];
  std::vector<Timer> timers;
  size_t ntimers = 0;
  size_t n_sets = 0, n_pks = 0;
  std::vector<uint32_t> pk_off, pk_cnt;  // host copy of the staged set -> pk ranges
  std::vector<std::vector<int32_t>> sets_pks;
};

namespace {

int fail(lsg_ctx* c, const char* what, hipError_t e) {
  c->err = std::string(what) + ": " + hipGetErrorString(e);
  return LSG_ERR_DEVICE;
}

#define LSG_HIP(c, call)                               \
  do {                                                 \
    hipError_t _e = (call);                            \
    if (_e != hipSuccess) return fail((c), #call, _e); \
  } while (0)

int ensure(lsg_ctx* c, DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 64;
  if (b.cap >= bytes) return LSG_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t cap = std::max(bytes + bytes / 4, (size_t)4096);
  hipError_t e = hipMalloc(&b.p, cap);
  if (e != hipSuccess) return fail(c, "hipMalloc", e);
  b.cap = cap;
  return LSG_OK;
}

template <class T>
T* P_(DevBuf& b) {
  return (T*)b.p;
}

int lane_blocks(size_t items) { return (int)((items + LSG_ITEMS_PER_BLOCK - 1) / LSG_ITEMS_PER_BLOCK); }

inline hipStream_t S_(lsg_ctx* c) { return c->st[c->cur]; }

void timer_reset(lsg_ctx* c) {
  c->ntimers = 0;
  c->cur = 0;
}

void timer_begin(lsg_ctx* c, const char* name) {
  if (c->ntimers >= c->timers.size()) {
    Timer t;
    (void)hipEventCreate(&t.a);
    (void)hipEventCreate(&t.b);
    c->timers.push_back(t);
  }
  Timer& t = c->timers[c->ntimers];
  t.name = name;
  (void)hipEventRecord(t.a, S_(c));
}

void timer_end(lsg_ctx* c) {
  (void)hipEventRecord(c->timers[c->ntimers].b, S_(c));
  c->ntimers++;
}

#define LAUNCH_T(c, name, kern, grid, tpb, ...)                                       \
  do {                                                                                \
    timer_begin((c), name);                                                           \
    hipLaunchKernelGGL(kern, dim3(grid), dim3(tpb), 0, S_(c), __VA_ARGS__);           \
    timer_end((c));                                                                   \
    hipError_t _le = hipGetLastError();                                               \
    if (_le != hipSuccess) return fail((c), name, _le);                               \
  } while (0)
#define LAUNCH(c, kern, items, ...) LAUNCH_T(c, #kern, kern, lane_blocks(items), LSG_TPB, __VA_ARGS__)

int sync_all(lsg_ctx* c) {
  for (int k = 0; k < 3; k++) LSG_HIP(c, hipStreamSynchronize(c->st[k]));
  return LSG_OK;
}

// ---- stage a package of sets into device memory (one synchronous batch of copies)
int stage_sets(lsg_ctx* c, const lsg_set* const* sets, size_t n, uint64_t seed, bool scale) {
  size_t npk = 0, msg_total = 0;
  for (size_t i = 0; i < n; i++) {
    npk += sets[i]->n_pks;
    msg_total += sets[i]->msg_len;
  }
  c->n_sets = n;
  c->n_pks = npk;
  size_t nn = std::max(n, (size_t)1), np = std::max(npk, (size_t)1);
  std::vector<uint8_t> sig(192 * nn, 0), msg(std::max(msg_total, (size_t)1)), pk(96 * np, 0);
  std::vector<uint32_t> siglen(nn), msgoff(nn), msglen(nn), pklen(np);
  std::vector<uint64_t> rnd(nn);
  c->pk_off.assign(n, 0);
  c->pk_cnt.assign(n, 0);
  size_t mo = 0, po = 0;
  uint64_t s = seed;
  FILE* ur = nullptr;
  if (scale && seed == 0) ur = fopen("/dev/urandom", "rb");
  for (size_t i = 0; i < n; i++) {
    const lsg_set* q = sets[i];
    siglen[i] = q->sig_len;
    if ((q->sig_len == 96 || q->sig_len == 192) && q->sig) memcpy(&sig[192 * i], q->sig, q->sig_len);
    msgoff[i] = (uint32_t)mo;
    msglen[i] = q->msg_len;
    if (q->msg_len) memcpy(&msg[mo], q->msg, q->msg_len);
    mo += q->msg_len;
    c->pk_off[i] = (uint32_t)po;
    c->pk_cnt[i] = q->n_pks;
    for (uint32_t k = 0; k < q->n_pks; k++) {
      pklen[po] = q->pk_len;
      if (q->pk_len == 48 || q->pk_len == 96) memcpy(&pk[96 * po], q->pks + (size_t)q->pk_len * k, q->pk_len);
      po++;
    }
    uint64_t r = 0;
    if (scale) {
      do {
        if (ur) {
          if (fread(&r, 8, 1, ur) != 1) r = splitmix64(s) ^ now_ns();
        } else {
          r = splitmix64(s);
        }
      } while (r == 0);
    }
    rnd[i] = r;
  }
  if (ur) fclose(ur);
  // per-set pubkey index lists for the aggregation tree (a set without keys points at
  // pk 0 and is reported as an empty aggregate by read_status)
  c->sets_pks.assign(n, {});
  for (size_t i = 0; i < n; i++) {
    for (uint32_t k = 0; k < c->pk_cnt[i]; k++) c->sets_pks[i].push_back((int32_t)(c->pk_off[i] + k));
    if (c->sets_pks[i].empty()) c->sets_pks[i].push_back(0);
  }
  int rc;
  if ((rc = ensure(c, c->d_sig, sig.size())) || (rc = ensure(c, c->d_siglen, 4 * nn)) ||
      (rc = ensure(c, c->d_msg, msg.size())) || (rc = ensure(c, c->d_msgoff, 4 * nn)) ||
      (rc = ensure(c, c->d_msglen, 4 * nn)) || (rc = ensure(c, c->d_pk, pk.size())) ||
      (rc = ensure(c, c->d_pklen, 4 * np)) || (rc = ensure(c, c->d_rnd, 8 * nn)) || (rc = ensure(c, c->d_dst, 256)) ||
      (rc = ensure(c, c->d_ub, 256 * nn)) || (rc = ensure(c, c->d_sigaff, 4 * W_G2A * nn)) ||
      (rc = ensure(c, c->d_siginf, nn)) || (rc = ensure(c, c->d_seterr, 4 * nn)) ||
      (rc = ensure(c, c->d_pkp, 4 * W_G1P * np)) || (rc = ensure(c, c->d_pkerr, 4 * np)) ||
      (rc = ensure(c, c->d_agg, 4 * W_G1P * nn)) || (rc = ensure(c, c->d_P, 4 * W_G1A * nn)) ||
      (rc = ensure(c, c->d_pinf, nn)) || (rc = ensure(c, c->d_H, 4 * W_G2A * nn)) || (rc = ensure(c, c->d_hinf, nn)) ||
      (rc = ensure(c, c->d_rs, 4 * W_G2P * nn)))
    return rc;
  hipStream_t S = c->st[0];
  LSG_HIP(c, hipMemcpyAsync(c->d_sig.p, sig.data(), sig.size(), hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_siglen.p, siglen.data(), 4 * nn, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_msg.p, msg.data(), msg.size(), hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_msgoff.p, msgoff.data(), 4 * nn, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_msglen.p, msglen.data(), 4 * nn, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_pk.p, pk.data(), pk.size(), hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_pklen.p, pklen.data(), 4 * np, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_rnd.p, rnd.data(), 8 * nn, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_dst.p, DST_POP, DST_POP_LEN, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipStreamSynchronize(S));  // host vectors die at return; other streams see the data
  return LSG_OK;
}

// Segmented pairwise reduction of lane-form values on the current stream: for each group,
// combine the slots groups[g] of `src` (OP 0: G1 add, 1: G2 add, 2: Fp12 mul) into dense
// out[g].  All levels' index pairs are built on the host and uploaded once; each level is
// one launch over all pairs of all groups.  `slot` selects private scratch so that trees on
// different streams can run concurrently.
template <int OP>
int tree_reduce(lsg_ctx* c, int slot, const char* name, const uint32_t* src,
                const std::vector<std::vector<int32_t>>& groups, uint32_t* out) {
  size_t ng = groups.size();
  if (ng == 0) return LSG_OK;
  TreeSlot& T = c->tree[slot];
  size_t W = OP == 0 ? W_G1P : (OP == 1 ? W_G2P : W_F12);
  std::vector<std::vector<int32_t>> cur = groups;
  std::vector<int32_t>& idx = T.host;
  idx.clear();
  std::vector<std::pair<size_t, size_t>> levels;  // (offset into idx, count)
  size_t max_level = 0;
  for (;;) {
    bool done = true;
    for (auto& g : cur)
      if (g.size() > 1) done = false;
    size_t cnt = 0;
    std::vector<int32_t> ia, ib;
    std::vector<std::vector<int32_t>> nxt(ng);
    if (done) {  // final gather into out[g]
      for (size_t g = 0; g < ng; g++) {
        ia.push_back(!cur[g].empty() ? cur[g][0] : -1);
        ib.push_back(-1);
      }
      cnt = ng;
    } else {
      for (size_t g = 0; g < ng; g++) {
        for (size_t k = 0; k < cur[g].size(); k += 2) {
          ia.push_back(cur[g][k]);
          ib.push_back(k + 1 < cur[g].size() ? cur[g][k + 1] : -1);
          nxt[g].push_back((int32_t)cnt++);
        }
      }
    }
    levels.push_back({idx.size(), cnt});
    idx.insert(idx.end(), ia.begin(), ia.end());
    idx.insert(idx.end(), ib.begin(), ib.end());
    max_level = std::max(max_level, cnt);
    if (done) break;
    cur.swap(nxt);
  }
  int rc;
  if ((rc = ensure(c, T.idx, 4 * idx.size())) || (rc = ensure(c, T.tA, 4 * W * max_level)) ||
      (rc = ensure(c, T.tB, 4 * W * max_level)))
    return rc;
  LSG_HIP(c, hipMemcpyAsync(T.idx.p, idx.data(), 4 * idx.size(), hipMemcpyHostToDevice, S_(c)));
  const uint32_t* in = src;
  uint32_t* bufs[2] = {P_<uint32_t>(T.tA), P_<uint32_t>(T.tB)};
  for (size_t L = 0; L < levels.size(); L++) {
    size_t off = levels[L].first, cnt = levels[L].second;
    bool last = L + 1 == levels.size();
    uint32_t* dst = last ? out : bufs[L & 1];
    const int32_t* ia = P_<int32_t>(T.idx) + off;
    LAUNCH_T(c, name, k_tree_level<OP>, lane_blocks(cnt), LSG_TPB, (int)cnt, ia, ia + cnt, in, dst);
    in = dst;
  }
  return LSG_OK;
}

// Per-set stages on three streams (no host synchronisation):
//   S1: pubkeys -> aggregation tree -> [r_i] scaling            (event ev_pk)
//   S2: signature decode -> subgroup check (event ev_sig) -> [r_i] scaling
//   S0: expand_message -> hash_to_G2 -> wait ev_pk -> Miller loops f_i
// f_i is written to d_fall[0..n); the caller sized d_fall for n + groups slots.
int launch_set_stages(lsg_ctx* c) {
  int n = (int)c->n_sets, np = (int)c->n_pks;
  if (n == 0) return LSG_OK;
  // S1: pubkeys
  c->cur = 1;
  if (np > 0) {
    LAUNCH(c, k_pk_decode, np, np, P_<uint8_t>(c->d_pk), P_<uint32_t>(c->d_pklen), P_<uint32_t>(c->d_pkp),
           P_<int32_t>(c->d_pkerr));
    int rc = tree_reduce<0>(c, 1, "tree_g1_aggregate", P_<uint32_t>(c->d_pkp), c->sets_pks, P_<uint32_t>(c->d_agg));
    if (rc) return rc;
  }
  LAUNCH(c, k_pk_scale, n, n, P_<uint32_t>(c->d_agg), P_<uint64_t>(c->d_rnd), P_<uint32_t>(c->d_P),
         P_<uint8_t>(c->d_pinf));
  LSG_HIP(c, hipEventRecord(c->ev_pk, c->st[1]));
  // S2: signatures
  c->cur = 2;
  LAUNCH(c, k_sig_decode, n, n, P_<uint8_t>(c->d_sig), P_<uint32_t>(c->d_siglen), P_<uint32_t>(c->d_sigaff),
         P_<uint8_t>(c->d_siginf), P_<int32_t>(c->d_seterr));
  LAUNCH(c, k_sig_subgroup, n, n, P_<uint32_t>(c->d_sigaff), P_<uint8_t>(c->d_siginf), P_<int32_t>(c->d_seterr));
  LSG_HIP(c, hipEventRecord(c->ev_sig, c->st[2]));  // signature errors known
  LAUNCH(c, k_sig_scale, n, n, P_<uint32_t>(c->d_sigaff), P_<uint8_t>(c->d_siginf), P_<int32_t>(c->d_seterr),
         P_<uint64_t>(c->d_rnd), P_<uint32_t>(c->d_rs));
  // S0: messages, then the per-set Miller loops once pubkeys are scaled and signature
  // errors are known (k_miller_sets reads d_seterr)
  c->cur = 0;
  LAUNCH_T(c, "k_expand_msg", k_expand_msg, (n + 63) / 64, 64, n, P_<uint8_t>(c->d_msg), P_<uint32_t>(c->d_msgoff),
           P_<uint32_t>(c->d_msglen), P_<uint8_t>(c->d_dst), DST_POP_LEN, P_<uint8_t>(c->d_ub));
  LAUNCH(c, k_hash_map, n, n, P_<uint8_t>(c->d_ub), P_<uint32_t>(c->d_H), P_<uint8_t>(c->d_hinf));
  LSG_HIP(c, hipStreamWaitEvent(c->st[0], c->ev_pk, 0));
  LSG_HIP(c, hipStreamWaitEvent(c->st[0], c->ev_sig, 0));
  LAUNCH(c, k_miller_sets, n, n, P_<uint32_t>(c->d_P), P_<uint8_t>(c->d_pinf), P_<uint32_t>(c->d_H),
         P_<uint8_t>(c->d_hinf), P_<int32_t>(c->d_seterr), P_<uint32_t>(c->d_fall));
  return LSG_OK;
}

int size_miller_slots(lsg_ctx* c, size_t groups) {
  return ensure(c, c->d_fall, 4 * W_F12 * std::max(c->n_sets + groups, (size_t)1));
}

// Group stages (no host synchronisation): S2 sums [r_i] sig_i per group and runs the
// signature Miller loop; S0 multiplies each group's f_i with it and, if fe, runs the final
// exponentiation into d_verdict (else leaves the products in d_F).  Sets with errors
// contribute identities (f_i = 1, [r_i] sig_i = O), so groups may include them.
int launch_groups(lsg_ctx* c, const std::vector<std::vector<int32_t>>& groups, bool fe) {
  size_t ng = groups.size();
  if (ng == 0) return LSG_OK;
  size_t n = c->n_sets;
  int rc;
  if (c->d_fall.cap < 4 * W_F12 * (n + ng)) {
    c->err = "internal: Miller slot array too small";
    return LSG_ERR_INVALID_ARG;
  }
  if ((rc = ensure(c, c->d_S, 4 * W_G2P * ng)) || (rc = ensure(c, c->d_F, 4 * W_F12 * ng)) ||
      (rc = ensure(c, c->d_verdict, 4 * ng)))
    return rc;
  c->cur = 2;
  if ((rc = tree_reduce<1>(c, 2, "tree_g2_sigsum", P_<uint32_t>(c->d_rs), groups, P_<uint32_t>(c->d_S)))) return rc;
  LAUNCH(c, k_miller_groups, ng, (int)ng, P_<uint32_t>(c->d_S), n, P_<uint32_t>(c->d_fall));
  LSG_HIP(c, hipEventRecord(c->ev_grp, c->st[2]));
  c->cur = 0;
  LSG_HIP(c, hipStreamWaitEvent(c->st[0], c->ev_grp, 0));
  std::vector<std::vector<int32_t>> fg = groups;
  for (size_t g = 0; g < ng; g++) fg[g].push_back((int32_t)(n + g));
  if ((rc = tree_reduce<2>(c, 0, "tree_fp12_product", P_<uint32_t>(c->d_fall), fg, P_<uint32_t>(c->d_F)))) return rc;
  if (fe) LAUNCH(c, k_final_exp_check, ng, (int)ng, P_<uint32_t>(c->d_F), P_<int32_t>(c->d_verdict));
  return LSG_OK;
}

struct SetStatus {
  std::vector<int32_t> err;    // per set: BLST code (0 ok)
  std::vector<uint8_t> pinf;   // per set: aggregated pk is infinity (2: no keys at all)
  std::vector<int32_t> pkerr;  // per pubkey
};

// Copies per-set status (and optionally ng verdicts) to the host on S0 and waits for all
// streams; S0 has already waited on S1/S2 through events.
int finish(lsg_ctx* c, SetStatus* ss, std::vector<int32_t>* verdict, size_t ng) {
  size_t n = c->n_sets, np = c->n_pks;
  hipStream_t S = c->st[0];
  if (ss) {
    ss->err.assign(n, 0);
    ss->pinf.assign(n, 0);
    ss->pkerr.assign(np, 0);
    if (n) {
      LSG_HIP(c, hipMemcpyAsync(ss->err.data(), c->d_seterr.p, 4 * n, hipMemcpyDeviceToHost, S));
      LSG_HIP(c, hipMemcpyAsync(ss->pinf.data(), c->d_pinf.p, n, hipMemcpyDeviceToHost, S));
    }
    if (np) LSG_HIP(c, hipMemcpyAsync(ss->pkerr.data(), c->d_pkerr.p, 4 * np, hipMemcpyDeviceToHost, S));
  }
  if (verdict) {
    verdict->assign(ng, 0);
    if (ng) LSG_HIP(c, hipMemcpyAsync(verdict->data(), c->d_verdict.p, 4 * ng, hipMemcpyDeviceToHost, S));
  }
  int rc = sync_all(c);
  if (rc) return rc;
  if (ss)
    for (size_t i = 0; i < n; i++)
      if (c->pk_cnt[i] == 0) ss->pinf[i] = 2;  // PublicKey.aggregate([]) throws
  return LSG_OK;
}

// chunkifyMaximizeChunkSize (multithread/utils.ts:4-19)
std::vector<std::pair<size_t, size_t>> chunkify(size_t len, size_t min_per_chunk) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t chunk_count = len / min_per_chunk;
  if (chunk_count <= 1) {
    out.push_back({0, len});
    return out;
  }
  size_t per = (len + chunk_count - 1) / chunk_count;
  for (size_t i = 0; i < len; i += per) out.push_back({i, std::min(len, i + per)});
  return out;
}

int32_t set_error(const SetStatus& ss, size_t s) {
  if (ss.err[s]) return ss.err[s];
  if (ss.pinf[s] == 2) return LSG_ERR_EMPTY_AGGREGATE;
  return ss.pinf[s] ? LSG_BLST_PK_IS_INFINITY : 0;
}

// Error a job's maybeBatch call would throw, in the reference's order:
// Signature.fromBytes over all sets first (maybeBatch.ts:17-26 map), then
// mul_n_aggregate rejecting an infinite public key (BLST_PK_IS_INFINITY).
int32_t job_error(const SetStatus& ss, size_t first, size_t count) {
  if (count == 0) return LSG_ERR_EMPTY_SET;
  for (size_t k = 0; k < count; k++)
    if (ss.err[first + k]) return ss.err[first + k];
  for (size_t k = 0; k < count; k++)
    if (ss.pinf[first + k]) return set_error(ss, first + k);
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------------- C ABI
extern "C" {

int lsg_init(int device_ordinal, lsg_ctx** out) {
  if (!out) return LSG_ERR_INVALID_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return LSG_ERR_NO_DEVICE;
  int dev = device_ordinal < 0 ? 0 : device_ordinal;
  if (dev >= count) return LSG_ERR_NO_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return LSG_ERR_NO_DEVICE;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return LSG_ERR_NO_DEVICE;
  lsg_ctx* c = new lsg_ctx();
  c->device = dev;
  bool ok = hipSetDevice(dev) == hipSuccess;
  for (int k = 0; k < 3 && ok; k++) ok = hipStreamCreateWithFlags(&c->st[k], hipStreamNonBlocking) == hipSuccess;
  hipEvent_t* evs[] = {&c->ev_pk, &c->ev_sig, &c->ev_grp};
  for (hipEvent_t* e : evs)
    if (ok) ok = hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    lsg_destroy(c);
    return LSG_ERR_DEVICE;
  }
  *out = c;
  return LSG_OK;
}

int lsg_destroy(lsg_ctx* c) {
  if (!c) return LSG_ERR_INVALID_ARG;
  (void)hipSetDevice(c->device);
  for (int k = 0; k < 3; k++)
    if (c->st[k]) (void)hipStreamSynchronize(c->st[k]);
  DevBuf* bufs[] = {&c->d_sig,   &c->d_siglen, &c->d_msg,    &c->d_msgoff, &c->d_msglen, &c->d_pk,
                    &c->d_pklen, &c->d_rnd,    &c->d_dst,    &c->d_ub,     &c->d_sigaff, &c->d_siginf,
                    &c->d_seterr, &c->d_pkp,   &c->d_pkerr,  &c->d_agg,    &c->d_P,      &c->d_pinf,
                    &c->d_H,     &c->d_hinf,   &c->d_rs,     &c->d_fall,   &c->d_S,      &c->d_F,
                    &c->d_verdict, &c->d_blob, &c->d_aux};
  for (DevBuf* b : bufs)
    if (b->p) (void)hipFree(b->p);
  for (TreeSlot& t : c->tree) {
    DevBuf* tb[] = {&t.idx, &t.tA, &t.tB};
    for (DevBuf* b : tb)
      if (b->p) (void)hipFree(b->p);
  }
  for (Timer& t : c->timers) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  hipEvent_t evs[] = {c->ev_pk, c->ev_sig, c->ev_grp};
  for (hipEvent_t e : evs)
    if (e) (void)hipEventDestroy(e);
  for (int k = 0; k < 3; k++)
    if (c->st[k]) (void)hipStreamDestroy(c->st[k]);
  delete c;
  return LSG_OK;
}

const char* lsg_last_error(lsg_ctx* c) { return c ? c->err.c_str() : "null context"; }

int lsg_device_name(lsg_ctx* c, char* buf, size_t len) {
  if (!c || !buf || !len) return LSG_ERR_INVALID_ARG;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) return LSG_ERR_DEVICE;
  snprintf(buf, len, "%s (%s, %d CUs)", prop.name, prop.gcnArchName, prop.multiProcessorCount);
  return LSG_OK;
}

// Phase A is launched speculatively: every batchable chunk and every non-batchable job gets
// its group (sum of [r_i] sig_i, Miller product, final exponentiation) before the per-set
// status is known, so the whole package costs one host synchronisation.  Sets that fail
// to decode contribute identities; the host then discards the verdicts of groups that the
// reference would have thrown on (worker.ts:51-96) and re-runs those jobs one by one.
int lsg_verify_jobs(lsg_ctx* c, const lsg_job* jobs, size_t n_jobs, uint64_t seed, lsg_job_result* results,
                    lsg_stats* stats) {
  if (!c || (n_jobs && (!jobs || !results))) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  lsg_stats stt;
  memset(&stt, 0, sizeof(stt));
  stt.start_ns = now_ns();
  timer_reset(c);
  std::vector<const lsg_set*> flat;
  std::vector<size_t> jfirst(n_jobs), jcount(n_jobs);
  for (size_t j = 0; j < n_jobs; j++) {
    jfirst[j] = flat.size();
    jcount[j] = jobs[j].n_sets;
    for (uint32_t k = 0; k < jobs[j].n_sets; k++) flat.push_back(&jobs[j].sets[k]);
  }
  for (size_t j = 0; j < n_jobs; j++) results[j] = {LSG_INVALID, 0};
  std::vector<size_t> batchable, nonbatch;
  for (size_t j = 0; j < n_jobs; j++) (jobs[j].flags & LSG_JOB_BATCHABLE ? batchable : nonbatch).push_back(j);
  auto job_group = [&](size_t j) {
    std::vector<int32_t> m;
    for (size_t k = 0; k < jcount[j]; k++) m.push_back((int32_t)(jfirst[j] + k));
    return m;
  };
  // Phase A groups: batchable chunks (worker.ts:51-86) + non-batchable jobs (worker.ts:88-96)
  std::vector<std::vector<int32_t>> groups;
  std::vector<std::vector<size_t>> group_jobs;
  std::vector<bool> group_is_chunk;
  std::vector<std::vector<size_t>> empty_chunks;  // chunks without sets: always throw
  if (!batchable.empty()) {
    for (auto ch : chunkify(batchable.size(), 16)) {
      std::vector<int32_t> m;
      std::vector<size_t> js;
      for (size_t q = ch.first; q < ch.second; q++) {
        size_t j = batchable[q];
        js.push_back(j);
        std::vector<int32_t> jm = job_group(j);
        m.insert(m.end(), jm.begin(), jm.end());
      }
      if (m.empty()) {
        empty_chunks.push_back(js);
        continue;
      }
      groups.push_back(m);
      group_jobs.push_back(js);
      group_is_chunk.push_back(true);
    }
  }
  for (size_t j : nonbatch) {
    if (jcount[j] == 0) {
      results[j] = {LSG_ERROR, LSG_ERR_EMPTY_SET};
      continue;
    }
    groups.push_back(job_group(j));
    group_jobs.push_back({j});
    group_is_chunk.push_back(false);
  }
  int rc = stage_sets(c, flat.data(), flat.size(), seed, true);
  if (rc) return rc;
  if ((rc = size_miller_slots(c, std::max(groups.size(), n_jobs)))) return rc;
  if ((rc = launch_set_stages(c))) return rc;
  if ((rc = launch_groups(c, groups, true))) return rc;
  SetStatus ss;
  std::vector<int32_t> verdict;
  if ((rc = finish(c, &ss, &verdict, groups.size()))) return rc;
  stt.n_final_exps += (uint32_t)groups.size();
  // worker.ts:108-114: deserializeSet runs before anything else; a bad pubkey throws
  // out of verifyManySignatureSets and rejects every job of the package.
  int32_t pkfail = 0;
  for (size_t k = 0; k < c->n_pks && !pkfail; k++) pkfail = ss.pkerr[k];
  if (pkfail) {
    for (size_t j = 0; j < n_jobs; j++) results[j] = {LSG_ERROR, pkfail};
    stt.end_ns = now_ns();
    if (stats) *stats = stt;
    return LSG_OK;
  }
  std::vector<size_t> retry;
  for (auto& js : empty_chunks) {
    stt.batch_retries++;
    retry.insert(retry.end(), js.begin(), js.end());
  }
  for (size_t g = 0; g < groups.size(); g++) {
    if (group_is_chunk[g]) {
      bool throws = false;
      for (int32_t s : groups[g])
        if (set_error(ss, (size_t)s)) throws = true;
      if (!throws && verdict[g]) {
        for (size_t j : group_jobs[g]) {
          results[j] = {LSG_VALID, 0};
          stt.batch_sigs_success += (uint32_t)jcount[j];
        }
      } else {
        stt.batch_retries++;
        retry.insert(retry.end(), group_jobs[g].begin(), group_jobs[g].end());
      }
    } else {
      size_t j = group_jobs[g][0];
      int32_t e = job_error(ss, jfirst[j], jcount[j]);
      results[j] = e ? lsg_job_result{LSG_ERROR, e} : lsg_job_result{verdict[g] ? LSG_VALID : LSG_INVALID, 0};
    }
  }
  // Phase B: per-job retry of failed chunks (worker.ts:74-96)
  if (!retry.empty()) {
    std::vector<std::vector<int32_t>> g2;
    std::vector<size_t> g2job;
    for (size_t j : retry) {
      int32_t e = job_error(ss, jfirst[j], jcount[j]);
      if (e) {
        results[j] = {LSG_ERROR, e};
      } else {
        g2.push_back(job_group(j));
        g2job.push_back(j);
      }
    }
    if ((rc = launch_groups(c, g2, true))) return rc;
    if ((rc = finish(c, nullptr, &verdict, g2.size()))) return rc;
    stt.n_final_exps += (uint32_t)g2.size();
    for (size_t g = 0; g < g2.size(); g++) results[g2job[g]] = {verdict[g] ? LSG_VALID : LSG_INVALID, 0};
  }
  stt.end_ns = now_ns();
  if (stats) *stats = stt;
  return LSG_OK;
}

int lsg_verify_sets(lsg_ctx* c, const lsg_set* sets, size_t n_sets, uint64_t seed, lsg_job_result* result) {
  if (!c || !result || (n_sets && !sets)) return LSG_ERR_INVALID_ARG;
  lsg_job job;
  job.sets = sets;
  job.n_sets = (uint32_t)n_sets;
  job.flags = 0;
  return lsg_verify_jobs(c, &job, 1, seed, result, nullptr);
}

int lsg_aggregate_pubkeys(lsg_ctx* c, const uint8_t* pks, uint32_t pk_len, size_t n, uint8_t* out96,
                          int32_t* err_code) {
  if (!c || !out96 || !err_code || (n && !pks)) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  timer_reset(c);
  *err_code = 0;
  if (n == 0) {
    *err_code = LSG_ERR_EMPTY_AGGREGATE;
    return LSG_OK;
  }
  lsg_set s;
  memset(&s, 0, sizeof(s));
  s.pks = pks;
  s.pk_len = pk_len;
  s.n_pks = (uint32_t)n;
  const lsg_set* sp = &s;
  int rc = stage_sets(c, &sp, 1, 0, false);
  if (rc) return rc;
  int np = (int)n;
  LAUNCH(c, k_pk_decode, np, np, P_<uint8_t>(c->d_pk), P_<uint32_t>(c->d_pklen), P_<uint32_t>(c->d_pkp),
         P_<int32_t>(c->d_pkerr));
  std::vector<std::vector<int32_t>> g(1);
  for (int k = 0; k < np; k++) g[0].push_back(k);
  if ((rc = tree_reduce<0>(c, 1, "tree_g1_aggregate", P_<uint32_t>(c->d_pkp), g, P_<uint32_t>(c->d_agg)))) return rc;
  if ((rc = ensure(c, c->d_blob, 192))) return rc;
  LAUNCH(c, k_g1p_to_bytes, 1, 1, P_<uint32_t>(c->d_agg), P_<uint8_t>(c->d_blob));
  std::vector<int32_t> pkerr(n);
  LSG_HIP(c, hipMemcpyAsync(pkerr.data(), c->d_pkerr.p, 4 * n, hipMemcpyDeviceToHost, c->st[0]));
  LSG_HIP(c, hipMemcpyAsync(out96, c->d_blob.p, 96, hipMemcpyDeviceToHost, c->st[0]));
  LSG_HIP(c, hipStreamSynchronize(c->st[0]));
  for (size_t k = 0; k < n; k++)
    if (pkerr[k]) {
      *err_code = pkerr[k];
      break;
    }
  return LSG_OK;
}

int lsg_hash_to_g2(lsg_ctx* c, const uint8_t* msgs, uint32_t msg_len, size_t n, const uint8_t* dst,
                   uint32_t dst_len, uint8_t* out192) {
  if (!c || (n && msg_len && !msgs) || dst_len > 255 || (dst_len && !dst)) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  timer_reset(c);
  if (n == 0) return LSG_OK;
  std::vector<lsg_set> sets(n);
  std::vector<const lsg_set*> sp(n);
  for (size_t i = 0; i < n; i++) {
    memset(&sets[i], 0, sizeof(lsg_set));
    sets[i].msg = msgs + (size_t)msg_len * i;
    sets[i].msg_len = msg_len;
    sp[i] = &sets[i];
  }
  int rc = stage_sets(c, sp.data(), n, 0, false);
  if (rc) return rc;
  LSG_HIP(c, hipMemcpyAsync(c->d_dst.p, dst, dst_len, hipMemcpyHostToDevice, c->st[0]));
  int nn = (int)n;
  LAUNCH_T(c, "k_expand_msg", k_expand_msg, (nn + 63) / 64, 64, nn, P_<uint8_t>(c->d_msg), P_<uint32_t>(c->d_msgoff),
           P_<uint32_t>(c->d_msglen), P_<uint8_t>(c->d_dst), dst_len, P_<uint8_t>(c->d_ub));
  LAUNCH(c, k_hash_map, nn, nn, P_<uint8_t>(c->d_ub), P_<uint32_t>(c->d_H), P_<uint8_t>(c->d_hinf));
  if (!out192) {  // internal use (lsg_sign): leave H in d_H
    LSG_HIP(c, hipStreamSynchronize(c->st[0]));
    return LSG_OK;
  }
  if ((rc = ensure(c, c->d_blob, 192 * n))) return rc;
  LAUNCH(c, k_g2a_to_bytes, nn, nn, P_<uint32_t>(c->d_H), P_<uint8_t>(c->d_hinf), P_<uint8_t>(c->d_blob));
  LSG_HIP(c, hipMemcpyAsync(out192, c->d_blob.p, 192 * n, hipMemcpyDeviceToHost, c->st[0]));
  LSG_HIP(c, hipStreamSynchronize(c->st[0]));
  return LSG_OK;
}

int lsg_sig_decode(lsg_ctx* c, const uint8_t* sigs, uint32_t sig_len, size_t n, uint8_t* out192, int32_t* err) {
  if (!c || !out192 || !err || (n && !sigs)) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  timer_reset(c);
  if (n == 0) return LSG_OK;
  std::vector<lsg_set> sets(n);
  std::vector<const lsg_set*> sp(n);
  for (size_t i = 0; i < n; i++) {
    memset(&sets[i], 0, sizeof(lsg_set));
    sets[i].sig = sigs + (size_t)sig_len * i;
    sets[i].sig_len = sig_len;
    sp[i] = &sets[i];
  }
  int rc = stage_sets(c, sp.data(), n, 0, false);
  if (rc) return rc;
  int nn = (int)n;
  LAUNCH(c, k_sig_decode, nn, nn, P_<uint8_t>(c->d_sig), P_<uint32_t>(c->d_siglen), P_<uint32_t>(c->d_sigaff),
         P_<uint8_t>(c->d_siginf), P_<int32_t>(c->d_seterr));
  LAUNCH(c, k_sig_subgroup, nn, nn, P_<uint32_t>(c->d_sigaff), P_<uint8_t>(c->d_siginf), P_<int32_t>(c->d_seterr));
  if ((rc = ensure(c, c->d_blob, 192 * n))) return rc;
  LAUNCH(c, k_g2a_to_bytes, nn, nn, P_<uint32_t>(c->d_sigaff), P_<uint8_t>(c->d_siginf), P_<uint8_t>(c->d_blob));
  LSG_HIP(c, hipMemcpyAsync(out192, c->d_blob.p, 192 * n, hipMemcpyDeviceToHost, c->st[0]));
  LSG_HIP(c, hipMemcpyAsync(err, c->d_seterr.p, 4 * n, hipMemcpyDeviceToHost, c->st[0]));
  LSG_HIP(c, hipStreamSynchronize(c->st[0]));
  return LSG_OK;
}

int lsg_sign(lsg_ctx* c, const uint8_t* sks32, const uint8_t* msgs, uint32_t msg_len, size_t n, uint8_t* out96) {
  if (!c || !out96 || (n && (!sks32 || !msgs))) return LSG_ERR_INVALID_ARG;
  int rc = lsg_hash_to_g2(c, msgs, msg_len, n, DST_POP, DST_POP_LEN, nullptr);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = ensure(c, c->d_blob, 96 * std::max(n, (size_t)1))) || (rc = ensure(c, c->d_aux, 32 * std::max(n, (size_t)1))))
    return rc;
  LSG_HIP(c, hipMemcpyAsync(c->d_aux.p, sks32, 32 * n, hipMemcpyHostToDevice, c->st[0]));
  int nn = (int)n;
  LAUNCH(c, k_sign, nn, nn, P_<uint8_t>(c->d_aux), P_<uint32_t>(c->d_H), P_<uint8_t>(c->d_blob));
  LSG_HIP(c, hipMemcpyAsync(out96, c->d_blob.p, 96 * n, hipMemcpyDeviceToHost, c->st[0]));
  LSG_HIP(c, hipStreamSynchronize(c->st[0]));
  return LSG_OK;
}

int lsg_sk_to_pk(lsg_ctx* c, const uint8_t* sks32, size_t n, uint8_t* out96) {
  if (!c || !out96 || (n && !sks32)) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure(c, c->d_blob, 96 * std::max(n, (size_t)1))) || (rc = ensure(c, c->d_aux, 32 * std::max(n, (size_t)1))))
    return rc;
  LSG_HIP(c, hipMemcpyAsync(c->d_aux.p, sks32, 32 * n, hipMemcpyHostToDevice, c->st[0]));
  int nn = (int)n;
  LAUNCH(c, k_sk_to_pk, nn, nn, P_<uint8_t>(c->d_aux), P_<uint8_t>(c->d_blob));
  LSG_HIP(c, hipMemcpyAsync(out96, c->d_blob.p, 96 * n, hipMemcpyDeviceToHost, c->st[0]));
  LSG_HIP(c, hipStreamSynchronize(c->st[0]));
  return LSG_OK;
}

int lsg_batch_stage(lsg_ctx* c, const lsg_set* sets, size_t n_sets, uint64_t seed) {
  if (!c || (n_sets && !sets)) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  std::vector<const lsg_set*> sp(n_sets);
  for (size_t i = 0; i < n_sets; i++) sp[i] = &sets[i];
  return stage_sets(c, sp.data(), n_sets, seed, true);
}

int lsg_batch_run(lsg_ctx* c, uint8_t* out576, int32_t* set_err, int32_t* any_error) {
  if (!c || !out576 || !any_error) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  timer_reset(c);
  size_t n_sets = c->n_sets;
  int rc;
  std::vector<std::vector<int32_t>> groups(1);
  for (size_t i = 0; i < n_sets; i++) groups[0].push_back((int32_t)i);
  if ((rc = size_miller_slots(c, 1))) return rc;
  if ((rc = ensure(c, c->d_blob, 576))) return rc;
  if ((rc = launch_set_stages(c))) return rc;
  // errored sets contribute identities, so the partial covers exactly the valid sets (an
  // empty package gives the identity)
  if ((rc = launch_groups(c, groups, false))) return rc;
  LAUNCH(c, k_fp12_to_canon, 1, 1, P_<uint32_t>(c->d_F), P_<uint8_t>(c->d_blob));
  LSG_HIP(c, hipMemcpyAsync(out576, c->d_blob.p, 576, hipMemcpyDeviceToHost, c->st[0]));
  SetStatus ss;
  if ((rc = finish(c, &ss, nullptr, 0))) return rc;
  *any_error = 0;
  for (size_t i = 0; i < n_sets; i++) {
    int32_t e = set_error(ss, i);
    if (set_err) set_err[i] = e;
    if (e) *any_error = 1;
  }
  for (size_t k = 0; k < c->n_pks; k++)
    if (ss.pkerr[k]) *any_error = 1;
  return LSG_OK;
}

int lsg_batch_partial(lsg_ctx* c, const lsg_set* sets, size_t n_sets, uint64_t seed, uint8_t* out576,
                      int32_t* set_err, int32_t* any_error) {
  int rc = lsg_batch_stage(c, sets, n_sets, seed);
  if (rc) return rc;
  return lsg_batch_run(c, out576, set_err, any_error);
}

int lsg_final_verify(lsg_ctx* c, const uint8_t* partials576, size_t n_partials, int32_t* valid) {
  if (!c || !valid || (n_partials && !partials576)) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  timer_reset(c);
  int rc;
  size_t np = std::max(n_partials, (size_t)1);
  if ((rc = ensure(c, c->d_blob, 576 * np)) || (rc = ensure(c, c->d_aux, 4 * W_F12 * np)) ||
      (rc = ensure(c, c->d_F, 4 * W_F12)) || (rc = ensure(c, c->d_verdict, 4)))
    return rc;
  if (n_partials == 0) {
    *valid = 0;
    return LSG_OK;
  }
  LSG_HIP(c, hipMemcpyAsync(c->d_blob.p, partials576, 576 * n_partials, hipMemcpyHostToDevice, c->st[0]));
  LAUNCH(c, k_blobs_to_fp12, n_partials, (int)n_partials, P_<uint8_t>(c->d_blob), P_<uint32_t>(c->d_aux));
  std::vector<std::vector<int32_t>> g(1);
  for (size_t k = 0; k < n_partials; k++) g[0].push_back((int32_t)k);
  if ((rc = tree_reduce<2>(c, 0, "tree_fp12_product", P_<uint32_t>(c->d_aux), g, P_<uint32_t>(c->d_F)))) return rc;
  LAUNCH(c, k_final_exp_check, 1, 1, P_<uint32_t>(c->d_F), P_<int32_t>(c->d_verdict));
  LSG_HIP(c, hipMemcpyAsync(valid, c->d_verdict.p, 4, hipMemcpyDeviceToHost, c->st[0]));
  LSG_HIP(c, hipStreamSynchronize(c->st[0]));
  return LSG_OK;
}

int lsg_probe_fp_mul_rate(lsg_ctx* c, double* fp_mul_per_s, double* mad_per_s) {
  if (!c || !fp_mul_per_s || !mad_per_s) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  hipDeviceProp_t prop;
  LSG_HIP(c, hipGetDeviceProperties(&prop, c->device));
  int items = prop.multiProcessorCount * 128;  // 32 waves of 4 rows per CU
  int rc;
  if ((rc = ensure(c, c->d_aux, 4 * 16 * (size_t)items))) return rc;
  std::vector<uint32_t> init(16 * (size_t)items, 0);
  for (size_t i = 0; i < init.size(); i++)
    if ((i & 15) < 11) init[i] = (uint32_t)(i * 2654435761u);
  LSG_HIP(c, hipMemcpy(c->d_aux.p, init.data(), 4 * init.size(), hipMemcpyHostToDevice));
  const int iters = 64;
  hipLaunchKernelGGL(k_probe_fp_mul, dim3(lane_blocks(items)), dim3(LSG_TPB), 0, c->st[0], items, 2,
                     P_<uint32_t>(c->d_aux));
  hipEvent_t a, b;
  LSG_HIP(c, hipEventCreate(&a));
  LSG_HIP(c, hipEventCreate(&b));
  LSG_HIP(c, hipEventRecord(a, c->st[0]));
  hipLaunchKernelGGL(k_probe_fp_mul, dim3(lane_blocks(items)), dim3(LSG_TPB), 0, c->st[0], items, iters,
                     P_<uint32_t>(c->d_aux));
  LSG_HIP(c, hipEventRecord(b, c->st[0]));
  LSG_HIP(c, hipEventSynchronize(b));
  float ms = 0;
  LSG_HIP(c, hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  double muls = (double)items * iters * 4.0;
  *fp_mul_per_s = muls / (ms * 1e-3);
  *mad_per_s = *fp_mul_per_s * 300.0;
  return LSG_OK;
}

int lsg_last_kernel_times(lsg_ctx* c, const char** names, double* ms, int max) {
  if (!c) return 0;
  for (int k = 0; k < 3; k++) (void)hipStreamSynchronize(c->st[k]);
  int n = 0;
  for (size_t i = 0; i < c->ntimers && n < max; i++) {
    float t = 0;
    if (hipEventElapsedTime(&t, c->timers[i].a, c->timers[i].b) != hipSuccess) t = -1;
    if (names) names[n] = c->timers[i].name;
    if (ms) ms[n] = t;
    n++;
  }
  return n;
}

}  // extern "C"
