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
// Device pipeline for one work package (all sets of all jobs at once, thread per item):
//   k_sig_decode      96/192-byte signature -> affine G2 (flags, x<p, sqrt, sign)     [M2]
//   k_sig_subgroup    psi(P) == [x]P                                                 [M2]
//   k_pk_decode       48/96-byte pubkey -> affine G1 (on-curve only, worker.ts:110)   [H8]
//   k_pk_agg_scale    sum of a set's pubkeys, times the set's 64-bit randomizer r_i  [M1,M4]
//   k_hash_to_g2      H(m_i)                                                         [M3]
//   k_sig_scale       [r_i] sig_i                                                    [M4]
//   k_miller_sets     f_i = ML([r_i]PK_i, H(m_i))                                    [M5]
// then per group (an RLC batch = one chunk of batchable jobs, or one job):
//   k_group_sum       S_g = sum_{i in g} [r_i] sig_i
//   k_miller_groups   f_g = ML(-G1, S_g)
//   k_group_fe        FE(f_g * prod_{i in g} f_i) == 1                                [M6]
// Per-set values stay resident between the batch attempt and the per-job retry, so a
// failed batch costs only the group sums, one extra Miller loop and one FE per job.
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
#include "lsg_h2c.hpp"
#include "lsg_pairing.hpp"

#define LSG_TPB 64

static __device__ __forceinline__ int gtid() { return blockIdx.x * blockDim.x + threadIdx.x; }

// ---------------------------------------------------------------------------- kernels
__global__ void __launch_bounds__(LSG_TPB) k_sig_decode(int n, const uint8_t* __restrict__ sig,
                                                         const uint32_t* __restrict__ sig_len, g2a_t* __restrict__ out,
                                                         uint8_t* __restrict__ inf, int32_t* __restrict__ err) {
  int i = gtid();
  if (i >= n) return;
  uint32_t len = sig_len[i];
  g2a_t p;
  p.x = fp2_zero();
  p.y = fp2_zero();
  bool is_inf = false;
  int e;
  if (len == 96)
    e = g2_uncompress(p, is_inf, sig + 192 * (size_t)i);
  else if (len == 192)
    e = g2_deserialize_uncompressed(p, is_inf, sig + 192 * (size_t)i);
  else
    e = LSG_BLST_INVALID_SIZE;
  out[i] = p;
  inf[i] = is_inf ? 1 : 0;
  err[i] = e;
}

__global__ void __launch_bounds__(LSG_TPB) k_sig_subgroup(int n, const g2a_t* __restrict__ sig,
                                                           const uint8_t* __restrict__ inf, int32_t* __restrict__ err) {
  int i = gtid();
  if (i >= n) return;
  if (err[i] != 0 || inf[i]) return;
  if (!g2_in_group(proj_from_aff(sig[i]))) err[i] = LSG_BLST_POINT_NOT_IN_GROUP;
}

__global__ void __launch_bounds__(LSG_TPB) k_pk_decode(int n, const uint8_t* __restrict__ pk,
                                                        const uint32_t* __restrict__ pk_len, g1a_t* __restrict__ out,
                                                        uint8_t* __restrict__ inf, int32_t* __restrict__ err) {
  int i = gtid();
  if (i >= n) return;
  uint32_t len = pk_len[i];
  g1a_t p;
  p.x = fp_zero();
  p.y = fp_zero();
  bool is_inf = false;
  int e = (len == 48 || len == 96) ? g1_deserialize(p, is_inf, pk + 96 * (size_t)i, (int)len) : LSG_BLST_INVALID_SIZE;
  out[i] = p;
  inf[i] = is_inf ? 1 : 0;
  err[i] = e;
}

// P_i = [r_i] * sum(pks of set i) in affine; pinf[i] = aggregate is infinity.
// r_i == 0 means "no scaling" (used by lsg_aggregate_pubkeys).
__global__ void __launch_bounds__(LSG_TPB) k_pk_agg_scale(int n, const uint32_t* __restrict__ pk_off,
                                                           const uint32_t* __restrict__ pk_cnt,
                                                           const g1a_t* __restrict__ pk, const uint8_t* __restrict__ pk_inf,
                                                           const uint64_t* __restrict__ rnd, g1a_t* __restrict__ out,
                                                           uint8_t* __restrict__ pinf) {
  int i = gtid();
  if (i >= n) return;
  g1p_t acc = proj_inf<fp_t>();
  uint32_t o = pk_off[i], c = pk_cnt[i];
  for (uint32_t k = 0; k < c; k++) {
    if (!pk_inf[o + k]) acc = g1_add_mixed(acc, pk[o + k]);
  }
  uint64_t r = rnd[i];
  if (r != 0 && !proj_is_inf(acc)) acc = proj_mul_u64(acc, r);
  bool is_inf = proj_is_inf(acc);
  g1a_t a;
  if (is_inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  } else {
    a = proj_to_aff(acc);
  }
  out[i] = a;
  pinf[i] = is_inf ? 1 : 0;
}

__global__ void __launch_bounds__(LSG_TPB) k_hash_to_g2(int n, const uint8_t* __restrict__ msg,
                                                         const uint32_t* __restrict__ msg_off,
                                                         const uint32_t* __restrict__ msg_len,
                                                         const uint8_t* __restrict__ dst, uint32_t dst_len,
                                                         g2a_t* __restrict__ out, uint8_t* __restrict__ hinf) {
  int i = gtid();
  if (i >= n) return;
  uint8_t ub[256];
  expand_message_xmd_256(ub, msg + msg_off[i], msg_len[i], dst, dst_len);
  fp2_t u0 = fp2_make(fp_from_be64_mod(ub), fp_from_be64_mod(ub + 64));
  fp2_t u1 = fp2_make(fp_from_be64_mod(ub + 128), fp_from_be64_mod(ub + 192));
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
  out[i] = a;
  hinf[i] = is_inf ? 1 : 0;
}

__global__ void __launch_bounds__(LSG_TPB) k_sig_scale(int n, const g2a_t* __restrict__ sig,
                                                        const uint8_t* __restrict__ inf, const int32_t* __restrict__ err,
                                                        const uint64_t* __restrict__ rnd, g2p_t* __restrict__ out) {
  int i = gtid();
  if (i >= n) return;
  g2p_t r = proj_inf<fp2_t>();
  if (err[i] == 0 && !inf[i]) r = proj_mul_u64(proj_from_aff(sig[i]), rnd[i]);
  out[i] = r;
}

__global__ void __launch_bounds__(LSG_TPB) k_miller_sets(int n, const g1a_t* __restrict__ P,
                                                          const uint8_t* __restrict__ pinf, const g2a_t* __restrict__ H,
                                                          const uint8_t* __restrict__ hinf,
                                                          const int32_t* __restrict__ err, fp12_t* __restrict__ f) {
  int i = gtid();
  if (i >= n) return;
  fp12_t r = fp12_one();
  if (err[i] == 0 && !pinf[i] && !hinf[i]) r = miller_loop(P[i], H[i]);
  f[i] = r;
}

__global__ void __launch_bounds__(LSG_TPB) k_group_sum(int ng, const uint32_t* __restrict__ goff,
                                                        const uint32_t* __restrict__ members,
                                                        const g2p_t* __restrict__ rs, g2a_t* __restrict__ S,
                                                        uint8_t* __restrict__ sinf) {
  int g = gtid();
  if (g >= ng) return;
  g2p_t acc = proj_inf<fp2_t>();
  for (uint32_t k = goff[g]; k < goff[g + 1]; k++) acc = g2_add(acc, rs[members[k]]);
  bool is_inf = proj_is_inf(acc);
  g2a_t a;
  if (is_inf) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  } else {
    a = proj_to_aff(acc);
  }
  S[g] = a;
  sinf[g] = is_inf ? 1 : 0;
}

// f_g = ML(-G1, S_g) = conj(ML(G1, S_g))
__global__ void __launch_bounds__(LSG_TPB) k_miller_groups(int ng, const g2a_t* __restrict__ S,
                                                            const uint8_t* __restrict__ sinf, fp12_t* __restrict__ f) {
  int g = gtid();
  if (g >= ng) return;
  fp12_t r = fp12_one();
  if (!sinf[g]) {
    g1a_t ng1;
    ng1.x = G1_GEN_X;
    ng1.y = G1_GEN_NEG_Y;
    r = miller_loop(ng1, S[g]);
  }
  f[g] = r;
}

__global__ void __launch_bounds__(LSG_TPB) k_group_product(int ng, const uint32_t* __restrict__ goff,
                                                            const uint32_t* __restrict__ members,
                                                            const fp12_t* __restrict__ fset,
                                                            const fp12_t* __restrict__ fgrp, fp12_t* __restrict__ out) {
  int g = gtid();
  if (g >= ng) return;
  fp12_t acc = fgrp[g];
  for (uint32_t k = goff[g]; k < goff[g + 1]; k++) acc = fp12_mul(acc, fset[members[k]]);
  out[g] = acc;
}

__global__ void __launch_bounds__(LSG_TPB) k_final_exp_check(int ng, const fp12_t* __restrict__ F,
                                                              int32_t* __restrict__ verdict) {
  int g = gtid();
  if (g >= ng) return;
  verdict[g] = fp12_is_one(final_exp(F[g])) ? 1 : 0;
}

// partials: canonical big-endian 576-byte Fp12 blobs -> product (Montgomery)
__global__ void k_partials_product(int n, const uint8_t* __restrict__ blobs, fp12_t* __restrict__ out) {
  if (gtid() != 0) return;
  fp12_t acc = fp12_one();
  for (int k = 0; k < n; k++) {
    const uint8_t* b = blobs + 576 * (size_t)k;
    fp12_t f;
    fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
    for (int j = 0; j < 6; j++) {
      c[j]->c0 = fp_to_mont(fp_from_be48(b + 96 * j));
      c[j]->c1 = fp_to_mont(fp_from_be48(b + 96 * j + 48));
    }
    acc = fp12_mul(acc, f);
  }
  out[0] = acc;
}

__global__ void k_fp12_to_canon(const fp12_t* __restrict__ in, uint8_t* __restrict__ out) {
  if (gtid() != 0) return;
  const fp12_t f = in[0];
  const fp2_t* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int j = 0; j < 6; j++) {
    fp_to_be48(out + 96 * j, fp_from_mont(c[j]->c0));
    fp_to_be48(out + 96 * j + 48, fp_from_mont(c[j]->c1));
  }
}

__global__ void __launch_bounds__(LSG_TPB) k_g1_to_bytes(int n, const g1a_t* __restrict__ a,
                                                          const uint8_t* __restrict__ inf, uint8_t* __restrict__ out) {
  int i = gtid();
  if (i >= n) return;
  g1_serialize(out + 96 * (size_t)i, a[i], inf[i] != 0);
}

__global__ void __launch_bounds__(LSG_TPB) k_g2_to_bytes(int n, const g2a_t* __restrict__ a,
                                                          const uint8_t* __restrict__ inf, uint8_t* __restrict__ out) {
  int i = gtid();
  if (i >= n) return;
  g2_serialize(out + 192 * (size_t)i, a[i], inf[i] != 0);
}

// roofline probe: 4 independent Montgomery chains per thread
__global__ void __launch_bounds__(256) k_probe_fp_mul(int iters, fp_t* __restrict__ io) {
  int i = gtid();
  fp_t a = io[i], b = io[i + 1], c = io[i + 2], d = io[i + 3];
  for (int k = 0; k < iters; k++) {
    a = fp_mul(a, b);
    b = fp_mul(b, c);
    c = fp_mul(c, d);
    d = fp_mul(d, a);
  }
  io[i] = fp_add(fp_add(a, b), fp_add(c, d));
}

// ---------------------------------------------------------------------------- host side
namespace {

const uint8_t DST_POP[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
const uint32_t DST_POP_LEN = 43;

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

struct lsg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::string err;
  // device buffers (grow-only)
  DevBuf d_sig, d_siglen, d_msg, d_msgoff, d_msglen, d_pk, d_pklen, d_pkoff, d_pkcnt, d_rnd;
  DevBuf d_sigaff, d_siginf, d_seterr, d_pkaff, d_pkinf, d_pkerr, d_P, d_pinf, d_H, d_hinf, d_rs, d_fset;
  DevBuf d_goff, d_members, d_S, d_sinf, d_fgrp, d_F, d_verdict, d_dst, d_blob, d_probe;
  // timing of the last call
  std::vector<Timer> timers;
  size_t ntimers = 0;
  std::vector<std::string> timer_names;
};

namespace {

int fail(lsg_ctx* c, const char* what, hipError_t e) {
  c->err = std::string(what) + ": " + hipGetErrorString(e);
  return LSG_ERR_DEVICE;
}

#define LSG_HIP(c, call)                              \
  do {                                                \
    hipError_t _e = (call);                           \
    if (_e != hipSuccess) return fail((c), #call, _e); \
  } while (0)

int ensure(lsg_ctx* c, DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 64;
  if (b.cap >= bytes) return LSG_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t cap = std::max(bytes, (size_t)4096);
  hipError_t e = hipMalloc(&b.p, cap);
  if (e != hipSuccess) return fail(c, "hipMalloc", e);
  b.cap = cap;
  return LSG_OK;
}

template <class T>
T* P_(DevBuf& b) {
  return (T*)b.p;
}

int blocks(size_t n) { return (int)((n + LSG_TPB - 1) / LSG_TPB); }

void timer_reset(lsg_ctx* c) { c->ntimers = 0; }

void timer_begin(lsg_ctx* c, const char* name) {
  if (c->ntimers >= c->timers.size()) {
    Timer t;
    (void)hipEventCreate(&t.a);
    (void)hipEventCreate(&t.b);
    c->timers.push_back(t);
  }
  Timer& t = c->timers[c->ntimers];
  t.name = name;
  (void)hipEventRecord(t.a, c->stream);
}

void timer_end(lsg_ctx* c) {
  (void)hipEventRecord(c->timers[c->ntimers].b, c->stream);
  c->ntimers++;
}

#define LAUNCH(c, name, grid, ...)                                        \
  do {                                                                    \
    timer_begin((c), #name);                                              \
    hipLaunchKernelGGL(name, dim3(grid), dim3(LSG_TPB), 0, (c)->stream, __VA_ARGS__); \
    timer_end((c));                                                       \
    hipError_t _le = hipGetLastError();                                   \
    if (_le != hipSuccess) return fail((c), #name, _le);                  \
  } while (0)

// Flattened view of a package of sets, staged to the device.
struct Staged {
  size_t n_sets = 0, n_pks = 0;
  std::vector<int32_t> host_err;  // per set (host-side size errors)
};

int stage_sets(lsg_ctx* c, const lsg_set* const* sets, size_t n, uint64_t seed, bool scale, Staged& st) {
  st.n_sets = n;
  size_t npk = 0, msg_total = 0;
  for (size_t i = 0; i < n; i++) {
    npk += sets[i]->n_pks;
    msg_total += sets[i]->msg_len;
  }
  st.n_pks = npk;
  std::vector<uint8_t> sig(192 * std::max(n, (size_t)1), 0), msg(std::max(msg_total, (size_t)1)),
      pk(96 * std::max(npk, (size_t)1), 0);
  std::vector<uint32_t> siglen(n), msgoff(n), msglen(n), pklen(std::max(npk, (size_t)1)), pkoff(n), pkcnt(n);
  std::vector<uint64_t> rnd(n);
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
    pkoff[i] = (uint32_t)po;
    pkcnt[i] = q->n_pks;
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
  int rc;
  size_t nn = std::max(n, (size_t)1), np = std::max(npk, (size_t)1);
  if ((rc = ensure(c, c->d_sig, sig.size())) || (rc = ensure(c, c->d_siglen, 4 * nn)) ||
      (rc = ensure(c, c->d_msg, msg.size())) || (rc = ensure(c, c->d_msgoff, 4 * nn)) ||
      (rc = ensure(c, c->d_msglen, 4 * nn)) || (rc = ensure(c, c->d_pk, pk.size())) ||
      (rc = ensure(c, c->d_pklen, 4 * np)) || (rc = ensure(c, c->d_pkoff, 4 * nn)) ||
      (rc = ensure(c, c->d_pkcnt, 4 * nn)) || (rc = ensure(c, c->d_rnd, 8 * nn)) ||
      (rc = ensure(c, c->d_sigaff, sizeof(g2a_t) * nn)) || (rc = ensure(c, c->d_siginf, nn)) ||
      (rc = ensure(c, c->d_seterr, 4 * nn)) || (rc = ensure(c, c->d_pkaff, sizeof(g1a_t) * np)) ||
      (rc = ensure(c, c->d_pkinf, np)) || (rc = ensure(c, c->d_pkerr, 4 * np)) ||
      (rc = ensure(c, c->d_P, sizeof(g1a_t) * nn)) || (rc = ensure(c, c->d_pinf, nn)) ||
      (rc = ensure(c, c->d_H, sizeof(g2a_t) * nn)) || (rc = ensure(c, c->d_hinf, nn)) ||
      (rc = ensure(c, c->d_rs, sizeof(g2p_t) * nn)) || (rc = ensure(c, c->d_fset, sizeof(fp12_t) * nn)) ||
      (rc = ensure(c, c->d_dst, 256)))
    return rc;
  hipStream_t S = c->stream;
  LSG_HIP(c, hipMemcpyAsync(c->d_sig.p, sig.data(), sig.size(), hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_siglen.p, siglen.data(), 4 * n, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_msg.p, msg.data(), msg.size(), hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_msgoff.p, msgoff.data(), 4 * n, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_msglen.p, msglen.data(), 4 * n, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_pk.p, pk.data(), pk.size(), hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_pklen.p, pklen.data(), 4 * np, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_pkoff.p, pkoff.data(), 4 * n, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_pkcnt.p, pkcnt.data(), 4 * n, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_rnd.p, rnd.data(), 8 * n, hipMemcpyHostToDevice, S));
  LSG_HIP(c, hipMemcpyAsync(c->d_dst.p, DST_POP, DST_POP_LEN, hipMemcpyHostToDevice, S));
  // host copies must outlive the async copies: synchronize before the vectors die
  LSG_HIP(c, hipStreamSynchronize(S));
  return LSG_OK;
}

// Per-set stages (everything that does not depend on the grouping).
int run_set_stages(lsg_ctx* c, const Staged& st) {
  int n = (int)st.n_sets, np = (int)st.n_pks;
  if (n == 0) return LSG_OK;
  LAUNCH(c, k_sig_decode, blocks(n), n, P_<uint8_t>(c->d_sig), P_<uint32_t>(c->d_siglen), P_<g2a_t>(c->d_sigaff),
         P_<uint8_t>(c->d_siginf), P_<int32_t>(c->d_seterr));
  LAUNCH(c, k_sig_subgroup, blocks(n), n, P_<g2a_t>(c->d_sigaff), P_<uint8_t>(c->d_siginf), P_<int32_t>(c->d_seterr));
  if (np > 0)
    LAUNCH(c, k_pk_decode, blocks(np), np, P_<uint8_t>(c->d_pk), P_<uint32_t>(c->d_pklen), P_<g1a_t>(c->d_pkaff),
           P_<uint8_t>(c->d_pkinf), P_<int32_t>(c->d_pkerr));
  LAUNCH(c, k_pk_agg_scale, blocks(n), n, P_<uint32_t>(c->d_pkoff), P_<uint32_t>(c->d_pkcnt), P_<g1a_t>(c->d_pkaff),
         P_<uint8_t>(c->d_pkinf), P_<uint64_t>(c->d_rnd), P_<g1a_t>(c->d_P), P_<uint8_t>(c->d_pinf));
  LAUNCH(c, k_hash_to_g2, blocks(n), n, P_<uint8_t>(c->d_msg), P_<uint32_t>(c->d_msgoff), P_<uint32_t>(c->d_msglen),
         P_<uint8_t>(c->d_dst), DST_POP_LEN, P_<g2a_t>(c->d_H), P_<uint8_t>(c->d_hinf));
  LAUNCH(c, k_sig_scale, blocks(n), n, P_<g2a_t>(c->d_sigaff), P_<uint8_t>(c->d_siginf), P_<int32_t>(c->d_seterr),
         P_<uint64_t>(c->d_rnd), P_<g2p_t>(c->d_rs));
  LAUNCH(c, k_miller_sets, blocks(n), n, P_<g1a_t>(c->d_P), P_<uint8_t>(c->d_pinf), P_<g2a_t>(c->d_H),
         P_<uint8_t>(c->d_hinf), P_<int32_t>(c->d_seterr), P_<fp12_t>(c->d_fset));
  return LSG_OK;
}

// Evaluate groups of set indices: verdict[g] = FE(ML(-G1, S_g) prod f_i) == 1.
// If out_F != null the un-exponentiated products are returned instead (no FE).
int run_groups(lsg_ctx* c, const std::vector<std::vector<uint32_t>>& groups, std::vector<int32_t>& verdict,
               fp12_t* out_F_host) {
  int ng = (int)groups.size();
  verdict.assign(ng, 0);
  if (ng == 0) return LSG_OK;
  std::vector<uint32_t> goff(ng + 1), members;
  for (int g = 0; g < ng; g++) {
    goff[g] = (uint32_t)members.size();
    members.insert(members.end(), groups[g].begin(), groups[g].end());
  }
  goff[ng] = (uint32_t)members.size();
  int rc;
  if ((rc = ensure(c, c->d_goff, 4 * (ng + 1))) || (rc = ensure(c, c->d_members, 4 * std::max(members.size(), (size_t)1))) ||
      (rc = ensure(c, c->d_S, sizeof(g2a_t) * ng)) || (rc = ensure(c, c->d_sinf, ng)) ||
      (rc = ensure(c, c->d_fgrp, sizeof(fp12_t) * ng)) || (rc = ensure(c, c->d_F, sizeof(fp12_t) * ng)) ||
      (rc = ensure(c, c->d_verdict, 4 * ng)))
    return rc;
  hipStream_t S = c->stream;
  LSG_HIP(c, hipMemcpyAsync(c->d_goff.p, goff.data(), 4 * (ng + 1), hipMemcpyHostToDevice, S));
  if (!members.empty())
    LSG_HIP(c, hipMemcpyAsync(c->d_members.p, members.data(), 4 * members.size(), hipMemcpyHostToDevice, S));
  LAUNCH(c, k_group_sum, blocks(ng), ng, P_<uint32_t>(c->d_goff), P_<uint32_t>(c->d_members), P_<g2p_t>(c->d_rs),
         P_<g2a_t>(c->d_S), P_<uint8_t>(c->d_sinf));
  LAUNCH(c, k_miller_groups, blocks(ng), ng, P_<g2a_t>(c->d_S), P_<uint8_t>(c->d_sinf), P_<fp12_t>(c->d_fgrp));
  LAUNCH(c, k_group_product, blocks(ng), ng, P_<uint32_t>(c->d_goff), P_<uint32_t>(c->d_members),
         P_<fp12_t>(c->d_fset), P_<fp12_t>(c->d_fgrp), P_<fp12_t>(c->d_F));
  if (out_F_host) {
    LSG_HIP(c, hipMemcpyAsync(out_F_host, c->d_F.p, sizeof(fp12_t) * ng, hipMemcpyDeviceToHost, S));
    LSG_HIP(c, hipStreamSynchronize(S));
    return LSG_OK;
  }
  LAUNCH(c, k_final_exp_check, blocks(ng), ng, P_<fp12_t>(c->d_F), P_<int32_t>(c->d_verdict));
  LSG_HIP(c, hipMemcpyAsync(verdict.data(), c->d_verdict.p, 4 * ng, hipMemcpyDeviceToHost, S));
  LSG_HIP(c, hipStreamSynchronize(S));
  return LSG_OK;
}

struct SetStatus {
  std::vector<int32_t> err;    // per set: BLST code (0 ok)
  std::vector<uint8_t> pinf;   // per set: aggregated pk is infinity
  std::vector<int32_t> pkerr;  // per pubkey
};

int read_status(lsg_ctx* c, const Staged& st, SetStatus& ss) {
  size_t n = st.n_sets, np = st.n_pks;
  ss.err.assign(n, 0);
  ss.pinf.assign(n, 0);
  ss.pkerr.assign(np, 0);
  hipStream_t S = c->stream;
  if (n) {
    LSG_HIP(c, hipMemcpyAsync(ss.err.data(), c->d_seterr.p, 4 * n, hipMemcpyDeviceToHost, S));
    LSG_HIP(c, hipMemcpyAsync(ss.pinf.data(), c->d_pinf.p, n, hipMemcpyDeviceToHost, S));
  }
  if (np) LSG_HIP(c, hipMemcpyAsync(ss.pkerr.data(), c->d_pkerr.p, 4 * np, hipMemcpyDeviceToHost, S));
  LSG_HIP(c, hipStreamSynchronize(S));
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

// Error a job's maybeBatch call would throw, in the reference's order:
// Signature.fromBytes over all sets first (maybeBatch.ts:17-26 map), then
// mul_n_aggregate rejecting an infinite public key (BLST_PK_IS_INFINITY).
int32_t job_error(const SetStatus& ss, size_t first, size_t count) {
  if (count == 0) return LSG_ERR_EMPTY_SET;
  for (size_t k = 0; k < count; k++)
    if (ss.err[first + k]) return ss.err[first + k];
  for (size_t k = 0; k < count; k++)
    if (ss.pinf[first + k]) return LSG_BLST_PK_IS_INFINITY;
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
  if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return LSG_ERR_DEVICE;
  }
  *out = c;
  return LSG_OK;
}

int lsg_destroy(lsg_ctx* c) {
  if (!c) return LSG_ERR_INVALID_ARG;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  DevBuf* bufs[] = {&c->d_sig,  &c->d_siglen, &c->d_msg,    &c->d_msgoff, &c->d_msglen, &c->d_pk,    &c->d_pklen,
                    &c->d_pkoff, &c->d_pkcnt, &c->d_rnd,    &c->d_sigaff, &c->d_siginf, &c->d_seterr, &c->d_pkaff,
                    &c->d_pkinf, &c->d_pkerr, &c->d_P,      &c->d_pinf,   &c->d_H,      &c->d_hinf,  &c->d_rs,
                    &c->d_fset,  &c->d_goff,  &c->d_members, &c->d_S,     &c->d_sinf,   &c->d_fgrp,  &c->d_F,
                    &c->d_verdict, &c->d_dst, &c->d_blob,   &c->d_probe};
  for (DevBuf* b : bufs)
    if (b->p) (void)hipFree(b->p);
  for (Timer& t : c->timers) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  (void)hipStreamDestroy(c->stream);
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

int lsg_verify_jobs(lsg_ctx* c, const lsg_job* jobs, size_t n_jobs, uint64_t seed, lsg_job_result* results,
                    lsg_stats* stats) {
  if (!c || (n_jobs && (!jobs || !results))) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  lsg_stats stt;
  memset(&stt, 0, sizeof(stt));
  stt.start_ns = now_ns();
  timer_reset(c);
  // flatten
  std::vector<const lsg_set*> flat;
  std::vector<size_t> jfirst(n_jobs), jcount(n_jobs);
  for (size_t j = 0; j < n_jobs; j++) {
    jfirst[j] = flat.size();
    jcount[j] = jobs[j].n_sets;
    for (uint32_t k = 0; k < jobs[j].n_sets; k++) flat.push_back(&jobs[j].sets[k]);
  }
  Staged st;
  int rc = stage_sets(c, flat.data(), flat.size(), seed, true, st);
  if (rc) return rc;
  if ((rc = run_set_stages(c, st))) return rc;
  SetStatus ss;
  if ((rc = read_status(c, st, ss))) return rc;
  // worker.ts:108-114: deserializeSet runs before anything else; a bad pubkey throws
  // out of verifyManySignatureSets and rejects every job of the package.
  int32_t pkfail = 0;
  for (size_t k = 0; k < st.n_pks && !pkfail; k++) pkfail = ss.pkerr[k];
  if (pkfail) {
    for (size_t j = 0; j < n_jobs; j++) results[j] = {LSG_ERROR, pkfail};
    stt.end_ns = now_ns();
    if (stats) *stats = stt;
    return LSG_OK;
  }
  std::vector<size_t> batchable, nonbatch;
  for (size_t j = 0; j < n_jobs; j++) (jobs[j].flags & LSG_JOB_BATCHABLE ? batchable : nonbatch).push_back(j);
  for (size_t j = 0; j < n_jobs; j++) results[j] = {LSG_INVALID, 0};

  // Phase A: batchable chunks (worker.ts:51-86) + non-batchable jobs (worker.ts:88-96)
  std::vector<std::vector<uint32_t>> groups;
  std::vector<std::vector<size_t>> group_jobs;  // jobs covered by a group
  std::vector<bool> group_is_chunk;
  std::vector<size_t> retry;  // jobs to verify individually after a failed chunk
  auto job_group = [&](size_t j) {
    std::vector<uint32_t> m;
    for (size_t k = 0; k < jcount[j]; k++) m.push_back((uint32_t)(jfirst[j] + k));
    return m;
  };
  if (!batchable.empty()) {
    for (auto ch : chunkify(batchable.size(), 16)) {
      std::vector<uint32_t> m;
      bool throws = false;
      size_t nsets = 0;
      // the flattened chunk's maybeBatch call throws on the first bad set / pk infinity / empty
      for (size_t q = ch.first; q < ch.second; q++) {
        size_t j = batchable[q];
        nsets += jcount[j];
        for (size_t k = 0; k < jcount[j]; k++) {
          size_t s = jfirst[j] + k;
          if (ss.err[s] || ss.pinf[s]) throws = true;
          m.push_back((uint32_t)s);
        }
      }
      if (nsets == 0) throws = true;
      std::vector<size_t> js;
      for (size_t q = ch.first; q < ch.second; q++) js.push_back(batchable[q]);
      if (throws) {
        stt.batch_retries++;
        retry.insert(retry.end(), js.begin(), js.end());
      } else {
        groups.push_back(m);
        group_jobs.push_back(js);
        group_is_chunk.push_back(true);
      }
    }
  }
  for (size_t j : nonbatch) {
    int32_t e = job_error(ss, jfirst[j], jcount[j]);
    if (e) {
      results[j] = {LSG_ERROR, e};
    } else {
      groups.push_back(job_group(j));
      group_jobs.push_back({j});
      group_is_chunk.push_back(false);
    }
  }
  std::vector<int32_t> verdict;
  if ((rc = run_groups(c, groups, verdict, nullptr))) return rc;
  stt.n_final_exps += (uint32_t)groups.size();
  for (size_t g = 0; g < groups.size(); g++) {
    if (group_is_chunk[g]) {
      if (verdict[g]) {
        for (size_t j : group_jobs[g]) {
          results[j] = {LSG_VALID, 0};
          stt.batch_sigs_success += (uint32_t)jcount[j];
        }
      } else {
        stt.batch_retries++;
        retry.insert(retry.end(), group_jobs[g].begin(), group_jobs[g].end());
      }
    } else {
      results[group_jobs[g][0]] = {verdict[g] ? LSG_VALID : LSG_INVALID, 0};
    }
  }
  // Phase B: per-job retry of failed chunks
  if (!retry.empty()) {
    std::vector<std::vector<uint32_t>> g2;
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
    if ((rc = run_groups(c, g2, verdict, nullptr))) return rc;
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
  Staged st;
  int rc = stage_sets(c, &sp, 1, 0, false, st);
  if (rc) return rc;
  int np = (int)n;
  LAUNCH(c, k_pk_decode, blocks(np), np, P_<uint8_t>(c->d_pk), P_<uint32_t>(c->d_pklen), P_<g1a_t>(c->d_pkaff),
         P_<uint8_t>(c->d_pkinf), P_<int32_t>(c->d_pkerr));
  LAUNCH(c, k_pk_agg_scale, 1, 1, P_<uint32_t>(c->d_pkoff), P_<uint32_t>(c->d_pkcnt), P_<g1a_t>(c->d_pkaff),
         P_<uint8_t>(c->d_pkinf), P_<uint64_t>(c->d_rnd), P_<g1a_t>(c->d_P), P_<uint8_t>(c->d_pinf));
  if ((rc = ensure(c, c->d_blob, 192))) return rc;
  LAUNCH(c, k_g1_to_bytes, 1, 1, P_<g1a_t>(c->d_P), P_<uint8_t>(c->d_pinf), P_<uint8_t>(c->d_blob));
  std::vector<int32_t> pkerr(n);
  LSG_HIP(c, hipMemcpyAsync(pkerr.data(), c->d_pkerr.p, 4 * n, hipMemcpyDeviceToHost, c->stream));
  LSG_HIP(c, hipMemcpyAsync(out96, c->d_blob.p, 96, hipMemcpyDeviceToHost, c->stream));
  LSG_HIP(c, hipStreamSynchronize(c->stream));
  for (size_t k = 0; k < n; k++)
    if (pkerr[k]) {
      *err_code = pkerr[k];
      break;
    }
  return LSG_OK;
}

int lsg_hash_to_g2(lsg_ctx* c, const uint8_t* msgs, uint32_t msg_len, size_t n, const uint8_t* dst,
                   uint32_t dst_len, uint8_t* out192) {
  if (!c || !out192 || (n && msg_len && !msgs) || dst_len > 255 || (dst_len && !dst)) return LSG_ERR_INVALID_ARG;
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
  Staged st;
  int rc = stage_sets(c, sp.data(), n, 0, false, st);
  if (rc) return rc;
  LSG_HIP(c, hipMemcpyAsync(c->d_dst.p, dst, dst_len, hipMemcpyHostToDevice, c->stream));
  int nn = (int)n;
  LAUNCH(c, k_hash_to_g2, blocks(nn), nn, P_<uint8_t>(c->d_msg), P_<uint32_t>(c->d_msgoff), P_<uint32_t>(c->d_msglen),
         P_<uint8_t>(c->d_dst), dst_len, P_<g2a_t>(c->d_H), P_<uint8_t>(c->d_hinf));
  if ((rc = ensure(c, c->d_blob, 192 * n))) return rc;
  LAUNCH(c, k_g2_to_bytes, blocks(nn), nn, P_<g2a_t>(c->d_H), P_<uint8_t>(c->d_hinf), P_<uint8_t>(c->d_blob));
  LSG_HIP(c, hipMemcpyAsync(out192, c->d_blob.p, 192 * n, hipMemcpyDeviceToHost, c->stream));
  LSG_HIP(c, hipStreamSynchronize(c->stream));
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
  Staged st;
  int rc = stage_sets(c, sp.data(), n, 0, false, st);
  if (rc) return rc;
  int nn = (int)n;
  LAUNCH(c, k_sig_decode, blocks(nn), nn, P_<uint8_t>(c->d_sig), P_<uint32_t>(c->d_siglen), P_<g2a_t>(c->d_sigaff),
         P_<uint8_t>(c->d_siginf), P_<int32_t>(c->d_seterr));
  LAUNCH(c, k_sig_subgroup, blocks(nn), nn, P_<g2a_t>(c->d_sigaff), P_<uint8_t>(c->d_siginf), P_<int32_t>(c->d_seterr));
  if ((rc = ensure(c, c->d_blob, 192 * n))) return rc;
  LAUNCH(c, k_g2_to_bytes, blocks(nn), nn, P_<g2a_t>(c->d_sigaff), P_<uint8_t>(c->d_siginf), P_<uint8_t>(c->d_blob));
  LSG_HIP(c, hipMemcpyAsync(out192, c->d_blob.p, 192 * n, hipMemcpyDeviceToHost, c->stream));
  LSG_HIP(c, hipMemcpyAsync(err, c->d_seterr.p, 4 * n, hipMemcpyDeviceToHost, c->stream));
  LSG_HIP(c, hipStreamSynchronize(c->stream));
  return LSG_OK;
}

int lsg_batch_partial(lsg_ctx* c, const lsg_set* sets, size_t n_sets, uint64_t seed, uint8_t* out576,
                      int32_t* set_err, int32_t* any_error) {
  if (!c || !out576 || !any_error || (n_sets && !sets)) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  timer_reset(c);
  std::vector<const lsg_set*> sp(n_sets);
  for (size_t i = 0; i < n_sets; i++) sp[i] = &sets[i];
  Staged st;
  int rc = stage_sets(c, sp.data(), n_sets, seed, true, st);
  if (rc) return rc;
  if ((rc = run_set_stages(c, st))) return rc;
  SetStatus ss;
  if ((rc = read_status(c, st, ss))) return rc;
  *any_error = 0;
  for (size_t i = 0; i < n_sets; i++) {
    int32_t e = ss.err[i] ? ss.err[i] : (ss.pinf[i] ? LSG_BLST_PK_IS_INFINITY : 0);
    if (set_err) set_err[i] = e;
    if (e) *any_error = 1;
  }
  for (size_t k = 0; k < st.n_pks; k++)
    if (ss.pkerr[k]) *any_error = 1;
  std::vector<std::vector<uint32_t>> groups(1);
  for (size_t i = 0; i < n_sets; i++)
    if (!(set_err ? set_err[i] : 0)) groups[0].push_back((uint32_t)i);
  std::vector<int32_t> verdict;
  fp12_t F;
  if ((rc = run_groups(c, groups, verdict, &F))) return rc;
  if ((rc = ensure(c, c->d_blob, 576))) return rc;
  LAUNCH(c, k_fp12_to_canon, 1, P_<fp12_t>(c->d_F), P_<uint8_t>(c->d_blob));
  LSG_HIP(c, hipMemcpyAsync(out576, c->d_blob.p, 576, hipMemcpyDeviceToHost, c->stream));
  LSG_HIP(c, hipStreamSynchronize(c->stream));
  return LSG_OK;
}

int lsg_final_verify(lsg_ctx* c, const uint8_t* partials576, size_t n_partials, int32_t* valid) {
  if (!c || !valid || (n_partials && !partials576)) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  timer_reset(c);
  int rc;
  if ((rc = ensure(c, c->d_blob, 576 * std::max(n_partials, (size_t)1))) || (rc = ensure(c, c->d_F, sizeof(fp12_t))) ||
      (rc = ensure(c, c->d_verdict, 4)))
    return rc;
  LSG_HIP(c, hipMemcpyAsync(c->d_blob.p, partials576, 576 * n_partials, hipMemcpyHostToDevice, c->stream));
  LAUNCH(c, k_partials_product, 1, (int)n_partials, P_<uint8_t>(c->d_blob), P_<fp12_t>(c->d_F));
  LAUNCH(c, k_final_exp_check, 1, 1, P_<fp12_t>(c->d_F), P_<int32_t>(c->d_verdict));
  LSG_HIP(c, hipMemcpyAsync(valid, c->d_verdict.p, 4, hipMemcpyDeviceToHost, c->stream));
  LSG_HIP(c, hipStreamSynchronize(c->stream));
  return LSG_OK;
}

int lsg_probe_fp_mul_rate(lsg_ctx* c, double* fp_mul_per_s, double* mad_per_s) {
  if (!c || !fp_mul_per_s || !mad_per_s) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  LSG_HIP(c, hipSetDevice(c->device));
  hipDeviceProp_t prop;
  LSG_HIP(c, hipGetDeviceProperties(&prop, c->device));
  int threads = prop.multiProcessorCount * 1024;  // 16 waves per CU
  int rc;
  if ((rc = ensure(c, c->d_probe, sizeof(fp_t) * (threads + 4)))) return rc;
  std::vector<fp_t> init(threads + 4);
  for (size_t i = 0; i < init.size(); i++) {
    init[i] = FP_ONE;
    init[i].l[0] ^= (uint32_t)i;
  }
  LSG_HIP(c, hipMemcpy(c->d_probe.p, init.data(), sizeof(fp_t) * init.size(), hipMemcpyHostToDevice));
  const int iters = 256;
  hipLaunchKernelGGL(k_probe_fp_mul, dim3(threads / 256), dim3(256), 0, c->stream, 8, P_<fp_t>(c->d_probe));
  hipEvent_t a, b;
  LSG_HIP(c, hipEventCreate(&a));
  LSG_HIP(c, hipEventCreate(&b));
  LSG_HIP(c, hipEventRecord(a, c->stream));
  hipLaunchKernelGGL(k_probe_fp_mul, dim3(threads / 256), dim3(256), 0, c->stream, iters, P_<fp_t>(c->d_probe));
  LSG_HIP(c, hipEventRecord(b, c->stream));
  LSG_HIP(c, hipEventSynchronize(b));
  float ms = 0;
  LSG_HIP(c, hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  double muls = (double)threads * iters * 4.0;
  *fp_mul_per_s = muls / (ms * 1e-3);
  *mad_per_s = *fp_mul_per_s * 300.0;
  return LSG_OK;
}

int lsg_last_kernel_times(lsg_ctx* c, const char** names, double* ms, int max) {
  if (!c) return 0;
  (void)hipStreamSynchronize(c->stream);
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
