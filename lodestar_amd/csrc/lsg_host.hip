// lsg_host.hip -- host orchestration and the C ABI (include/lodestar_bls.h) of the MI355X
// BLS12-381 signature-set verifier.  No kernels live here (they are in lsg_k_*.hip and
// lsg_serial.hip, reached through lsg_launch.h / lsg_serial.h).
//
// Reference path replaced (file:line under /root/reference):
//   packages/beacon-node/src/chain/bls/multithread/worker.ts:30-114  verifyManySignatureSets,
//       deserializeSet: batch-of-jobs verification with the per-job retry fallback
//   packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39         RLC batch vs single verify
//   packages/beacon-node/src/chain/bls/utils.ts:5-26               pubkey aggregation
//   + the un-vendored @chainsafe/blst@0.2.8 arithmetic underneath.
//
// One package (BlsWorkReq[]: the jobs one worker would get) runs as ONE ticket:
//   phase A (submit, no host synchronisation): every batchable set of the package is one RLC
//     group (bucket MSM for its signature sum), every non-batchable job its own group; each
//     group gets its Miller product and one final exponentiation, launched speculatively.
//   resolve (wait): the reference's verdict rules (worker.ts:51-96).  A passing package
//     group answers every batchable job at once; only when it fails are the 16-job chunks of
//     worker.ts (phase B) and then the jobs of failing chunks (phase C) checked, on the
//     per-set values still resident, so per-job verdicts and the batch_retries /
//     batch_sigs_success counters are the reference's.
// Per device a context owns LSG_SLOTS pipeline slots (two streams each, all buffers
// preallocated by lsg_reserve); several devices share one ticket (whole jobs per device, one
// all-gather of the 576-byte partials, one node final exponentiation: SURVEY.md 8e).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <errno.h>
#include <string.h>
#include <sys/random.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <chrono>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <unordered_map>
#include <string>
#include <vector>

#include "../../include/lodestar_bls.h"
#include "lsg_launch.h"
#include "lsg_layout.h"
#include "lsg_serial.h"
#include "lsg_ab.h"

using namespace lsgl;

namespace {

const uint8_t DST_POP[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
const uint32_t DST_POP_LEN = 43;
constexpr int LSG_SLOTS = 64;      // packages in flight per device (created on first use)
#ifndef LSG_DEFAULT_HW_QUEUES
#define LSG_DEFAULT_HW_QUEUES "16"  // GPU_MAX_HW_QUEUES when the process sets none (lsg_init_devices)
#endif
constexpr int LSG_FINALS = 64;     // final-exponentiation entries in flight (lsg_final_*)
constexpr int LSG_FE_STREAMS = 8;  // streams the final-exponentiation entries share
constexpr int LSG_MAX_DEVICES = 16;
constexpr int LSG_MILLER_KMAX = 4;

uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);  // process.hrtime's clock (the Node host's metrics)
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// OS CSPRNG bytes (getrandom(2)); false if the kernel cannot provide them.  There is no
// deterministic fallback: predictable RLC multipliers would let forged sets cancel.
bool os_random(void* buf, size_t len) {
  uint8_t* p = (uint8_t*)buf;
  while (len) {
    ssize_t r = getrandom(p, len, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += r;
    len -= (size_t)r;
  }
  return true;
}

std::atomic<uint64_t> g_allocs{0};  // device + pinned allocations made (lsg_allocation_count)

// env LSG_TRACE_HOST=1: one stderr line per phase-A submission with its host time per stage
// (staging, planning, per-set launches, group launches), to find host-bound workloads
bool trace_host() {
  static const bool on = [] {
    const char* e = getenv("LSG_TRACE_HOST");
    return e && e[0] == '1';
  }();
  return on;
}

// env LSG_TRACE_ALLOC=1: one stderr line per allocation (size and caller), for steady-state checks
void trace_alloc(const char* kind, size_t bytes) {
  const char* e = getenv("LSG_TRACE_ALLOC");  // read per allocation: allocations are rare
  const bool on = e && atoi(e) != 0;
  if (on) fprintf(stderr, "[lsg alloc] %s %zu bytes\n", kind, bytes);
  (void)on;
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};
struct HostBuf {  // pinned host memory (async copies)
  void* p = nullptr;
  size_t cap = 0;
};
struct Timer {
  const char* name;
  hipEvent_t a, b;
};

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


// ---- segmented-reduction plans (lsgk::seg_reduce): int32 words appended to a slot's plan
// arena, uploaded once per phase
struct SegPass {
  int ips_log2 = 0, n_chunks = 0;
  size_t chunk_off = 0;  // words into the arena
  int src = 0;           // 0: the reduction's input, 1/2: tmp buffer A/B
  int tmp_out = 1;       // tmp buffer (1/2) that negative outputs go to
};
struct SegPlan {
  int op = 0;
  bool has_idx = false;
  size_t idx_off = 0;
  std::vector<SegPass> passes;
  size_t tmp_items = 0;  // per tmp buffer
};
constexpr int SEG_FOLD = 16;  // at most this many serial folds per lane pair within one pass
// Fp12 products (op 2) cost ~50 us each on one lane pair: their passes fold at most 4 terms
// per pair before the butterfly (an 8193-term package product: 17 serial products in two
// passes instead of 28)
constexpr int SEG_FOLD_FP12 = 4;
// work-bound passes (>= SEG_WIDE_PAIRS lane pairs at a wave's 32 pairs per segment): up to 64
// folds per pair
constexpr int SEG_FOLD_WIDE = 64;
constexpr size_t SEG_WIDE_PAIRS = 131072;

// lane pairs per chunk (log2): enough that the longest segment fits one chunk of SEG_FOLD
// folds per pair (one pass), and at least a quarter of the mean length (latency: folds are
// serial, the butterfly is log2(ips) steps); at most a wave's 32 pairs
int ips_for(double avg, int32_t max_len, int fold) {
  int l = 0;
  while (l < 5 && ((int32_t)(fold << l) < max_len || (double)(2 << l) * 4.0 <= avg)) l++;
  return l;
}

// Segments s = 0..ns-1: elements [seg_off[s], seg_off[s] + seg_len[s]) of the idx list (at
// idx_off in the arena; has_idx) or of the input itself; result s goes to dst[dst_base + s].
SegPlan plan_seg(std::vector<int32_t>& A, int op, const std::vector<int32_t>& seg_off,
                 const std::vector<int32_t>& seg_len, bool has_idx, size_t idx_off, int32_t dst_base) {
  SegPlan P;
  P.op = op;
  P.has_idx = has_idx;
  P.idx_off = idx_off;
  const size_t ns = seg_len.size();
  if (ns == 0) return P;
  size_t total = 0;
  for (int32_t l : seg_len) total += (size_t)l;
  // pending: (segment, element offset, length, source) still to reduce
  struct Pend {
    int32_t seg, off, len;
  };
  std::vector<Pend> cur(ns);
  for (size_t s = 0; s < ns; s++) cur[s] = {(int32_t)s, seg_off[s], seg_len[s]};
  double avg = (double)total / (double)ns;
  int src = 0, tmp_out = 1;
  while (!cur.empty()) {
    SegPass pass;
    int32_t max_len = 0;
    for (const Pend& p : cur) max_len = std::max(max_len, p.len);
    int fold = op == 2 ? SEG_FOLD_FP12 : SEG_FOLD;
    pass.ips_log2 = ips_for(avg, max_len, fold);
    // many segments (a block body's ~8k aggregations of ~450 keys): the launch is work-bound,
    // and every butterfly level costs each lane pair one operation, so use as few pairs per
    // chunk as keep the chip full, folding up to SEG_FOLD_WIDE terms each
    if (op != 2 && (cur.size() << 5) >= SEG_WIDE_PAIRS) {
      const int wide = (int)lsg_ab_long("LSG_SEG_FOLD_WIDE", SEG_FOLD_WIDE);  // (A/B build)
      int l = 0;
      while (l < pass.ips_log2 && (int32_t)(wide << l) < max_len) l++;
      pass.ips_log2 = l;
      fold = wide;
    }
    pass.src = src;
    pass.tmp_out = tmp_out;
    const int32_t cap = (int32_t)((1 << pass.ips_log2) * fold);
    pass.chunk_off = A.size();
    std::vector<Pend> nxt;
    int32_t t = 0;
    size_t nxt_total = 0;
    for (const Pend& p : cur) {
      if (p.len <= cap) {
        A.push_back(p.off);
        A.push_back(p.len);
        A.push_back(dst_base + p.seg);
        pass.n_chunks++;
      } else {
        const int32_t first = t;
        for (int32_t o = 0; o < p.len; o += cap) {
          A.push_back(p.off + o);
          A.push_back(std::min(cap, p.len - o));
          A.push_back(-(t + 1));
          t++;
          pass.n_chunks++;
        }
        nxt.push_back({p.seg, first, t - first});
        nxt_total += (size_t)(t - first);
      }
    }
    P.tmp_items = std::max(P.tmp_items, (size_t)t);
    P.passes.push_back(pass);
    avg = nxt.empty() ? 1.0 : (double)nxt_total / (double)nxt.size();
    cur.swap(nxt);
    src = tmp_out;  // the next pass reads this pass's partial results, contiguously
    tmp_out = tmp_out == 1 ? 2 : 1;
  }
  return P;
}

}  // namespace

// ---------------------------------------------------------------------------- state
namespace {

enum SlotKind {
  SLOT_FREE = 0,
  SLOT_JOBS = 1,
  SLOT_STAGING = 2, /* reserved by a submission staging it with the context lock released */
  SLOT_FINAL = 3,
  SLOT_MERGE = 4 /* tickets of coalesced packages */
};

// a small package held for a coalesced launch (lsg_set_coalesce): the caller's jobs, sets
// and bytes copied, so the caller's buffers are free once lsg_submit_jobs returns
struct PendingPkg {
  uint64_t serial = 0, seed = 0;
  size_t n_sets = 0;
  std::vector<lsg_job> jobs;
  std::vector<lsg_set> sets;
  std::vector<uint8_t> data;
};
struct MergeTicket {
  int slot = -1;  // -1: not launched yet
  int sub = -1;
  int rc = 0;       // != 0: its coalesced launch failed (the wait reports rc and err)
  std::string err;
};

struct Dev;

// One RLC group: sets [first, first + len) (a contiguous range: the package group, one
// non-batchable job, one 16-job chunk or one job).
struct Grp {
  size_t first = 0, len = 0;
  bool msm = false;
};

// ---- group stages of one phase (no host synchronisation).  Groups with msm sum their
// signatures by the bucket MSM over the unscaled points in d_rs (MSM groups must come first);
// the rest sum the scaled points in rs.  Then per group ML(-G1, S_g) on a row, the product
// with the group's Miller items (fall: items [0, n_items) followed by one slot per group),
// the canonical product F_g (d_Fb, D2H into h_blob when export), and FE(F_g) into d_verdict.
struct PhasePlan {
  std::vector<Grp> groups;
  size_t n_msm = 0;
  SegPlan buckets, bits, sums, prod;
  size_t n_items = 0;   // Miller items of the phase's groups (fall slots 0 .. n_items-1)
  size_t item_off = 0;  // item_first / item_cnt in the plan arena
  size_t term_base = 0;  // fall slot of group g's ML(-G1, S_g) term: term_base + g
  // per group, optional set sub-ranges items must not cross (the package group's 16-job
  // chunks); sub_items = the item range of every sub-range, in order
  std::vector<std::vector<std::pair<size_t, size_t>>> sub;
  std::vector<std::pair<int32_t, int32_t>> sub_items;
  // reuse: the groups' products take their items from an earlier phase (given item ranges)
  bool reuse_items = false;
  std::vector<std::pair<int32_t, int32_t>> given;
  // host copy of the items (first set, set count): phase C's item-aligned job groups
  std::vector<int32_t> it_first, it_cnt;
  bool single_items = false;  // every item is one set: the list form of the Miller loop runs
  // one Miller pair per distinct message for group agg_g (>= 0): its items are the n_magg
  // message items (plan arena at magg_off) after the n_set_items per-set items
  int agg_g = -1;
  size_t n_magg = 0, magg_off = 0, n_set_items = 0;
};

// PublicKey.aggregate as the batch-affine pairwise tree (lsg_k_pk.hip k_agg_*, lsg_launch.h
// AggTreeArgs): L levels, T items per lane pair, n_c0 level-0 lane pairs, N0 level-0 points;
// plan arena offsets of the per-block set map, the per-set (o0, len, pk0) and k_agg_final's
// per-set sources
constexpr int64_t LSG_ITEMS_PER_BLOCK_HOST = 128;  // lane pairs per block (lsg_kcommon.hpp)
struct AggPlan {
  bool tree = false;
  int L = 0, T = 1;
  int64_t n_c0 = 0, N0 = 0;
  size_t blk_off = 0, o0_off = 0, len_off = 0, pk0_off = 0, src_off = 0;
};
constexpr size_t AGG_TREE_MIN_KEYS = 32768;  // smaller packages: the serial fold + butterfly

struct JobRec {
  size_t first = 0, count = 0;  // staged set range
  uint32_t flags = 0;
};

struct Slot {
  Dev* d = nullptr;
  int index = 0;
  hipStream_t st[2] = {nullptr, nullptr};  // [0] main, [1] side
  bool own_streams = true;
  // the slot's high-priority stream pair (created on first use): a package carrying an
  // LSG_JOB_PRIORITY job runs on it, so its kernels are dispatched ahead of the packages in
  // flight (verifyOnMainThread's latency under load)
  hipStream_t st_norm[2] = {nullptr, nullptr}, st_prio[2] = {nullptr, nullptr};
  int cur = 0;
  hipEvent_t ev_xp = nullptr;  // the exported partial's copy is complete (lsg_jobs_partial*)
  hipEvent_t ev_in = nullptr, ev_sig = nullptr, ev_grp = nullptr, ev_part = nullptr, ev_done = nullptr,
             ev_node = nullptr;
  // inputs (device copies of the pinned staging arena)
  DevBuf d_sig, d_siglen, d_msg, d_msgoff, d_msglen, d_pk, d_pklen, d_rnd, d_mode, d_dst;
  HostBuf h_arena;
  size_t n_sets = 0, n_pks = 0;
  std::vector<uint32_t> pk_cnt, pk_first;
  std::vector<uint64_t> rnd;
  // distinct messages of the staged package: set i hashes message msg_id[i] (n_msgs of them);
  // msg_dedup when some sets share one (a committee's attestations sign one AttestationData)
  size_t n_msgs = 0;
  bool msg_dedup = false;
  std::vector<uint32_t> mtab, mfirst;
  std::vector<uint64_t> mkey;
  std::vector<uint32_t> msg_id;  // host copy of the set -> message map (msg_dedup)
  SegPlan msum;                  // msg_agg: per message, the masked scaled keys of the package group
  DevBuf d_mmask, d_PmP, d_Pm, d_pinfm, d_errm;
  bool single_keys = false;  // every set has exactly one key (key i is set i's)
  uint32_t pk_stride = 96;   // bytes per key slot in d_pk: 4 when every key is a table index
  // per-set state
  DevBuf d_ub, d_sigaff, d_siginf, d_seterr, d_pkp, d_pkerr, d_agg, d_P, d_pinf, d_H, d_hinf, d_rs, d_rs2, d_fall,
      d_fall2;
  DevBuf d_Pp, d_zP, d_zPi, d_U, d_nrm, d_nrmi, d_Hp, d_zN, d_zNi, d_mid, d_Hm, d_hinfm;
  DevBuf binv_lv[2], binv_iv[2];
  DevBuf d_lines;
  bool rs2_ready = false;
  std::vector<uint8_t> rs2_scaled;  // per set: [r_i] sig_i is in d_rs2 (fallback phases share it)
  std::vector<uint8_t> rs_raw;      // per set: d_rs holds the unscaled point (a phase-A MSM group's)
  // groups
  DevBuf d_S, d_F, d_verdict, d_Sb, d_fgb, d_Fb, d_bkt, d_bits, d_aux, d_gath, d_nodeF, d_nodeV;
  DevBuf seg_tmp[3][2];  // reduction scratch per use: [0] pubkeys, [1] signature sums, [2] Fp12 products
  // plan arena
  std::vector<int32_t> plan;
  HostBuf h_plan;
  DevBuf d_plan;
  PhasePlan phA;   // phase A: the package group + non-batchable jobs
  SegPlan pkagg;   // pubkey aggregation of multi-key sets (small packages)
  AggPlan agg;     // ... and as the batch-affine tree (large packages)
  DevBuf d_agga, d_aggi, d_aggpre, d_aggtot, d_aggflag;
  SegPlan phA_node;  // device 0 of a multi-device ticket: product of the gathered partials
  HostBuf h_mode;  // per-set sig_prep modes of a phase
  // pinned result mirrors
  HostBuf h_err, h_pinf, h_pkerr, h_verdict, h_blob, h_nodeV;
  std::vector<Timer> timers;
  size_t ntimers = 0;
  // ticket state
  int kind = SLOT_FREE;
  uint64_t serial = 0;
  std::vector<JobRec> jobs;         // this device's share of the package, caller order
  std::vector<size_t> job_ids;      // caller job index of jobs[k]
  std::vector<size_t> batch_order;  // indices into jobs: batchable jobs in staging order
  size_t nb_sets = 0;               // sets of the batchable jobs (staged first)
  std::vector<Grp> groups;          // phase-A groups (MSM groups first)
  int big_g = -1;                   // the package group's index in groups
  int K = 4;                        // Miller pairs per item for this package
  std::vector<std::pair<int32_t, int32_t>> chunk_items;  // package mode: per chunk, its phase-A items
  bool chunk_mode = false;          // phase A ran one group per 16-job chunk (LSG_PACKAGE_GROUP=0)
  std::vector<int> chunk_group;     // chunk mode: per chunk of batch_order, its phase-A group
  std::vector<int> sub_big;         // a coalesced launch: per sub-package, its package group (-1: none)
  std::vector<int> job_group;       // per job: its phase-A group (non-batchable), else -1
  // the non-batchable jobs' merged group (-1: one group per job) and, per job, its phase-A
  // items (the merged group's items never cross a job: a failing merged group is localised
  // per job over them)
  int nb_g = -1;
  std::vector<std::pair<int32_t, int32_t>> nb_items;
  std::vector<lsg_job_result> results;
  lsg_stats stats;
  bool has_node = false;  // this slot computed the node check (device 0 of a multi-device ticket)
  size_t n_jobs = 0;      // device 0: the ticket's job count
  // the package group is one set verified unscaled (r_i = 0, a plain verify): its partial is
  // raised to a fresh 64-bit randomizer before it leaves the slot (lsg_jobs_partial*)
  bool lone_unscaled = false;
  uint64_t seed = 0;  // the package's randomizer seed (0: OS CSPRNG)
  DevBuf d_xport;
  HostBuf h_xport;
  // multi-device ticket: the package group's final exponentiation was not launched -- the
  // node check over every device's partial decides, and this one runs only if that fails
  bool big_fe_pending = false;
  // coalesced launch (lsg_set_coalesce): n_sub caller packages in one slot.  sub_first: their
  // job-index bounds in the merged job list; bpos_first: their bounds in batch_order.  Each
  // one keeps its own 16-job chunks, deserialisation rule and counters; the slot is freed
  // when every sub-package's ticket has been waited on.
  int n_sub = 0;
  std::vector<size_t> sub_first, bpos_first;
  std::vector<uint64_t> sub_serial;
  std::vector<lsg_stats> sub_stats;
  std::vector<int32_t> sub_pkfail;
  std::vector<uint8_t> sub_done;
  bool resolved = false, resolving = false;
  int resolve_rc = LSG_OK;
};

struct Dev {
  lsg_ctx* c = nullptr;
  int device = 0;
  int ord = 0;  // position in the context's device list
  hipStream_t s_util = nullptr;
  hipStream_t s_fe[LSG_FE_STREAMS] = {};
  // the node protocol's streams at the greatest priority, created on first use (idle
  // high-priority streams cost the packages hardware-queue concurrency: firehose 2.87M ->
  // ~2.4M sets/s with nine of them created up front): partial exports, node final exps
  hipStream_t s_xp = nullptr, s_nfe = nullptr;
  hipStream_t s_pp[2] = {nullptr, nullptr};  // priority packages (slot_streams), on first use
  Slot slots[LSG_SLOTS];
  Slot finals[LSG_FINALS];
  Slot util;
  // validator pubkey table (lsg_pubkey_table_set): projective lane-form keys + validity bytes
  DevBuf d_pktab, d_pktab_ok;
  size_t pktab_n = 0, pktab_cap = 0;
  // kernel times of the last package / call completed on this device (lsg_last_kernel_times),
  // read from the slot's timing events when it completed, before the slot can be reused
  std::vector<std::pair<const char*, float>> last_times;
};

}  // namespace

struct lsg_ctx {
  std::mutex mu;
  std::condition_variable cv;  // waiters of a coalesced slot being resolved by another thread
  std::string err;
  // Packages are staged with `mu` released (submit_pkg): `tab_mu` keeps the validator pubkey
  // table they read from changing meanwhile (shared while staging, exclusive in
  // lsg_pubkey_table_set, always taken before `mu`), `xmu` orders the RCCL exchanges of
  // packages staged at the same time, `staging` counts the submissions in flight.
  std::shared_mutex tab_mu;
  std::mutex xmu;
  int staging = 0;
  // coalescing (lsg_set_coalesce): packages of <= co_max_sets sets wait in `pending` while
  // co_inflight launches are on the device, then go out as one launch
  uint32_t co_max_sets = 0;
  int co_inflight = 2;
  size_t co_max_pending = 16384;
  std::vector<PendingPkg> pending;
  size_t pending_sets = 0;
  std::unordered_map<uint64_t, MergeTicket> merged;
  int n_dev = 0;
  Dev* dev[LSG_MAX_DEVICES] = {};
  bool rccl = false;  // several distinct devices: the partials are all-gathered over RCCL
  ncclComm_t comm[LSG_MAX_DEVICES] = {};
  uint64_t next_serial = 1;
};

namespace {

// A thread staging a package without the context lock reports its errors here; the
// submitter copies them into c->err once it holds the lock again (submit_pkg).
thread_local std::string* t_err_sink = nullptr;
void set_err(lsg_ctx* c, std::string m) {
  if (t_err_sink)
    *t_err_sink = std::move(m);
  else
    c->err = std::move(m);
}

int fail_c(lsg_ctx* c, const char* what, hipError_t e) {
  set_err(c, std::string(what) + ": " + hipGetErrorString(e));
  return LSG_ERR_DEVICE;
}
int fail(Slot* s, const char* what, hipError_t e) { return fail_c(s->d->c, what, e); }

#define LSG_HIP(s, call)                               \
  do {                                                 \
    hipError_t _e = (call);                            \
    if (_e != hipSuccess) return fail((s), #call, _e); \
  } while (0)
#define LSG_HIPC(c, call)                                \
  do {                                                   \
    hipError_t _e = (call);                              \
    if (_e != hipSuccess) return fail_c((c), #call, _e); \
  } while (0)
#define LSG_RC(call)         \
  do {                       \
    int _rc = (call);        \
    if (_rc) return _rc;     \
  } while (0)

int ensure(Slot* s, DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 64;
  if (b.cap >= bytes) return LSG_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t cap = std::max(bytes + bytes / 4, (size_t)4096);
  hipError_t e = hipMalloc(&b.p, cap);
  if (e != hipSuccess) return fail(s, "hipMalloc", e);
  g_allocs++;
  trace_alloc("device", cap);
  b.cap = cap;
  return LSG_OK;
}

int ensure_host(Slot* s, HostBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 64;
  if (b.cap >= bytes) return LSG_OK;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t cap = std::max(bytes + bytes / 4, (size_t)4096);
  hipError_t e = hipHostMalloc(&b.p, cap, hipHostMallocDefault);
  if (e != hipSuccess) return fail(s, "hipHostMalloc", e);
  g_allocs++;
  trace_alloc("pinned", cap);
  b.cap = cap;
  return LSG_OK;
}

void free_dev(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}
void free_host(HostBuf& b) {
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}

template <class T>
T* P_(const DevBuf& b) {
  return (T*)b.p;
}
template <class T>
T* H_(const HostBuf& b) {
  return (T*)b.p;
}

inline hipStream_t S_(Slot* s) { return s->st[s->cur]; }

void timer_reset(Slot* s) {
  s->ntimers = 0;
  s->cur = 0;
}
void timer_begin(Slot* s, const char* name) {
  if (s->ntimers >= s->timers.size()) {
    Timer t;
    (void)hipEventCreate(&t.a);
    (void)hipEventCreate(&t.b);
    s->timers.push_back(t);
  }
  Timer& t = s->timers[s->ntimers];
  t.name = name;
  (void)hipEventRecord(t.a, S_(s));
}
void timer_end(Slot* s) {
  (void)hipEventRecord(s->timers[s->ntimers].b, S_(s));
  s->ntimers++;
}

// a launch through lsg_launch.h on the slot's current stream, timed with HIP events
#define KL(s, name, call)                                 \
  do {                                                    \
    timer_begin((s), name);                               \
    hipError_t _le = (call);                              \
    timer_end((s));                                       \
    if (_le != hipSuccess) return fail((s), name, _le);   \
  } while (0)

// device pointer of arena word `off`
inline const int32_t* PL(Slot* s, size_t off) { return P_<int32_t>(s->d_plan) + off; }

// snapshot a completed slot's kernel times for lsg_last_kernel_times (-1: not measured)
void keep_times(Slot* s) {
  auto& v = s->d->last_times;
  v.clear();
  for (size_t i = 0; i < s->ntimers; i++) {
    float t = 0;
    if (hipEventElapsedTime(&t, s->timers[i].a, s->timers[i].b) != hipSuccess) t = -1;
    v.push_back({s->timers[i].name, t});
  }
}

// a greatest-priority stream of the device, created on first use
int prio_stream(lsg_ctx* c, Dev* d, hipStream_t* st) {
  if (!*st) {
    int least = 0, greatest = 0;
    LSG_HIPC(c, hipSetDevice(d->device));
    LSG_HIPC(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
    LSG_HIPC(c, hipStreamCreateWithPriority(st, hipStreamNonBlocking, greatest));
  }
  return LSG_OK;
}

// Host wait for a completion event without holding a core: hipEventSynchronize spins on this
// stack (with hipEventBlockingSync too: the gossip bench's 64 waiter threads kept 16 cores
// busy, tools/thread_cpu.py), so poll -- back to back for the first 20 us, then with 30 us
// sleeps; the added latency is well under 0.1 ms per wait.
hipError_t event_wait(hipEvent_t e) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t r = hipEventQuery(e);
    if (r != hipErrorNotReady) return r;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(20))
      std::this_thread::sleep_for(std::chrono::microseconds(30));
  }
}

// LSG_BLOCKING_WAITS=1: waiters sleep on the completion events (hipEventBlockingSync)
bool blocking_waits() {
  const char* e = getenv("LSG_BLOCKING_WAITS");
  return e && atoi(e) != 0;
}

int slot_create(Dev* d, Slot* s, int index, hipStream_t shared) {
  s->d = d;
  s->index = index;
  if (shared) {
    s->st[0] = s->st[1] = shared;
    s->own_streams = false;
  } else {
    for (int k = 0; k < 2; k++) LSG_HIP(s, hipStreamCreateWithFlags(&s->st_norm[k], hipStreamNonBlocking));
    s->st[0] = s->st_norm[0];
    s->st[1] = s->st_norm[1];
  }
  hipEvent_t* evs[] = {&s->ev_in, &s->ev_sig, &s->ev_grp, &s->ev_part, &s->ev_done, &s->ev_node, &s->ev_xp};
  for (hipEvent_t* e : evs) LSG_HIP(s, hipEventCreateWithFlags(e, hipEventDisableTiming));
  if (blocking_waits()) {  // the events a waiter blocks on: sleep instead of spinning
    for (hipEvent_t* e : {&s->ev_part, &s->ev_done}) {
      LSG_HIP(s, hipEventDestroy(*e));
      LSG_HIP(s, hipEventCreateWithFlags(e, hipEventDisableTiming | hipEventBlockingSync));
    }
  }
  LSG_RC(ensure(s, s->d_dst, 256));
  LSG_HIP(s, hipMemcpy(s->d_dst.p, DST_POP, DST_POP_LEN, hipMemcpyHostToDevice));
  return LSG_OK;
}

void slot_destroy(Slot* s) {
  if (!s->d) return;
  for (int k = 0; k < 2; k++)
    if (s->st[k]) (void)hipStreamSynchronize(s->st[k]);
  DevBuf* bufs[] = {&s->d_sig,  &s->d_siglen, &s->d_msg,  &s->d_msgoff, &s->d_msglen, &s->d_pk,    &s->d_pklen,
                    &s->d_rnd,  &s->d_mode,   &s->d_dst,  &s->d_ub,     &s->d_sigaff, &s->d_siginf, &s->d_seterr,
                    &s->d_pkp,  &s->d_pkerr,  &s->d_agg,  &s->d_P,      &s->d_pinf,   &s->d_H,     &s->d_hinf,
                    &s->d_rs,   &s->d_rs2,    &s->d_fall, &s->d_fall2,  &s->d_Pp,     &s->d_zP,    &s->d_zPi,
                    &s->d_U,    &s->d_nrm,    &s->d_nrmi, &s->d_Hp,     &s->d_zN,     &s->d_zNi,   &s->binv_lv[0],
                    &s->binv_lv[1], &s->binv_iv[0], &s->binv_iv[1], &s->d_lines, &s->d_S, &s->d_F, &s->d_verdict,
                    &s->d_Sb,   &s->d_fgb,    &s->d_Fb,   &s->d_bkt,    &s->d_bits,   &s->d_aux,   &s->d_gath,
                    &s->d_nodeF, &s->d_nodeV, &s->d_plan, &s->d_mid, &s->d_Hm, &s->d_hinfm,
                    &s->d_mmask, &s->d_PmP, &s->d_Pm, &s->d_pinfm, &s->d_errm, &s->d_xport,
                    &s->d_agga, &s->d_aggi, &s->d_aggpre, &s->d_aggtot, &s->d_aggflag};
  for (DevBuf* b : bufs) free_dev(*b);
  for (auto& u : s->seg_tmp)
    for (DevBuf& b : u) free_dev(b);
  HostBuf* hb[] = {&s->h_arena, &s->h_err, &s->h_pinf, &s->h_pkerr, &s->h_verdict, &s->h_blob, &s->h_plan, &s->h_nodeV,
                   &s->h_xport};
  for (HostBuf* b : hb) free_host(*b);
  for (Timer& t : s->timers) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  s->timers.clear();
  hipEvent_t evs[] = {s->ev_in, s->ev_sig, s->ev_grp, s->ev_part, s->ev_done, s->ev_node, s->ev_xp};
  for (hipEvent_t e : evs)
    if (e) (void)hipEventDestroy(e);
  if (s->own_streams) {
    for (int k = 0; k < 2; k++) {
      if (s->st_prio[k]) (void)hipStreamSynchronize(s->st_prio[k]);
      if (s->st_norm[k]) (void)hipStreamSynchronize(s->st_norm[k]);
    }
    for (int k = 0; k < 2; k++) {
      if (s->st_norm[k]) (void)hipStreamDestroy(s->st_norm[k]);
      // (st_prio: the device's shared pair, destroyed with the device)
      s->st_norm[k] = s->st_prio[k] = s->st[k] = nullptr;
    }
  }
  s->d = nullptr;
}

// select the slot's stream pair for its next package (the slot is free: nothing of an
// earlier package is in flight on either pair)
int slot_streams(Slot* s, bool prio) {
  if (!s->own_streams) return LSG_OK;
  // priority packages share one pair of greatest-priority streams per device, created on
  // first use: a pair per slot would leave idle high-priority streams behind that take
  // hardware-queue concurrency from every later package
  if (prio && !s->st_prio[0]) {
    Dev* d = s->d;
    for (int k = 0; k < 2; k++) LSG_RC(prio_stream(d->c, d, &d->s_pp[k]));
    s->st_prio[0] = d->s_pp[0];
    s->st_prio[1] = d->s_pp[1];
  }
  hipStream_t* p = prio ? s->st_prio : s->st_norm;
  s->st[0] = p[0];
  s->st[1] = p[1];
  return LSG_OK;
}

// the pipeline slot `s` of device `d`, created on first use
int slot_ready(Dev* d, Slot* s, int index) {
  if (s->d) return LSG_OK;
  const int rc = slot_create(d, s, index, nullptr);
  if (rc) slot_destroy(s);
  return rc;
}

// the 16-job chunks (worker.ts:51) of the slot's batchable jobs as batch_order positions:
// over the whole package, or per sub-package of a coalesced launch (never across two)
std::vector<std::pair<size_t, size_t>> slot_chunks(const Slot* s) {
  if (s->n_sub == 0) return chunkify(s->batch_order.size(), 16);
  std::vector<std::pair<size_t, size_t>> out;
  for (int k = 0; k < s->n_sub; k++) {
    const size_t a = s->bpos_first[k], b = s->bpos_first[k + 1];
    if (b == a) continue;
    for (auto& c : chunkify(b - a, 16)) out.push_back({a + c.first, a + c.second});
  }
  return out;
}
// sub-package of a batch_order position / of a job (coalesced launches; 0 otherwise)
int sub_of_pos(const Slot* s, size_t q) {
  if (s->n_sub == 0) return 0;
  return (int)(std::upper_bound(s->bpos_first.begin(), s->bpos_first.end(), q) - s->bpos_first.begin()) - 1;
}
int sub_of_job(const Slot* s, size_t j) {
  if (s->n_sub == 0) return 0;
  return (int)(std::upper_bound(s->sub_first.begin(), s->sub_first.end(), j) - s->sub_first.begin()) - 1;
}

// ---- sizes
// Miller pairs per item (one shared f and its squarings): K = 4 does the least work per set,
// but one item is one lane pair, so a small package has few items and its accumulation wave
// runs alone for ~14 ms; smaller K trades work for latency there.  Env LSG_MILLER_K forces K.
// The fused Miller kernel (k_miller_fused: lines in LDS, four waves per item of four pairs) is
// the default; LSG_MILLER_FUSED=0 selects the split pair k_miller_lines / k_miller_accum<K>.
bool miller_fused() { return lsg_ab_long("LSG_MILLER_FUSED", 1) != 0; }

size_t slp_items_max();
int miller_k_for(size_t n_sets) {
  if (miller_fused()) return n_sets <= slp_items_max() ? 1 : 4;  // fused: four waves' lane pairs per item
  const long v = lsg_ab_long("LSG_MILLER_K", 0);
  if (v == 1 || v == 2 || v == 4) return (int)v;
  return n_sets >= 8192 ? 4 : (n_sets >= 1024 ? 2 : 1);
}

// PublicKey.aggregate of large packages as the batch-affine tree: A/B build only
// (LSG_AGG_TREE=1).  Measured slower than the fused gather + mixed-addition fold
// (k_pk_agg_seg) on config C: 2.7 ms against 1.44 ms for a 3.7M-key block package alone,
// 0.90M against 0.98M sets/s loaded -- the per-level inversion, heap and
// point round trips cost more than the four products per key the affine additions save.
bool agg_tree_on() { return lsg_ab_long("LSG_AGG_TREE", 0) != 0; }

// Minimum RLC group size for the bucket MSM (A/B build: env LSG_MSM_MIN_GROUP).  By operation
// count the MSM wins from ~4 sets (2-bit windows: ~24 bucket additions plus 4 of the group's 64
// bit sums, ~1k Fp products, against ~2.25k for a 64-bit scalar multiplication; the group's
// Horner program ~4k more), but the per-set [r_i] sig_i kernel runs near 0.3 of the mad peak
// and the bucket and bit-sum reductions far below it, plus a Horner program per group: on
// config C (64 groups of 128 sets) 1.05-1.08M sets/s without the MSM against 1.01M with it
// (profiles/r04_msm_ab.txt).  The MSM stays for groups of 256 and more (8-bit windows: the
// firehose's package group, the fallback phases' halves).
size_t msm_min_group() {
  const long x = lsg_ab_long("LSG_MSM_MIN_GROUP", 256);
  return x < 1 ? (size_t)1 : (size_t)x;
}
// Window width c of a group's bucket MSM (plan_phase): per set 64/c digits (bucket
// additions), per group the 64 bit sums over 2^(c-1) buckets each.  n sets cost about
// n (64/c) + 2^(c-1) 64 G2 additions: c = 2 below 48 sets, 4 below 256, 8 from there.
int msm_window_bits(size_t n) { return n >= 256 ? 8 : (n >= 48 ? 4 : 2); }

// Phase A as the reference batches it: one RLC group per 16-job chunk instead of one package
// group (env LSG_PACKAGE_GROUP=0; A/B and the equivalence test of the two modes)
bool package_group_mode() { return lsg_ab_long("LSG_PACKAGE_GROUP", 1) != 0; }
// A coalesced launch with one package group per sub-package (A/B build: LSG_SUB_GROUPS=0 gives
// round 3's one group per 16-job chunk)
bool sub_groups_on() { return lsg_ab_long("LSG_SUB_GROUPS", 1) != 0; }
// A package's non-batchable jobs (>= 2 of them with sets) verified as ONE RLC group, localised
// per job only when it fails (A/B build: LSG_NB_MERGE=0 gives one group per job).  Each job's
// verdict is its own validity either way (worker.ts:88-96: such a job is verified alone), and
// non-batchable jobs never enter the batch counters.
bool nb_merge_on() { return lsg_ab_long("LSG_NB_MERGE", 1) != 0; }
// Phase B0 (pkg_resolve): with at least this many chunks to check, runs of up to
// LSG_B0_RUN consecutive chunks are checked as one group first (0: off)
size_t b0_min_chunks() { return (size_t)std::max(0L, lsg_ab_long("LSG_B0_MIN", 64)); }
size_t b0_run() { return (size_t)std::max(2L, lsg_ab_long("LSG_B0_RUN", 4)); }

void binv_sizes(size_t n, size_t* lv, size_t* iv);
size_t binv_lv_words(size_t n) {
  size_t a, b;
  binv_sizes(n, &a, &b);
  return a;
}
size_t binv_iv_words(size_t n) {
  size_t a, b;
  binv_sizes(n, &a, &b);
  return b;
}

// inputs for up to n sets / np keys / mb message bytes
int size_inputs(Slot* s, size_t n, size_t np, size_t mb) {
  const size_t nn = std::max(n, (size_t)1), pp = std::max(np, (size_t)1);
  auto al = [](size_t x) { return (x + 7) & ~(size_t)7; };
  const size_t arena = al(192 * nn) + al(4 * nn) * 4 + al(4 * pp) + al(8 * nn) + al(96 * pp) + al(std::max(mb, (size_t)1)) + nn;
  LSG_RC(ensure_host(s, s->h_arena, arena));
  LSG_RC(ensure(s, s->d_sig, 192 * nn));
  LSG_RC(ensure(s, s->d_siglen, 4 * nn));
  LSG_RC(ensure(s, s->d_msg, std::max(mb, (size_t)1)));
  LSG_RC(ensure(s, s->d_msgoff, 4 * nn));
  LSG_RC(ensure(s, s->d_msglen, 4 * nn));
  LSG_RC(ensure(s, s->d_pk, 96 * pp));
  LSG_RC(ensure(s, s->d_pklen, 4 * pp));
  LSG_RC(ensure(s, s->d_rnd, 8 * nn));
  LSG_RC(ensure(s, s->d_mode, nn));
  LSG_RC(ensure(s, s->d_mid, 4 * nn));
  return LSG_OK;
}

// per-set state and group buffers for n sets / np keys / ng groups (n_msm of them bucket-MSM
// groups) in any phase
// pkg: 0 utility calls; 1 phase A of a package (every per-set buffer); 2 a fallback phase
// (only its own buffers: the per-set state of phase A stays resident and is never moved)
int size_state(Slot* s, size_t n, size_t np, size_t ng, size_t n_msm, int pkg = 0) {
  const size_t nn = std::max(n, (size_t)1), pp = std::max(np, (size_t)1), gg = std::max(ng, (size_t)1);
  const size_t g_msm = std::max(n_msm, (size_t)1);
  struct {
    DevBuf* b;
    size_t bytes;
  } dev[] = {{&s->d_ub, 256 * nn},
             {&s->d_sigaff, 4 * W_G2A * nn},
             {&s->d_siginf, nn},
             {&s->d_seterr, 4 * nn},
             {&s->d_pkp, 4 * W_G1P * pp},
             {&s->d_pkerr, 4 * pp},
             {&s->d_agg, 4 * W_G1P * nn},
             {&s->d_P, 4 * W_G1A * nn},
             {&s->d_pinf, nn},
             {&s->d_H, 4 * W_G2A * nn},
             {&s->d_hinf, nn},
             {&s->d_rs, 4 * W_G2P * nn},
             {&s->d_Pp, 4 * W_G1P * nn},
             {&s->d_zP, 4 * W_FP * nn},
             {&s->d_zPi, 4 * W_FP * nn},
             {&s->d_U, 4 * W_H2CU * nn},
             {&s->d_nrm, 4 * W_FP * 2 * nn},
             {&s->d_nrmi, 4 * W_FP * 2 * nn},
             {&s->d_Hp, 4 * W_G2P * nn},
             {&s->d_zN, 4 * W_FP * nn},
             {&s->d_zNi, 4 * W_FP * nn},
             {&s->binv_lv[0], 4 * W_FP * binv_lv_words(2 * nn)},
             {&s->binv_iv[0], 4 * W_FP * binv_iv_words(2 * nn)},
             {&s->binv_lv[1], 4 * W_FP * binv_lv_words(nn)},
             {&s->binv_iv[1], 4 * W_FP * binv_iv_words(nn)},
             {&s->d_S, 4 * W_G2P * gg},
             {&s->d_F, 4 * W_F12 * gg},
             {&s->d_verdict, 4 * gg},
             {&s->d_Sb, (size_t)288 * (MSM_BITS * g_msm + gg)},
             {&s->d_fgb, 576 * gg},
             {&s->d_Fb, 576 * gg},
             {&s->d_bkt, 4 * W_G2P * (size_t)MSM_WINDOWS * MSM_DIGITS * g_msm},
             {&s->d_bits, 4 * W_G2P * (size_t)MSM_BITS * g_msm},
             {&s->d_gath, 576 * (LSG_MAX_DEVICES + 2)},  // partials, the identity, the node product
             {&s->d_nodeF, 4 * W_F12 * (LSG_MAX_DEVICES + 1)},
             {&s->d_nodeV, 64}};
  for (auto& x : dev) LSG_RC(ensure(s, *x.b, x.bytes));
  if (pkg == 1) {  // Miller lines (split kernels only) and items; fall also holds phase B's chunk terms
    if (!miller_fused()) LSG_RC(ensure(s, s->d_lines, 4 * (size_t)ML_STEPS * W_LINE * nn));
    // items, phase A's group terms, then the terms of a reusing phase (phase B's chunks, or
    // phase C's item-aligned job groups: at most one per item)
    LSG_RC(ensure(s, s->d_fall, 4 * W_F12 * (2 * nn + gg + 2)));
  }
  if (pkg) {  // fallback signature sums and Miller items: a phase C of single-set jobs needs
              // one item and one term slot per retried set
    LSG_RC(ensure(s, s->d_fall2, 4 * W_F12 * (nn + std::max(gg, nn))));
    LSG_RC(ensure(s, s->d_rs2, 4 * W_G2P * nn));
  }
  LSG_RC(ensure_host(s, s->h_err, 4 * nn));
  LSG_RC(ensure_host(s, s->h_pinf, nn));
  LSG_RC(ensure_host(s, s->h_pkerr, 4 * pp));
  LSG_RC(ensure_host(s, s->h_verdict, 4 * gg));
  LSG_RC(ensure_host(s, s->h_blob, 576 * gg));
  LSG_RC(ensure_host(s, s->h_nodeV, 64));
  return LSG_OK;
}

// reduction scratch for a plan
int size_seg(Slot* s, int use, const SegPlan& P) {
  if (P.tmp_items == 0) return LSG_OK;
  const size_t W = P.op == 0 ? W_G1P : (P.op == 1 ? W_G2P : W_F12);
  LSG_RC(ensure(s, s->seg_tmp[use][0], 4 * W * P.tmp_items));
  return ensure(s, s->seg_tmp[use][1], 4 * W * P.tmp_items);
}

// upload the plan arena (one copy on the main stream, before ev_in)
int upload_plan(Slot* s) {
  const size_t bytes = 4 * std::max(s->plan.size(), (size_t)1);
  LSG_RC(ensure_host(s, s->h_plan, bytes));
  LSG_RC(ensure(s, s->d_plan, bytes));
  if (!s->plan.empty()) {
    memcpy(s->h_plan.p, s->plan.data(), 4 * s->plan.size());
    LSG_HIP(s, hipMemcpyAsync(s->d_plan.p, s->h_plan.p, 4 * s->plan.size(), hipMemcpyHostToDevice, s->st[0]));
  }
  return LSG_OK;
}

// run a planned reduction on the current stream; use selects the scratch pair
int run_seg(Slot* s, int use, const char* name, const SegPlan& P, const uint32_t* src, uint32_t* dst) {
  LSG_RC(size_seg(s, use, P));
  uint32_t* tmp[3] = {nullptr, P_<uint32_t>(s->seg_tmp[use][0]), P_<uint32_t>(s->seg_tmp[use][1])};
  const int32_t* idx = P.has_idx ? PL(s, P.idx_off) : nullptr;
  for (size_t k = 0; k < P.passes.size(); k++) {
    const SegPass& q = P.passes[k];
    const uint32_t* in = q.src == 0 ? src : tmp[q.src];
    KL(s, name, lsgk::seg_reduce(S_(s), P.op, q.n_chunks, q.ips_log2, PL(s, q.chunk_off), k == 0 ? idx : nullptr, in, dst,
                                 tmp[q.tmp_out]));
  }
  return LSG_OK;
}

// PublicKey.aggregate of the slot's multi-key sets by the segmented reduction, its first pass
// fetching the staged keys itself (lsg_k_pk.hip k_pk_agg_seg; P = plan_pk_agg)
int run_pk_seg(Slot* s, const SegPlan& P, uint32_t* dst) {
  LSG_RC(size_seg(s, 0, P));
  Dev* d = s->d;
  uint32_t* tmp[3] = {nullptr, P_<uint32_t>(s->seg_tmp[0][0]), P_<uint32_t>(s->seg_tmp[0][1])};
  for (size_t k = 0; k < P.passes.size(); k++) {
    const SegPass& q = P.passes[k];
    if (k == 0)
      KL(s, "g1_aggregate", lsgk::pk_agg_seg(S_(s), q.n_chunks, q.ips_log2, PL(s, q.chunk_off), P_<uint8_t>(s->d_pk),
                                             s->pk_stride, P_<uint32_t>(s->d_pklen), P_<int32_t>(s->d_pkerr),
                                             P_<uint32_t>(d->d_pktab), P_<uint8_t>(d->d_pktab_ok), (uint32_t)d->pktab_n,
                                             dst, tmp[q.tmp_out]));
    else
      KL(s, "g1_aggregate", lsgk::seg_reduce(S_(s), 0, q.n_chunks, q.ips_log2, PL(s, q.chunk_off), nullptr,
                                             tmp[q.src], dst, tmp[q.tmp_out]));
  }
  return LSG_OK;
}

// batched inversions in one launch per call (k_binv_block); LSG_BINV_BLOCK=0 (A/B build): the
// multi-level fold / root / unfold launches
static bool binv_block_on() { return lsg_ab_long("LSG_BINV_BLOCK", 1) != 0; }

// Words (per Fp of W_FP) of the two scratch arrays a batched inversion of n values needs:
// lv = every level's prefix products plus levels >= 1's values, iv = levels >= 1's inverses
void binv_sizes(size_t n, size_t* lv, size_t* iv) {
  size_t a = 0, b = 0;
  for (size_t m = n; m > 1;) {
    const size_t up = (m + LSG_BINV_T - 1) / LSG_BINV_T;
    a += m + up;
    b += up;
    m = up;
  }
  *lv = std::max(a, (size_t)1);
  *iv = std::max(b, (size_t)1);
}

// out[i] = 1 / v[i] (0 for v[i] = 0) for n lane-form Fp values on the current stream
// (Montgomery's trick in chunks of LSG_BINV_T per lane pair: lsg_k_reduce.hip)
int batch_inv(Slot* s, int ws, const char* name, const uint32_t* v, size_t n, uint32_t* out) {
  if (n == 0) return LSG_OK;
  size_t lvw, ivw;
  binv_sizes(n, &lvw, &ivw);
  LSG_RC(ensure(s, s->binv_lv[ws], 4 * W_FP * lvw));
  LSG_RC(ensure(s, s->binv_iv[ws], 4 * W_FP * ivw));
  uint32_t* lv = P_<uint32_t>(s->binv_lv[ws]);
  uint32_t* iv = P_<uint32_t>(s->binv_iv[ws]);
  if (binv_block_on()) {  // one launch: a divstep root per block of 128 x T values
    // ~64 blocks: each holds its CU slot through one ~30 us divstep root (and the heap's
    // barriers), so fewer, longer blocks cost the loaded GPU less than one block per 128 values
    // (7 % of summed kernel time with T = 1, profiles/r05_rocprof_stats_a.csv)
    const int T = (int)std::min<size_t>(64, std::max<size_t>(1, (n + 128 * 64 - 1) / (128 * 64)));
    KL(s, name, lsgk::binv_block(S_(s), (int)n, T, 1, v, lv, out));
    return LSG_OK;
  }
  // level l: values val[l] (val[0] = v), prefix products pre[l], inverses inv[l] (inv[0] = out)
  std::vector<size_t> cnt{n};
  std::vector<uint32_t*> val{(uint32_t*)v}, pre, inv{out};
  size_t lo = 0, io = 0;
  while (cnt.back() > 1) {
    const size_t m = cnt.back(), up = (m + LSG_BINV_T - 1) / LSG_BINV_T;
    pre.push_back(lv + W_FP * lo);
    lo += m;
    val.push_back(lv + W_FP * lo);
    lo += up;
    inv.push_back(iv + W_FP * io);
    io += up;
    cnt.push_back(up);
  }
  const size_t L = cnt.size() - 1;
  if (L == 0) {  // one value: invert it directly (0 stays 0)
    KL(s, name, lsgk::binv_root(S_(s), v, out));
    return LSG_OK;
  }
  for (size_t l = 0; l < L; l++)
    KL(s, name, lsgk::binv_fold(S_(s), (int)cnt[l], l == 0 ? 1 : 0, val[l], pre[l], val[l + 1]));
  KL(s, name, lsgk::binv_root(S_(s), val[L], inv[L]));
  for (size_t l = L; l-- > 0;)
    KL(s, name, lsgk::binv_unfold(S_(s), (int)cnt[l], l == 0 ? 1 : 0, val[l], pre[l], inv[l + 1], inv[l]));
  return LSG_OK;
}

// Packages of up to LSG_SLP_ITEMS sets (default 2048; 0: never) run one-set Miller items as
// straight-line programs (lsg_slp.hip, one workgroup per set, ~0.8 ms) instead of the fused
// kernel, whose latency is one full loop per lane whatever the package size (~5.4 ms).
// one Miller pair per distinct message in the package group (LSG_MSG_AGG=0: one per set);
// read per package, so that a test can compare both forms in one process
static bool msg_agg_on() { return lsg_ab_long("LSG_MSG_AGG", 1) != 0; }

size_t slp_items_max() {
  const long v = lsg_ab_long("LSG_SLP_ITEMS", 2048);
  return lsg_serial_mode() == LSG_SERIAL_SLP && v > 0 ? (size_t)v : 0;
}

// hash_to_G2 of the slot's n expanded messages (d_ub) into H / hinf on the current stream
int launch_hash(Slot* s, int n, uint32_t* H, uint8_t* hinf) {
  KL(s, "k_h2c_prep", lsgk::h2c_prep(S_(s), n, P_<uint8_t>(s->d_ub), P_<uint32_t>(s->d_U), P_<uint32_t>(s->d_nrm)));
  LSG_RC(batch_inv(s, 0, "binv_sswu", P_<uint32_t>(s->d_nrm), 2 * (size_t)n, P_<uint32_t>(s->d_nrmi)));
  KL(s, "k_h2c_map", lsgk::h2c_map(S_(s), n, P_<uint32_t>(s->d_U), P_<uint32_t>(s->d_nrmi), P_<uint32_t>(s->d_Hp)));
  if ((size_t)n <= slp_items_max()) {  // small packages: clearing + affine as one program per set
    KL(s, "k_slp_h2c", lsg_slp_h2c_clear(S_(s), n, P_<uint32_t>(s->d_Hp), H, hinf));
    return LSG_OK;
  }
  KL(s, "k_h2c_clear", lsgk::h2c_clear(S_(s), n, P_<uint32_t>(s->d_Hp), P_<uint32_t>(s->d_zN), hinf));
  LSG_RC(batch_inv(s, 0, "binv_hash", P_<uint32_t>(s->d_zN), (size_t)n, P_<uint32_t>(s->d_zNi)));
  KL(s, "k_h2c_affine", lsgk::h2c_affine(S_(s), n, P_<uint32_t>(s->d_Hp), P_<uint32_t>(s->d_zNi), hinf, H));
  return LSG_OK;
}

// ---- staging: the package's sets into the slot's pinned arena (order given by `order`),
// randomizers drawn here (seed == 0: OS CSPRNG; else deterministic, for tests)
// 64-bit mix of a message (its length and 8-byte words; signing roots are SHA-256 outputs)
static uint64_t msg_key(const uint8_t* m, uint32_t len) {
  uint64_t h = 0x9e3779b97f4a7c15ull ^ len;
  uint32_t k = 0;
  for (; k + 8 <= len; k += 8) {
    uint64_t w;
    memcpy(&w, m + k, 8);
    h = (h ^ w) * 0xff51afd7ed558ccdull;
    h ^= h >> 32;
  }
  for (; k < len; k++) h = (h ^ m[k]) * 0x100000001b3ull;
  return h ^ (h >> 29);
}

int stage_sets(Slot* s, const lsg_set* const* sets, size_t n, uint64_t seed, bool scale,
               const std::vector<uint8_t>* noscale = nullptr, bool dedup = false) {
  size_t npk = 0, msg_total = 0;
  bool all_index = true;  // every key names a table row: 4-byte key slots (a block body's
                          // ~3.7M signers cross PCIe as 15 MB instead of 355 MB)
  for (size_t i = 0; i < n; i++) {
    npk += sets[i]->n_pks;
    msg_total += sets[i]->msg_len;
    if (sets[i]->n_pks && sets[i]->pk_len != LSG_PK_INDEX) all_index = false;
  }
  const size_t ks = all_index ? 4 : 96;
  s->pk_stride = (uint32_t)ks;
  s->n_sets = n;
  s->n_pks = npk;
  LSG_RC(size_inputs(s, n, npk, msg_total));
  const size_t nn = std::max(n, (size_t)1), np = std::max(npk, (size_t)1);
  auto al = [](size_t x) { return (x + 7) & ~(size_t)7; };
  const size_t o_sig = 0, o_siglen = al(o_sig + 192 * nn), o_msgoff = al(o_siglen + 4 * nn),
               o_msglen = al(o_msgoff + 4 * nn), o_mid = al(o_msglen + 4 * nn), o_pklen = al(o_mid + 4 * nn),
               o_rnd = al(o_pklen + 4 * np), o_pk = al(o_rnd + 8 * nn), o_msg = al(o_pk + ks * np);
  uint8_t* A = H_<uint8_t>(s->h_arena);
  uint32_t* siglen = (uint32_t*)(A + o_siglen);
  uint32_t* msgoff = (uint32_t*)(A + o_msgoff);
  uint32_t* msglen = (uint32_t*)(A + o_msglen);
  uint32_t* mid = (uint32_t*)(A + o_mid);
  uint32_t* pklen = (uint32_t*)(A + o_pklen);
  uint64_t* rnd = (uint64_t*)(A + o_rnd);
  siglen[0] = msgoff[0] = msglen[0] = pklen[0] = 0;
  rnd[0] = 0;
  s->pk_cnt.resize(n);
  s->pk_first.resize(n);
  s->rnd.resize(n);
  size_t mo = 0, po = 0, nm = 0;
  bool single = npk == n;
  // open-addressing table over the messages: slot -> distinct message id (mfirst: its set),
  // with the message's 64-bit key beside it so that a probe compares bytes only on a key match
  size_t cap = 0;
  static const bool dedup_on = lsg_ab_long("LSG_MSG_DEDUP", 1) != 0;
  // a package whose sample of 256 evenly spaced sets shows no repeated message is taken as all
  // distinct and staged without the table (the firehose of distinct gossip messages pays ~5 us,
  // not the table's ~1 ms under the context lock); committee-shaped packages repeat at once
  auto sample_repeats = [&]() {
    const size_t k = std::min(n, (size_t)256), step = n / k;
    uint64_t seen[512];
    bool used[512] = {false};
    for (size_t j = 0; j < k; j++) {
      const lsg_set* q = sets[j * step];
      const uint64_t key = msg_key(q->msg, q->msg_len);
      for (size_t h = (size_t)key & 511;; h = (h + 1) & 511) {
        if (!used[h]) {
          used[h] = true;
          seen[h] = key;
          break;
        }
        if (seen[h] == key) return true;
      }
    }
    return false;
  };
  if (dedup && dedup_on && n > 1 && sample_repeats()) {
    cap = 16;
    while (cap < 2 * n) cap <<= 1;
    s->mtab.assign(cap, UINT32_MAX);
    s->mkey.resize(cap);
    s->mfirst.resize(n);
  }
  for (size_t i = 0; i < n; i++) {
    const lsg_set* q = sets[i];
    siglen[i] = q->sig_len;
    uint8_t* sg = A + o_sig + 192 * i;
    if ((q->sig_len == 96 || q->sig_len == 192) && q->sig)
      memcpy(sg, q->sig, q->sig_len);
    else
      memset(sg, 0, 96);
    uint32_t id = (uint32_t)nm;
    if (cap) {
      const uint64_t key = msg_key(q->msg, q->msg_len);
      for (size_t h = (size_t)key & (cap - 1);; h = (h + 1) & (cap - 1)) {
        const uint32_t e = s->mtab[h];
        if (e == UINT32_MAX) {
          s->mtab[h] = id;
          s->mkey[h] = key;
          s->mfirst[id] = (uint32_t)i;
          break;
        }
        if (s->mkey[h] != key) continue;
        const lsg_set* r = sets[s->mfirst[e]];
        if (r->msg_len == q->msg_len && (q->msg_len == 0 || memcmp(r->msg, q->msg, q->msg_len) == 0)) {
          id = e;
          break;
        }
      }
    }
    mid[i] = id;
    if (id == nm) {  // a new message: staged once
      msgoff[nm] = (uint32_t)mo;
      msglen[nm] = q->msg_len;
      if (q->msg_len) memcpy(A + o_msg + mo, q->msg, q->msg_len);
      mo += q->msg_len;
      nm++;
    }
    s->pk_cnt[i] = q->n_pks;
    s->pk_first[i] = (uint32_t)po;
    if (q->n_pks != 1) single = false;
    if (all_index) {  // the set's indices are contiguous in the caller's buffer
      std::fill(pklen + po, pklen + po + q->n_pks, (uint32_t)LSG_PK_INDEX);
      if (q->pks)
        memcpy(A + o_pk + 4 * po, q->pks, 4 * (size_t)q->n_pks);
      else
        memset(A + o_pk + 4 * po, 0, 4 * (size_t)q->n_pks);
      po += q->n_pks;
      continue;
    }
    for (uint32_t k = 0; k < q->n_pks; k++) {
      pklen[po] = q->pk_len;
      uint8_t* pd = A + o_pk + 96 * po;
      if ((q->pk_len == 48 || q->pk_len == 96 || q->pk_len == LSG_PK_INDEX) && q->pks)
        memcpy(pd, q->pks + (size_t)q->pk_len * k, q->pk_len);
      else
        memset(pd, 0, 4);
      po++;
    }
  }
  s->single_keys = single && n > 0;
  s->n_msgs = nm;
  s->msg_dedup = nm < n;
  if (s->msg_dedup) s->msg_id.assign(mid, mid + n);
  if (scale && n) {
    if (seed == 0) {
      if (!os_random(rnd, 8 * n)) {
        set_err(s->d->c, "no entropy for the RLC randomizers (getrandom failed)");
        return LSG_ERR_ENTROPY;
      }
      for (size_t i = 0; i < n; i++)
        while (rnd[i] == 0)
          if (!os_random(&rnd[i], 8)) {
            set_err(s->d->c, "no entropy for the RLC randomizers (getrandom failed)");
            return LSG_ERR_ENTROPY;
          }
    } else {
      uint64_t sd = seed;
      for (size_t i = 0; i < n; i++) {
        uint64_t r;
        do r = splitmix64(sd);
        while (r == 0);
        rnd[i] = r;
      }
    }
  } else if (n) {
    memset(rnd, 0, 8 * n);
  }
  // sets that form a group of their own are verified as they are (maybeBatch.ts:34-38: one
  // set is a plain verify): r_i = 0 means "not scaled" to k_pk_scale and k_sig_scale
  if (scale && noscale)
    for (size_t i = 0; i < n; i++)
      if ((*noscale)[i]) rnd[i] = 0;
  memcpy(s->rnd.data(), rnd, 8 * n);
  hipStream_t S = s->st[0];
  struct {
    DevBuf* d;
    size_t off, len;
  } cp[] = {{&s->d_sig, o_sig, 192 * nn},      {&s->d_siglen, o_siglen, 4 * nn}, {&s->d_msg, o_msg, std::max(msg_total, (size_t)1)},
            {&s->d_msgoff, o_msgoff, 4 * nn}, {&s->d_msglen, o_msglen, 4 * nn}, {&s->d_pk, o_pk, ks * np},
            {&s->d_pklen, o_pklen, 4 * np},   {&s->d_rnd, o_rnd, 8 * nn}};
  for (auto& x : cp) LSG_HIP(s, hipMemcpyAsync(x.d->p, A + x.off, x.len, hipMemcpyHostToDevice, S));
  if (s->msg_dedup) LSG_HIP(s, hipMemcpyAsync(s->d_mid.p, A + o_mid, 4 * n, hipMemcpyHostToDevice, S));
  return LSG_OK;
}

// ---- Miller items: <= K consecutive sets of one range (group); item_first / item_cnt go to
// the arena.  Returns the number of items; set_item (optional) maps set -> item.
size_t plan_items(Slot* s, const std::vector<std::pair<size_t, size_t>>& ranges, size_t* off,
                  std::vector<int32_t>* set_item, std::vector<std::pair<int32_t, int32_t>>* range_items,
                  std::vector<int32_t>* host_first = nullptr, std::vector<int32_t>* host_cnt = nullptr) {
  const size_t K = (size_t)s->K;
  std::vector<int32_t> first, cnt;
  for (auto& r : ranges) {
    const int32_t i0 = (int32_t)first.size();
    for (size_t i = r.first; i < r.second; i += K) {
      size_t c = std::min(K, r.second - i);
      if (set_item)
        for (size_t k = 0; k < c; k++) (*set_item)[i + k] = (int32_t)first.size();
      first.push_back((int32_t)i);
      cnt.push_back((int32_t)c);
    }
    if (range_items) range_items->push_back({i0, (int32_t)first.size()});
  }
  *off = s->plan.size();
  s->plan.insert(s->plan.end(), first.begin(), first.end());
  s->plan.insert(s->plan.end(), cnt.begin(), cnt.end());
  if (host_first) *host_first = first;
  if (host_cnt) *host_cnt = cnt;
  return first.size();
}

int plan_phase(Slot* s, PhasePlan& Ph) {
  std::vector<int32_t>& A = s->plan;
  const size_t ng = Ph.groups.size();
  Ph.n_msm = 0;
  while (Ph.n_msm < ng && Ph.groups[Ph.n_msm].msm) Ph.n_msm++;
  // bucket MSM: per MSM group, bucket (w, d) = the sets whose w-th c-bit digit of r_i is d.
  // c = 8 (8 windows x 255 buckets) for large groups; c = 4 (16 x 15) below MSM_C8_MIN sets,
  // where 2040 buckets' bit sums would cost more than the sets' bucket additions (a block's
  // 128-set groups: 16 additions per set + 512 per group instead of a 64-bit scalar
  // multiplication per set).  Buckets are numbered compactly (group bases); bit k = c w + j
  // sums the buckets (w, d) whose digit d has bit j set, so every group has 64 bit sums and
  // one Horner program whatever its c.
  if (Ph.n_msm) {
    std::vector<int> cw(Ph.n_msm);
    std::vector<size_t> gbase(Ph.n_msm + 1, 0);
    for (size_t g = 0; g < Ph.n_msm; g++) {
      cw[g] = msm_window_bits(Ph.groups[g].len);
      gbase[g + 1] = gbase[g] + (size_t)(64 / cw[g]) * (size_t)((1u << cw[g]) - 1);
    }
    auto bucket = [&](size_t g, int w, uint32_t d) { return gbase[g] + (size_t)w * ((1u << cw[g]) - 1) + d - 1; };
    std::vector<int32_t> cnt(gbase[Ph.n_msm], 0);
    for (size_t g = 0; g < Ph.n_msm; g++) {
      const int c = cw[g], nw = 64 / c;
      const uint64_t dm = (1ull << c) - 1;
      for (size_t i = Ph.groups[g].first; i < Ph.groups[g].first + Ph.groups[g].len; i++) {
        const uint64_t r = s->rnd[i];
        for (int w = 0; w < nw; w++) {
          const uint32_t d = (uint32_t)((r >> (c * w)) & dm);
          if (d) cnt[bucket(g, w, d)]++;
        }
      }
    }
    std::vector<int32_t> seg_off(cnt.size()), seg_len(cnt);
    int32_t tot = 0;
    for (size_t b = 0; b < cnt.size(); b++) {
      seg_off[b] = tot;
      tot += cnt[b];
    }
    const size_t idx_off = A.size();
    A.resize(idx_off + (size_t)tot);
    int32_t* idx = A.data() + idx_off;
    std::vector<int32_t> fill(seg_off);
    for (size_t g = 0; g < Ph.n_msm; g++) {
      const int c = cw[g], nw = 64 / c;
      const uint64_t dm = (1ull << c) - 1;
      for (size_t i = Ph.groups[g].first; i < Ph.groups[g].first + Ph.groups[g].len; i++) {
        const uint64_t r = s->rnd[i];
        for (int w = 0; w < nw; w++) {
          const uint32_t d = (uint32_t)((r >> (c * w)) & dm);
          if (d) idx[fill[bucket(g, w, d)]++] = (int32_t)i;
        }
      }
    }
    Ph.buckets = plan_seg(A, 1, seg_off, seg_len, true, idx_off, 0);
    // bit (g, k = c w + j): the buckets (g, w, d) whose digit d has bit j set
    const size_t bidx = A.size();
    std::vector<int32_t> boff, blen;
    for (size_t g = 0; g < Ph.n_msm; g++) {
      const int c = cw[g], nw = 64 / c;
      for (int w = 0; w < nw; w++)
        for (int j = 0; j < c; j++) {
          boff.push_back((int32_t)(A.size() - bidx));
          for (uint32_t d = 1; d < (1u << c); d++)
            if ((d >> j) & 1u) A.push_back((int32_t)bucket(g, w, d));
          blen.push_back((int32_t)(A.size() - bidx) - boff.back());
        }
    }
    Ph.bits = plan_seg(A, 1, boff, blen, true, bidx, 0);
  }
  // scaled groups: S_g = sum of the contiguous scaled points
  if (Ph.n_msm < ng) {
    std::vector<int32_t> off, len;
    for (size_t g = Ph.n_msm; g < ng; g++) {
      off.push_back((int32_t)Ph.groups[g].first);
      len.push_back((int32_t)Ph.groups[g].len);
    }
    Ph.sums = plan_seg(A, 1, off, len, false, 0, (int32_t)Ph.n_msm);
  }
  // Miller items of this phase: <= K consecutive sets, never crossing a group (nor one of its
  // sub-ranges), unless the groups reuse an earlier phase's items
  std::vector<std::pair<int32_t, int32_t>> gi;
  if (Ph.reuse_items) {
    gi = Ph.given;
  } else {
    std::vector<std::pair<size_t, size_t>> ranges;
    std::vector<size_t> nsub(ng, 1);
    for (size_t g = 0; g < ng; g++) {
      if ((int)g == Ph.agg_g) {  // message items instead (below)
        nsub[g] = 0;
      } else if (g < Ph.sub.size() && !Ph.sub[g].empty()) {
        ranges.insert(ranges.end(), Ph.sub[g].begin(), Ph.sub[g].end());
        nsub[g] = Ph.sub[g].size();
      } else {
        ranges.push_back({Ph.groups[g].first, Ph.groups[g].first + Ph.groups[g].len});
      }
    }
    Ph.sub_items.clear();
    Ph.n_items = plan_items(s, ranges, &Ph.item_off, nullptr, &Ph.sub_items, &Ph.it_first, &Ph.it_cnt);
    Ph.single_items = true;
    for (int32_t c : Ph.it_cnt) Ph.single_items = Ph.single_items && c == 1;
    Ph.n_set_items = Ph.n_items;
    if (Ph.agg_g >= 0) {  // item n_set_items + j = message j (one pair)
      Ph.magg_off = A.size();
      for (size_t j = 0; j < Ph.n_magg; j++) A.push_back((int32_t)j);
      for (size_t j = 0; j < Ph.n_magg; j++) A.push_back(1);
      Ph.n_items += Ph.n_magg;
    }
    Ph.term_base = Ph.n_items;
    size_t r = 0;
    for (size_t g = 0; g < ng; g++) {
      if ((int)g == Ph.agg_g) {
        gi.push_back({(int32_t)Ph.n_set_items, (int32_t)Ph.n_items});
        continue;
      }
      gi.push_back({Ph.sub_items[r].first, Ph.sub_items[r + nsub[g] - 1].second});
      r += nsub[g];
    }
  }
  // F_g = f_g * prod of the group's items; element ids index fall
  const size_t pidx = A.size();
  std::vector<int32_t> poff, plen;
  for (size_t g = 0; g < ng; g++) {
    poff.push_back((int32_t)(A.size() - pidx));
    for (int32_t it = gi[g].first; it < gi[g].second; it++) A.push_back(it);
    A.push_back((int32_t)(Ph.term_base + g));
    plen.push_back((int32_t)(A.size() - pidx) - poff.back());
  }
  Ph.prod = plan_seg(A, 2, poff, plen, true, pidx, 0);
  return LSG_OK;
}

// Miller accumulation of planned items (after ev_sig on the main stream)
int launch_accum(Slot* s, size_t n_items, size_t item_off, uint32_t* fall, bool single = false) {
  const int ni = (int)n_items;
  const int32_t* items = PL(s, item_off);
  if (ni > 0 && (single || s->K == 1) && miller_fused() && (size_t)ni <= std::max(slp_items_max(), (size_t)8192) &&
      slp_items_max() > 0) {
    // one-set items (small packages, per-job fallback phases): straight-line programs
    KL(s, "k_slp_items1", lsg_slp_miller_items1(S_(s), ni, items, P_<uint32_t>(s->d_P), P_<uint8_t>(s->d_pinf),
                                                P_<uint8_t>(s->d_hinf), P_<int32_t>(s->d_seterr), P_<uint32_t>(s->d_H),
                                                fall));
    return LSG_OK;
  }
  if (single && ni > 0) {
    // every item is one pair (a fallback phase of single-set jobs): the fused kernel would run
    // four waves per item for one pair; the list form computes each set's lines once and
    // accumulates them alone (item k = set items[k])
    LSG_RC(ensure(s, s->d_lines, 4 * (size_t)ML_STEPS * W_LINE * n_items));
    KL(s, "k_miller_lines_list", lsgk::miller_lines_list(S_(s), ni, items, P_<uint32_t>(s->d_H), P_<uint32_t>(s->d_lines)));
    KL(s, "k_miller_accum_list",
       lsgk::miller_accum_list(S_(s), ni, items, P_<uint32_t>(s->d_P), P_<uint8_t>(s->d_pinf), P_<uint8_t>(s->d_hinf),
                               P_<int32_t>(s->d_seterr), P_<uint32_t>(s->d_lines), fall));
    return LSG_OK;
  }
  if (miller_fused()) {
    KL(s, "k_miller_fused", lsgk::miller_fused(S_(s), ni, items, items + ni, P_<uint32_t>(s->d_P), P_<uint8_t>(s->d_pinf),
                                              P_<uint8_t>(s->d_hinf), P_<int32_t>(s->d_seterr), P_<uint32_t>(s->d_H),
                                              fall));
    return LSG_OK;
  }
  KL(s, "k_miller_accum",
     lsgk::miller_accum(S_(s), s->K, ni, items, items + ni, P_<uint32_t>(s->d_P), P_<uint8_t>(s->d_pinf),
                        P_<uint8_t>(s->d_hinf), P_<int32_t>(s->d_seterr), (int)s->n_sets, P_<uint32_t>(s->d_lines),
                        fall));
  return LSG_OK;
}

// kernel-time label of a serial stage: the straight-line program that runs it (slp_*), or the
// row kernel with LSG_SERIAL=row in the A/B build (k_row_*)
#define SERIAL_LABEL(name) (lsg_serial_mode() == LSG_SERIAL_SLP ? "slp_" #name : "k_row_" #name)

// side stream: signature sums -> ML(-G1, S_g) -> fall slots; main stream: products, export, FE
// rs: the scaled points [r_i] sig_i the plain groups sum; rs_msm: the unscaled points the
// bucket MSM groups read (phase A: one buffer holds both kinds, by set)
int launch_phase(Slot* s, const PhasePlan& Ph, const uint32_t* rs, uint32_t* fall, bool export_blobs,
                 const uint32_t* rs_msm = nullptr) {
  if (!rs_msm) rs_msm = rs;
  const size_t ng = Ph.groups.size();
  if (ng == 0) return LSG_OK;
  LSG_RC(size_state(s, s->n_sets, s->n_pks, ng, Ph.n_msm, 2));
  s->cur = 1;
  if (Ph.n_msm) {
    LSG_RC(run_seg(s, 1, "msm_buckets", Ph.buckets, rs_msm, P_<uint32_t>(s->d_bkt)));
    LSG_RC(run_seg(s, 1, "msm_bits", Ph.bits, P_<uint32_t>(s->d_bkt), P_<uint32_t>(s->d_bits)));
    KL(s, "k_g2p_to_canon", lsgk::g2p_to_canon(S_(s), (int)(MSM_BITS * Ph.n_msm), P_<uint32_t>(s->d_bits),
                                               P_<uint8_t>(s->d_Sb)));
    KL(s, SERIAL_LABEL(horner_miller),
       lsg_row_horner_miller(S_(s), (int)Ph.n_msm, P_<uint8_t>(s->d_Sb), P_<uint8_t>(s->d_fgb)));
  }
  if (Ph.n_msm < ng) {
    const int nsm = (int)(ng - Ph.n_msm);
    LSG_RC(run_seg(s, 1, "sig_sums", Ph.sums, rs, P_<uint32_t>(s->d_S)));
    uint8_t* sb = P_<uint8_t>(s->d_Sb) + (size_t)288 * MSM_BITS * Ph.n_msm;
    KL(s, "k_g2p_to_canon", lsgk::g2p_to_canon(S_(s), nsm, P_<uint32_t>(s->d_S) + W_G2P * Ph.n_msm, sb));
    KL(s, SERIAL_LABEL(miller_neg_g1),
       lsg_row_miller_neg_g1(S_(s), nsm, sb, P_<uint8_t>(s->d_fgb) + 576 * Ph.n_msm));
  }
  KL(s, "k_blobs_to_fp12", lsgk::blobs_to_fp12(S_(s), (int)ng, P_<uint8_t>(s->d_fgb), fall + W_F12 * Ph.term_base));
  LSG_HIP(s, hipEventRecord(s->ev_grp, s->st[1]));
  s->cur = 0;
  LSG_HIP(s, hipStreamWaitEvent(s->st[0], s->ev_grp, 0));
  LSG_RC(run_seg(s, 2, "fp12_product", Ph.prod, fall, P_<uint32_t>(s->d_F)));
  KL(s, "k_fp12_to_canon", lsgk::fp12_to_canon(S_(s), (int)ng, P_<uint32_t>(s->d_F), P_<uint8_t>(s->d_Fb)));
  if (export_blobs) LSG_HIP(s, hipMemcpyAsync(s->h_blob.p, s->d_Fb.p, 576 * ng, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipEventRecord(s->ev_part, s->st[0]));
  return LSG_OK;
}

// FE of the phase's groups g0 .. g1-1 + verdict readback (main stream)
int launch_fe_range(Slot* s, size_t g0, size_t g1) {
  if (g1 <= g0) return LSG_OK;
  s->cur = 0;
  const size_t ng = g1 - g0;
  KL(s, SERIAL_LABEL(final_exp),
     lsg_row_final_exp(S_(s), (int)ng, P_<uint8_t>(s->d_Fb) + 576 * g0, P_<int32_t>(s->d_verdict) + g0));
  LSG_HIP(s, hipMemcpyAsync(H_<int32_t>(s->h_verdict) + g0, P_<int32_t>(s->d_verdict) + g0, 4 * ng,
                            hipMemcpyDeviceToHost, s->st[0]));
  return LSG_OK;
}
int launch_fe(Slot* s, size_t ng) { return launch_fe_range(s, 0, ng); }

int launch_agg_tree(Slot* s, const AggPlan& P, uint32_t* agg);

// Per-set stages of the slot's package (no host synchronisation):
//   side: pubkeys -> aggregation -> [r_i] scaling -> signature decode -> subgroup check (ev_sig)
//   main: expand_message -> hash_to_G2 [-> lines] -> wait ev_sig -> Miller items f (fall)
int launch_set_stages(Slot* s, const SegPlan* pkagg, const PhasePlan& Ph, uint32_t* fall) {
  const size_t n_items = Ph.agg_g >= 0 ? Ph.n_set_items : Ph.n_items, item_off = Ph.item_off;
  const int n = (int)s->n_sets, np = (int)s->n_pks;
  if (n == 0) return LSG_OK;
  Dev* d = s->d;
  LSG_HIP(s, hipEventRecord(s->ev_in, s->st[0]));
  s->cur = 1;
  LSG_HIP(s, hipStreamWaitEvent(s->st[1], s->ev_in, 0));
  if (!s->single_keys && s->agg.tree) {
    LSG_RC(launch_agg_tree(s, s->agg, P_<uint32_t>(s->d_agg)));
  } else if (s->single_keys) {
    // single-key sets decode straight into their aggregate slot
    if (np > 0)
      KL(s, "k_pk_decode", lsgk::pk_decode(S_(s), np, P_<uint8_t>(s->d_pk), s->pk_stride, P_<uint32_t>(s->d_pklen),
                                           P_<uint32_t>(s->d_agg), P_<int32_t>(s->d_pkerr), P_<uint32_t>(d->d_pktab),
                                           P_<uint8_t>(d->d_pktab_ok), (uint32_t)d->pktab_n));
  } else {
    LSG_RC(run_pk_seg(s, *pkagg, P_<uint32_t>(s->d_agg)));  // (every staged key is in one set)
  }
  KL(s, "k_pk_scale", lsgk::pk_scale(S_(s), n, P_<uint32_t>(s->d_agg), P_<uint64_t>(s->d_rnd), P_<uint32_t>(s->d_Pp),
                                     P_<uint32_t>(s->d_zP), P_<uint8_t>(s->d_pinf)));
  LSG_RC(batch_inv(s, 1, "binv_pk", P_<uint32_t>(s->d_zP), (size_t)n, P_<uint32_t>(s->d_zPi)));
  KL(s, "k_pk_affine", lsgk::pk_affine(S_(s), n, P_<uint32_t>(s->d_Pp), P_<uint32_t>(s->d_zPi), P_<uint32_t>(s->d_P)));
  KL(s, "k_sig_decode", lsgk::sig_decode(S_(s), n, P_<uint8_t>(s->d_sig), P_<uint32_t>(s->d_siglen),
                                         P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf), P_<int32_t>(s->d_seterr)));
  if ((size_t)n <= slp_items_max())  // small packages: one program per set (0.3 ms, not 1.3)
    KL(s, "k_slp_subgroup", lsg_slp_g2_subgroup(S_(s), n, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf),
                                                P_<int32_t>(s->d_seterr)));
  else
    KL(s, "k_sig_subgroup", lsgk::sig_subgroup(S_(s), n, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf),
                                               P_<int32_t>(s->d_seterr)));
  if (Ph.agg_g >= 0) {  // per message: sum of the package group's usable r_i pk_i, affine
    const Grp& g = Ph.groups[(size_t)Ph.agg_g];
    const size_t nm = Ph.n_magg;
    LSG_RC(ensure(s, s->d_mmask, 4 * W_G1P * std::max(g.first + g.len, (size_t)1)));
    LSG_RC(ensure(s, s->d_PmP, 4 * W_G1P * nm));
    LSG_RC(ensure(s, s->d_Pm, 4 * W_G1A * nm));
    LSG_RC(ensure(s, s->d_pinfm, nm));
    LSG_RC(ensure(s, s->d_errm, 4 * nm));
    KL(s, "k_pk_mask", lsgk::pk_mask(S_(s), (int)(g.first + g.len), P_<uint32_t>(s->d_Pp), P_<int32_t>(s->d_seterr),
                                     P_<uint8_t>(s->d_pinf), P_<uint32_t>(s->d_mmask)));
    LSG_RC(run_seg(s, 0, "msg_pk_sums", s->msum, P_<uint32_t>(s->d_mmask), P_<uint32_t>(s->d_PmP)));
    KL(s, "k_g1p_affine_inv", lsgk::g1p_affine_inv(S_(s), (int)nm, P_<uint32_t>(s->d_PmP), P_<uint32_t>(s->d_Pm),
                                                   P_<uint8_t>(s->d_pinfm)));
    LSG_HIP(s, hipMemsetAsync(s->d_errm.p, 0, 4 * nm, s->st[1]));
  }
  LSG_HIP(s, hipEventRecord(s->ev_sig, s->st[1]));
  s->cur = 0;
  // hash_to_G2 once per distinct message, then each set's point gathered from its message's
  const int nm = (int)s->n_msgs;
  KL(s, "k_expand_msg", lsgk::expand_msg(S_(s), nm, P_<uint8_t>(s->d_msg), P_<uint32_t>(s->d_msgoff),
                                         P_<uint32_t>(s->d_msglen), P_<uint8_t>(s->d_dst), DST_POP_LEN,
                                         P_<uint8_t>(s->d_ub)));
  if (s->msg_dedup) {
    LSG_RC(ensure(s, s->d_Hm, 4 * W_G2A * (size_t)nm));
    LSG_RC(ensure(s, s->d_hinfm, (size_t)nm));
    LSG_RC(launch_hash(s, nm, P_<uint32_t>(s->d_Hm), P_<uint8_t>(s->d_hinfm)));
    KL(s, "k_h2c_gather", lsgk::h2c_gather(S_(s), n, P_<uint32_t>(s->d_mid), P_<uint32_t>(s->d_Hm),
                                           P_<uint8_t>(s->d_hinfm), P_<uint32_t>(s->d_H), P_<uint8_t>(s->d_hinf)));
  } else {
    LSG_RC(launch_hash(s, n, P_<uint32_t>(s->d_H), P_<uint8_t>(s->d_hinf)));
  }
  if (!miller_fused())
    KL(s, "k_miller_lines", lsgk::miller_lines(S_(s), n, P_<uint32_t>(s->d_H), P_<uint32_t>(s->d_lines)));
  LSG_HIP(s, hipStreamWaitEvent(s->st[0], s->ev_sig, 0));
  if (n_items) LSG_RC(launch_accum(s, n_items, item_off, fall));
  if (Ph.agg_g >= 0)  // one pair per message: (sum of r_i pk_i, H(m)), one program each
    KL(s, "k_slp_items_msg",
       lsg_slp_miller_items1(S_(s), (int)Ph.n_magg, PL(s, Ph.magg_off), P_<uint32_t>(s->d_Pm), P_<uint8_t>(s->d_pinfm),
                             P_<uint8_t>(s->d_hinfm), P_<int32_t>(s->d_errm), P_<uint32_t>(s->d_Hm),
                             fall + (size_t)lsgl::W_F12 * Ph.n_set_items));
  return LSG_OK;
}

// pubkey aggregation plan (sets with several keys): segment i = keys pk_first[i] ..
SegPlan plan_pk_agg(Slot* s) {
  std::vector<int32_t> off(s->n_sets), len(s->n_sets);
  for (size_t i = 0; i < s->n_sets; i++) {
    off[i] = (int32_t)s->pk_first[i];
    len[i] = (int32_t)s->pk_cnt[i];
  }
  return plan_seg(s->plan, 0, off, len, false, 0, 0);
}

// The batch-affine tree's plan for the slot's sets (keys of set i: pk_first[i] .. + pk_cnt[i]).
// L is chosen by cost: a tree set of n keys costs ~7 products per level-0 point (padded to
// 2^L: one fold product, five in the step, a share of the heaps) plus 11 per complete mixed
// addition of its ceil(n / 2^L) level-L points; a set the tree would not make cheaper (few
// keys, or padding too large) is summed from its keys directly by k_agg_final.
AggPlan plan_agg_tree(Slot* s) {
  AggPlan P;
  P.tree = true;
  const size_t n = s->n_sets;
  auto tree_cost = [](int64_t len, int L) {
    const int64_t A = (int64_t)1 << L;
    return ((len + A - 1) / A) * A * 7 + ((len + A - 1) / A) * 11;
  };
  int64_t best = -1;
  for (int L = 0; L <= 9; L++) {
    int64_t cost = 0;
    for (size_t i = 0; i < n; i++) {
      const int64_t len = (int64_t)s->pk_cnt[i];
      cost += L > 0 ? std::min(tree_cost(len, L), len * 11) : len * 11;
    }
    if (best < 0 || cost < best) {
      best = cost;
      P.L = L;
    }
  }
  const int64_t A = (int64_t)1 << P.L;
  P.T = (int)std::max<long>(1, std::min<long>(64, lsg_ab_long("LSG_AGG_T", 8)));
  std::vector<int32_t> o0(n, 0), src(3 * n);
  int64_t N0 = 0;
  for (size_t i = 0; i < n; i++) {
    const int64_t len = (int64_t)s->pk_cnt[i];
    if (P.L > 0 && tree_cost(len, P.L) < len * 11) {
      o0[i] = (int32_t)N0;
      src[3 * i] = 0;
      src[3 * i + 1] = (int32_t)(N0 >> P.L);
      src[3 * i + 2] = (int32_t)((len + A - 1) / A);
      N0 += (len + A - 1) / A * A;
    } else {
      src[3 * i] = 1;
      src[3 * i + 1] = (int32_t)s->pk_first[i];
      src[3 * i + 2] = (int32_t)len;
    }
  }
  P.N0 = N0;
  if (N0 == 0) P.L = 0;
  if (P.L > 0) {
    // lane pairs: a multiple of 128 << (L - 1), so that every level's grid is whole blocks
    const int64_t unit = (int64_t)LSG_ITEMS_PER_BLOCK_HOST << (P.L - 1);
    const int64_t need = (N0 / 2 + P.T - 1) / P.T;
    P.n_c0 = (need + unit - 1) / unit * unit;
    P.blk_off = s->plan.size();
    s->plan.resize(P.blk_off + (size_t)(N0 >> P.L));
    int32_t* blk = s->plan.data() + P.blk_off;
    for (size_t i = 0; i < n; i++)
      if (src[3 * i] == 0)
        for (int32_t b = src[3 * i + 1], e = b + src[3 * i + 2]; b < e; b++) blk[b] = (int32_t)i;
  }
  P.o0_off = s->plan.size();
  s->plan.insert(s->plan.end(), o0.begin(), o0.end());
  P.len_off = s->plan.size();
  for (size_t i = 0; i < n; i++) s->plan.push_back((int32_t)s->pk_cnt[i]);
  P.pk0_off = s->plan.size();
  for (size_t i = 0; i < n; i++) s->plan.push_back((int32_t)s->pk_first[i]);
  P.src_off = s->plan.size();
  s->plan.insert(s->plan.end(), src.begin(), src.end());
  return P;
}

// the tree over the staged keys into d_agg (side stream: after the inputs' upload)
int launch_agg_tree(Slot* s, const AggPlan& P, uint32_t* agg) {
  Dev* d = s->d;
  lsgk::AggTreeArgs a;
  a.L = P.L;
  a.T = P.T;
  a.n_c0 = P.n_c0;
  a.N0 = P.N0;
  a.blk_set = PL(s, P.blk_off);
  a.set_o0 = PL(s, P.o0_off);
  a.set_len = PL(s, P.len_off);
  a.set_pk0 = PL(s, P.pk0_off);
  a.pk = P_<uint8_t>(s->d_pk);
  a.stride = s->pk_stride;
  a.pk_len = P_<uint32_t>(s->d_pklen);
  a.pk_err = P_<int32_t>(s->d_pkerr);
  a.tab = P_<uint32_t>(d->d_pktab);
  a.tab_ok = P_<uint8_t>(d->d_pktab_ok);
  a.tab_n = (uint32_t)d->pktab_n;
  if (P.L > 0) {
    const size_t npts = (size_t)(2 * P.N0), pre_w = W_FP * (size_t)(P.T * P.n_c0), cinv_w = W_FP * (size_t)P.n_c0;
    LSG_RC(ensure(s, s->d_agga, 4 * W_G1A * npts));
    LSG_RC(ensure(s, s->d_aggi, npts));
    LSG_RC(ensure(s, s->d_aggpre, 4 * 2 * pre_w));
    LSG_RC(ensure(s, s->d_aggtot, 4 * 2 * cinv_w));
    LSG_RC(ensure(s, s->d_aggflag, 2 * (size_t)P.n_c0));
    a.pts = P_<uint32_t>(s->d_agga);
    a.inf = P_<uint8_t>(s->d_aggi);
    a.pre[0] = P_<uint32_t>(s->d_aggpre);
    a.pre[1] = a.pre[0] + pre_w;
    a.cinv[0] = P_<uint32_t>(s->d_aggtot);
    a.cinv[1] = a.cinv[0] + cinv_w;
    a.flag[0] = P_<uint8_t>(s->d_aggflag);
    a.flag[1] = a.flag[0] + P.n_c0;
    KL(s, "g1_aggregate", lsgk::agg_leaf(S_(s), a));
    for (int t = 0; t < P.L; t++) KL(s, "g1_aggregate", lsgk::agg_step(S_(s), a, t));
  }
  KL(s, "g1_aggregate", lsgk::agg_final(S_(s), a, (int)s->n_sets, PL(s, P.src_off), agg));
  return LSG_OK;
}

// D2H of per-set status into the pinned mirrors, then ev_done on the main stream
int launch_readback(Slot* s, bool status) {
  hipStream_t S = s->st[0];
  const size_t n = s->n_sets, np = s->n_pks;
  if (s->own_streams) {  // join the side stream
    LSG_HIP(s, hipEventRecord(s->ev_grp, s->st[1]));
    LSG_HIP(s, hipStreamWaitEvent(S, s->ev_grp, 0));
  }
  if (status) {
    if (n) {
      LSG_HIP(s, hipMemcpyAsync(s->h_err.p, s->d_seterr.p, 4 * n, hipMemcpyDeviceToHost, S));
      LSG_HIP(s, hipMemcpyAsync(s->h_pinf.p, s->d_pinf.p, n, hipMemcpyDeviceToHost, S));
    }
    if (np) LSG_HIP(s, hipMemcpyAsync(s->h_pkerr.p, s->d_pkerr.p, 4 * np, hipMemcpyDeviceToHost, S));
  }
  LSG_HIP(s, hipEventRecord(s->ev_done, S));
  return LSG_OK;
}

struct SetStatus {
  const int32_t* err;         // per set: BLST code (0 ok)
  std::vector<uint8_t> pinf;  // per set: aggregated pk is infinity (2: no keys at all)
  const int32_t* pkerr;       // per pubkey
};

SetStatus read_status(Slot* s) {
  SetStatus ss;
  const size_t n = s->n_sets;
  ss.err = H_<int32_t>(s->h_err);
  ss.pkerr = H_<int32_t>(s->h_pkerr);
  ss.pinf.assign(H_<uint8_t>(s->h_pinf), H_<uint8_t>(s->h_pinf) + n);
  for (size_t i = 0; i < n; i++)
    if (s->pk_cnt[i] == 0) ss.pinf[i] = 2;  // PublicKey.aggregate([]) throws
  return ss;
}

int32_t set_error(const SetStatus& ss, size_t i) {
  if (ss.err[i]) return ss.err[i];
  if (ss.pinf[i] == 2) return LSG_ERR_EMPTY_AGGREGATE;
  return ss.pinf[i] ? LSG_BLST_PK_IS_INFINITY : 0;
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

// ---------------------------------------------------------------------------- packages
namespace {

const uint8_t* fp12_one_blob() {  // canonical Fp12 one: c0.c0.c0 = 1
  static uint8_t b[576] = {0};
  b[47] = 1;
  return b;
}

// sig_prep into `out` for the slot's sets on the side stream.  mode: per-set bytes (1 =
// scale) or null; rnd null = no scaling at all (every group sums by the bucket MSM).
int launch_sig_prep(Slot* s, bool scale, const std::vector<uint8_t>* mode, uint32_t* out) {
  const int n = (int)s->n_sets;
  if (n == 0) return LSG_OK;
  s->cur = 1;
  const uint8_t* dm = nullptr;
  if (scale && mode) {
    LSG_RC(ensure_host(s, s->h_mode, (size_t)n));
    LSG_RC(ensure(s, s->d_mode, (size_t)n));
    memcpy(s->h_mode.p, mode->data(), (size_t)n);
    LSG_HIP(s, hipMemcpyAsync(s->d_mode.p, s->h_mode.p, (size_t)n, hipMemcpyHostToDevice, s->st[1]));
    dm = P_<uint8_t>(s->d_mode);
  }
  if (scale && (size_t)n <= slp_items_max()) {
    // small packages: the unscaled points, then [r_i] sig_i as one program per scaled set
    // (0.45 ms instead of a 64-bit scalar multiplication per lane pair, 2.2 ms)
    KL(s, "k_sig_prep", lsgk::sig_prep(S_(s), n, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf),
                                       P_<int32_t>(s->d_seterr), P_<uint8_t>(s->d_pinf), nullptr, nullptr, out));
    KL(s, "k_slp_g2_scale", lsg_slp_g2_scale(S_(s), n, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf),
                                             P_<int32_t>(s->d_seterr), P_<uint8_t>(s->d_pinf), P_<uint64_t>(s->d_rnd),
                                             dm, out));
    return LSG_OK;
  }
  KL(s, "k_sig_prep", lsgk::sig_prep(S_(s), n, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf),
                                     P_<int32_t>(s->d_seterr), P_<uint8_t>(s->d_pinf),
                                     scale ? P_<uint64_t>(s->d_rnd) : nullptr, dm, out));
  return LSG_OK;
}

// Part 1 of phase A on one device: stage this device's jobs (ids into `jobs`; batchable jobs
// first), plan and launch every per-set stage and group stage up to the canonical products
// (ev_part).  n_node > 0: this slot also reduces the all-gathered partials of n_node devices
// (its plan holds that product's chunk list).
// lone_ok: a set alone in its phase-A group may be verified unscaled (a plain verify, as
// maybeBatch.ts:34-38).  False when the package group's partial is multiplied with other
// partials before its verdict (a multi-device ticket, lsg_batch_partial): there every r_i is
// random and nonzero, or two forged one-set shards (sig_a + D, sig_b - D) would pass together.
int pkg_part1(Slot* s, const lsg_job* jobs, const std::vector<size_t>& ids, uint64_t seed, int n_node,
              const std::vector<size_t>* subs = nullptr, bool lone_ok = true) {
  timer_reset(s);
  s->plan.clear();
  memset(&s->stats, 0, sizeof(s->stats));
  s->stats.start_ns = now_ns();
  const size_t nj = ids.size();
  s->jobs.assign(nj, JobRec());
  s->job_ids = ids;
  s->results.assign(nj, lsg_job_result{LSG_INVALID, 0});
  s->job_group.assign(nj, -1);
  s->batch_order.clear();
  s->big_g = -1;
  s->rs2_ready = false;
  s->rs2_scaled.clear();
  s->has_node = n_node > 0;
  s->lone_unscaled = false;
  s->big_fe_pending = false;
  s->seed = seed;
  s->nb_g = -1;
  s->nb_items.clear();
  std::vector<const lsg_set*> flat;
  std::vector<size_t> nonb;
  for (int pass = 0; pass < 2; pass++)
    for (size_t k = 0; k < nj; k++) {
      const lsg_job& J = jobs[ids[k]];
      const bool b = (J.flags & LSG_JOB_BATCHABLE) != 0;
      if (b != (pass == 0)) continue;
      s->jobs[k].first = flat.size();
      s->jobs[k].count = J.n_sets;
      s->jobs[k].flags = J.flags;
      for (uint32_t q = 0; q < J.n_sets; q++) flat.push_back(&J.sets[q]);
      (b ? s->batch_order : nonb).push_back(k);
    }
  s->nb_sets = 0;
  for (size_t k : s->batch_order) s->nb_sets += s->jobs[k].count;
  // a coalesced launch: sub-package bounds (jobs and batch_order positions), per-sub state
  s->n_sub = subs ? (int)subs->size() - 1 : 0;
  s->resolved = s->resolving = false;
  s->resolve_rc = LSG_OK;
  if (subs) {
    s->sub_first = *subs;
    s->bpos_first.assign(1, 0);
    size_t q = 0;
    for (int k = 0; k < s->n_sub; k++) {
      while (q < s->batch_order.size() && s->batch_order[q] < (*subs)[k + 1]) q++;
      s->bpos_first.push_back(q);
    }
    lsg_stats z;
    memset(&z, 0, sizeof(z));
    s->sub_stats.assign(s->n_sub, z);
    s->sub_pkfail.assign(s->n_sub, 0);
    s->sub_done.assign(s->n_sub, 0);
  }
  s->K = miller_k_for(flat.size());
  // sets alone in their phase-A group (and so in every later group): no RLC scaling
  std::vector<uint8_t> noscale(flat.size(), 0);
  if (!lone_ok) {
    // (non-batchable jobs below: their groups never enter the package partial)
  } else if (package_group_mode() && !subs) {
    if (s->nb_sets == 1) noscale[0] = s->lone_unscaled = true;
  } else if (package_group_mode() && sub_groups_on()) {  // a coalesced launch: one package group per sub-package
    for (int k = 0; k < s->n_sub; k++) {
      size_t len = 0, first = 0;
      for (size_t q = s->bpos_first[(size_t)k]; q < s->bpos_first[(size_t)k + 1]; q++) {
        if (!len) first = s->jobs[s->batch_order[q]].first;
        len += s->jobs[s->batch_order[q]].count;
      }
      if (len == 1) noscale[first] = 1;
    }
  } else {
    const auto ch = slot_chunks(s);
    for (auto& c : ch) {
      size_t len = 0;
      for (size_t q = c.first; q < c.second; q++) len += s->jobs[s->batch_order[q]].count;
      if (len == 1)
        for (size_t q = c.first; q < c.second; q++)
          if (s->jobs[s->batch_order[q]].count == 1) noscale[s->jobs[s->batch_order[q]].first] = 1;
    }
  }
  // the merged non-batchable group (nb_merge_on): every one of its sets is randomised, so a
  // one-set job in it is scaled too (its own check, if the group fails, stays exact: r_i != 0)
  size_t nb_live = 0;
  for (size_t k : nonb) nb_live += s->jobs[k].count ? 1 : 0;
  const bool nb_merge = nb_merge_on() && nb_live >= 2 && !subs && package_group_mode();
  for (size_t k : nonb)
    if (s->jobs[k].count == 1 && !nb_merge) noscale[s->jobs[k].first] = 1;
  const uint64_t th0 = trace_host() ? now_ns() : 0;
  LSG_RC(stage_sets(s, flat.data(), flat.size(), seed, true, &noscale, true));
  const uint64_t th1 = trace_host() ? now_ns() : 0;
  // phase-A groups, MSM groups first: the package group, then one per non-batchable job
  PhasePlan& A = s->phA;
  A = PhasePlan();
  std::vector<Grp> gm, gs;
  std::vector<int> om, os;  // owner: -2 the package group, else the job
  auto add = [&](size_t first, size_t len, int owner) {
    Grp g;
    g.first = first;
    g.len = len;
    g.msm = len >= std::max(msm_min_group(), (size_t)2);  // an r_i = 0 set never enters a bucket MSM
    (g.msm ? gm : gs).push_back(g);
    (g.msm ? om : os).push_back(owner);
  };
  // one RLC group per package; a coalesced launch: one per sub-package (each keeps its own
  // verdicts, chunks and fallback: pkg_resolve)
  s->chunk_mode = !package_group_mode() || (subs && !sub_groups_on());
  s->chunk_group.clear();
  s->sub_big.assign((size_t)s->n_sub, -1);
  std::vector<std::pair<size_t, size_t>> chunks;
  if (s->chunk_mode) {
    chunks = slot_chunks(s);
    for (size_t c = 0; c < chunks.size(); c++) {
      size_t len = 0;
      for (size_t q = chunks[c].first; q < chunks[c].second; q++) len += s->jobs[s->batch_order[q]].count;
      if (len) add(s->jobs[s->batch_order[chunks[c].first]].first, len, -3 - (int)c);
    }
    s->chunk_group.assign(chunks.size(), -1);
  } else if (s->n_sub) {
    for (int k = 0; k < s->n_sub; k++) {
      size_t len = 0, first = 0;
      for (size_t q = s->bpos_first[(size_t)k]; q < s->bpos_first[(size_t)k + 1]; q++) {
        if (!len) first = s->jobs[s->batch_order[q]].first;
        len += s->jobs[s->batch_order[q]].count;
      }
      if (len) add(first, len, -1000 - k);
    }
  } else if (s->nb_sets) {
    add(0, s->nb_sets, -2);
  }
  size_t nb_first = 0, nb_len = 0;
  for (size_t k : nonb) {
    if (s->jobs[k].count == 0) {
      s->results[k] = {LSG_ERROR, LSG_ERR_EMPTY_SET};  // maybeBatch.ts:29-31
    } else if (nb_merge) {  // staged contiguously after the batchable sets, in job order
      if (!nb_len) nb_first = s->jobs[k].first;
      nb_len += s->jobs[k].count;
    } else {
      add(s->jobs[k].first, s->jobs[k].count, (int)k);
    }
  }
  constexpr int NB_OWNER = INT32_MIN;  // (chunk owners are -3 - c, sub-package owners -1000 - k)
  if (nb_merge) add(nb_first, nb_len, NB_OWNER);
  A.groups = gm;
  A.groups.insert(A.groups.end(), gs.begin(), gs.end());
  om.insert(om.end(), os.begin(), os.end());
  // the package group's items never cross a 16-job chunk: if the group fails, each chunk's
  // check (phase B) reuses them instead of re-running the Miller accumulation
  std::vector<size_t> chunk_sub;  // chunks with sets, in order
  if (nb_merge || (!s->chunk_mode && s->nb_sets)) A.sub.assign(om.size(), {});
  if (nb_merge)  // the merged group's items never cross a job
    for (size_t g = 0; g < om.size(); g++)
      if (om[g] == NB_OWNER)
        for (size_t k : nonb)
          if (s->jobs[k].count) A.sub[g].push_back({s->jobs[k].first, s->jobs[k].first + s->jobs[k].count});
  if (!s->chunk_mode && s->nb_sets) {
    chunks = slot_chunks(s);
    for (size_t g = 0; g < om.size(); g++) {
      if ((om[g] != -2 && om[g] > -1000) || om[g] == NB_OWNER) continue;
      const int sub = om[g] <= -1000 ? -1000 - om[g] : -1;
      for (size_t c = 0; c < chunks.size(); c++) {
        if (sub >= 0 && sub_of_pos(s, chunks[c].first) != sub) continue;
        const size_t first = s->jobs[s->batch_order[chunks[c].first]].first;
        size_t len = 0;
        for (size_t q = chunks[c].first; q < chunks[c].second; q++) len += s->jobs[s->batch_order[q]].count;
        if (len) {
          A.sub[g].push_back({first, first + len});
          chunk_sub.push_back(c);
        }
      }
    }
  }
  for (size_t g = 0; g < om.size(); g++) {
    if (om[g] == -2)
      s->big_g = (int)g;
    else if (om[g] == NB_OWNER)
      s->nb_g = (int)g;
    else if (om[g] <= -3 && s->chunk_mode)  // (chunk mode has no sub-package owners)
      s->chunk_group[(size_t)(-3 - om[g])] = (int)g;
    else if (om[g] <= -1000)
      s->sub_big[(size_t)(-1000 - om[g])] = (int)g;
    else
      s->job_group[(size_t)om[g]] = (int)g;
  }
  LSG_RC(size_state(s, s->n_sets, s->n_pks, A.groups.size(), gm.size(), 1));
  s->agg = AggPlan();
  if (!s->single_keys) {
    if (s->n_pks >= AGG_TREE_MIN_KEYS && agg_tree_on())
      s->agg = plan_agg_tree(s);
    else
      s->pkagg = plan_pk_agg(s);
  }
  // sets of the package group that share a message share one Miller pair: Π e(r_i pk_i, H(m))
  // = e(Σ r_i pk_i, H(m)) exactly.  Its per-set items are then never computed, so a failing
  // package group's chunks (phase B) run their own items and phase C goes per job.
  A.agg_g = -1;
  if (s->msg_dedup && !s->chunk_mode && s->big_g >= 0 && msg_agg_on() && s->n_msgs <= (size_t)8192 &&
      slp_items_max() > 0) {
    const Grp& g = A.groups[(size_t)s->big_g];
    std::vector<int32_t> cnt(s->n_msgs, 0), off(s->n_msgs), fill;
    for (size_t i = g.first; i < g.first + g.len; i++) cnt[s->msg_id[i]]++;
    int32_t tot = 0;
    for (size_t j = 0; j < s->n_msgs; j++) {
      off[j] = tot;
      tot += cnt[j];
    }
    fill = off;
    const size_t idx_off = s->plan.size();
    s->plan.resize(idx_off + (size_t)tot);
    for (size_t i = g.first; i < g.first + g.len; i++) s->plan[idx_off + (size_t)fill[s->msg_id[i]]++] = (int32_t)i;
    s->msum = plan_seg(s->plan, 0, off, cnt, true, idx_off, 0);
    A.agg_g = s->big_g;
    A.n_magg = s->n_msgs;
  }
  LSG_RC(plan_phase(s, A));
  if (s->nb_g >= 0) {  // per non-batchable job, its items among the merged group's
    s->nb_items.assign(nj, {-1, -1});
    size_t r = 0;
    for (size_t g = 0; g < om.size(); g++) {
      if ((int)g == A.agg_g) continue;  // (message items: no sub_items entries)
      const size_t ns = g < A.sub.size() && !A.sub[g].empty() ? A.sub[g].size() : 1;
      if ((int)g == s->nb_g) {
        size_t q = r;
        for (size_t k : nonb)
          if (s->jobs[k].count) s->nb_items[k] = A.sub_items[q++];
      }
      r += ns;
    }
    for (size_t k : nonb)
      if (s->jobs[k].count) s->job_group[k] = s->nb_g;
  }
  s->chunk_items.assign(chunks.size(), {-1, -1});
  if (!chunk_sub.empty() && A.agg_g < 0) {  // sub_items of the package group, in chunk order
    size_t r = 0;
    for (size_t g = 0; g < om.size(); g++) {
      const size_t ns = g < A.sub.size() && !A.sub[g].empty() ? A.sub[g].size() : 1;
      const bool pkg = om[g] == -2 || (om[g] <= -1000 && om[g] != NB_OWNER);
      if (pkg)
        for (size_t k = 0; k < ns; k++) s->chunk_items[chunk_sub[k]] = A.sub_items[r + k];
      if (pkg) chunk_sub.erase(chunk_sub.begin(), chunk_sub.begin() + (long)ns);
      r += ns;
    }
  }
  SegPlan node;
  if (n_node > 0) {
    std::vector<int32_t> off{0}, len{(int32_t)n_node};
    node = plan_seg(s->plan, 2, off, len, false, 0, 0);
  }
  LSG_RC(upload_plan(s));
  const uint64_t th2 = trace_host() ? now_ns() : 0;
  LSG_RC(launch_set_stages(s, &s->pkagg, A, P_<uint32_t>(s->d_fall)));
  const uint64_t th3 = trace_host() ? now_ns() : 0;
  // signature points: unscaled for MSM groups, [r_i] sig_i for the rest
  s->rs_raw.assign(s->n_sets, 0);
  for (size_t g = 0; g < A.n_msm; g++) memset(s->rs_raw.data() + A.groups[g].first, 1, A.groups[g].len);
  if (!A.groups.empty()) {
    const bool any_small = A.n_msm < A.groups.size();
    std::vector<uint8_t> mode;
    if (any_small && A.n_msm) {
      mode.assign(s->n_sets, 0);
      for (size_t g = A.n_msm; g < A.groups.size(); g++)
        memset(mode.data() + A.groups[g].first, 1, A.groups[g].len);
    }
    LSG_RC(launch_sig_prep(s, any_small, mode.empty() ? nullptr : &mode, P_<uint32_t>(s->d_rs)));
  }
  LSG_RC(launch_phase(s, A, P_<uint32_t>(s->d_rs), P_<uint32_t>(s->d_fall), true));
  if (A.groups.empty() || s->big_g < 0) {  // no package group: the partial is the identity
    s->cur = 0;
    LSG_HIP(s, hipMemcpyAsync(P_<uint8_t>(s->d_gath) + 576 * LSG_MAX_DEVICES, fp12_one_blob(), 576,
                              hipMemcpyHostToDevice, s->st[0]));
    LSG_HIP(s, hipEventRecord(s->ev_part, s->st[0]));
  }
  s->phA_node = node;
  if (trace_host()) {
    const uint64_t th4 = now_ns();
    fprintf(stderr, "lsg host: sets %zu jobs %zu subs %d groups %zu | stage %.3f plan %.3f set-launch %.3f group-launch %.3f ms\n",
            (size_t)s->n_sets, nj, s->n_sub, A.groups.size(), (th1 - th0) * 1e-6, (th2 - th1) * 1e-6, (th3 - th2) * 1e-6,
            (th4 - th3) * 1e-6);
  }
  return LSG_OK;
}

// device pointer of the package group's canonical partial (576 bytes)
const uint8_t* pkg_partial_dev(Slot* s) {
  if (s->phA.groups.empty() || s->big_g < 0) return P_<uint8_t>(s->d_gath) + 576 * LSG_MAX_DEVICES;
  return P_<uint8_t>(s->d_Fb) + 576 * (size_t)s->big_g;
}

// The package group's partial as it may leave the slot (lsg_jobs_partial*), on the main stream:
// a lone unscaled set's f is raised to a fresh nonzero 64-bit randomizer (two
// one-set shards holding sig_a + D and sig_b - D must not pass a product check together).
// xs: launch the power there instead of on the slot's stream (the partial is complete)
int export_partial_dev(Slot* s, const uint8_t** src, hipStream_t xs = nullptr) {
  *src = pkg_partial_dev(s);
  if (!s->lone_unscaled) return LSG_OK;
  uint64_t r = 0;
  if (s->seed) {  // tests: reproducible
    uint64_t sd = s->seed ^ 0x5851f42d4c957f2dull;
    do r = splitmix64(sd);
    while (r == 0);
  } else {
    do {
      if (!os_random(&r, 8)) {
        set_err(s->d->c, "no entropy for the exported partial's randomizer (getrandom failed)");
        return LSG_ERR_ENTROPY;
      }
    } while (r == 0);
  }
  LSG_RC(ensure(s, s->d_xport, 576));
  s->cur = 0;
  if (xs) {
    const hipError_t e = lsgk::fp12_pow_u64(xs, *src, r, P_<uint8_t>(s->d_xport));
    if (e != hipSuccess) return fail(s, "k_fp12_pow", e);
  } else {
    KL(s, "k_fp12_pow", lsgk::fp12_pow_u64(S_(s), *src, r, P_<uint8_t>(s->d_xport)));
  }
  *src = P_<uint8_t>(s->d_xport);
  return LSG_OK;
}

// node check on this slot (device 0 of the ticket): product of the n gathered partials in
// d_gath, one final exponentiation -> h_nodeV (ev_node)
int pkg_node_check(Slot* s, int n) {
  s->cur = 0;
  const uint32_t* nf = P_<uint32_t>(s->d_nodeF);
  KL(s, "k_blobs_to_fp12", lsgk::blobs_to_fp12(S_(s), n, P_<uint8_t>(s->d_gath), P_<uint32_t>(s->d_nodeF)));
  LSG_RC(run_seg(s, 2, "fp12_product", s->phA_node, nf, P_<uint32_t>(s->d_nodeF) + W_F12 * (size_t)n));
  uint8_t* blob = P_<uint8_t>(s->d_gath) + 576 * (size_t)(LSG_MAX_DEVICES + 1);
  KL(s, "k_fp12_to_canon", lsgk::fp12_to_canon(S_(s), 1, P_<uint32_t>(s->d_nodeF) + W_F12 * (size_t)n, blob));
  KL(s, SERIAL_LABEL(final_exp), lsg_row_final_exp(S_(s), 1, blob, P_<int32_t>(s->d_nodeV)));
  LSG_HIP(s, hipMemcpyAsync(s->h_nodeV.p, s->d_nodeV.p, 4, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipEventRecord(s->ev_node, s->st[0]));
  return LSG_OK;
}

// Part 2 of phase A: every group's final exponentiation and the status readback (ev_done).
// skip_big (a multi-device ticket): the package group's final exponentiation is left out --
// the node check over all devices' partials decides it (one final
// exponentiation per node), and it runs only when that check fails (pkg_resolve).
int pkg_part2(Slot* s, bool skip_big = false) {
  const size_t ng = s->phA.groups.size();
  s->big_fe_pending = skip_big && !s->chunk_mode && s->big_g >= 0;
  if (s->big_fe_pending) {
    LSG_RC(launch_fe_range(s, 0, (size_t)s->big_g));
    LSG_RC(launch_fe_range(s, (size_t)s->big_g + 1, ng));
  } else {
    LSG_RC(launch_fe(s, ng));
  }
  return launch_readback(s, true);
}

// One fallback phase (worker.ts:74-96) over `groups` (scaled signature sums, own Miller items
// into fall2), synchronous; verdicts into v.
// The context mutex is released while a fallback phase runs on the device (the ticket's slots
// stay claimed, so no other caller touches them): other threads keep submitting and resolving.
typedef std::unique_lock<std::mutex> CtxLock;

// One fallback phase (worker.ts:74-96) over `groups` (scaled signature sums), synchronous;
// verdicts into v.  given: per group, its items among phase A's resident Miller items (the
// package group's chunk-aligned items: no new Miller accumulation); else the phase plans and
// accumulates its own items (into fall2).
int run_fallback_phase(Slot* s, CtxLock* lk, const std::vector<Grp>& groups,
                       const std::vector<std::pair<int32_t, int32_t>>* given, std::vector<int32_t>& v) {
  v.assign(groups.size(), 0);
  if (groups.empty()) return LSG_OK;
  const uint64_t tf0 = trace_host() ? now_ns() : 0;
  // Signature sums: a group whose sets' unscaled points are resident (they were in a phase-A
  // bucket-MSM group: d_rs) and that is large enough sums them by its own bucket MSM (no
  // per-set scaling); the others sum [r_i] sig_i (d_rs2, scaled below).  MSM groups go first
  // (plan_phase); `order` maps the phase's group k to the caller's.
  std::vector<size_t> order;
  std::vector<uint8_t> gm(groups.size(), 0);
  for (size_t g = 0; g < groups.size(); g++) {
    bool ok = groups[g].len >= std::max(msm_min_group(), (size_t)2) && s->rs_raw.size() == s->n_sets;
    for (size_t i = groups[g].first; ok && i < groups[g].first + groups[g].len; i++) ok = s->rs_raw[i] != 0;
    gm[g] = ok;
    if (ok) order.push_back(g);
  }
  const size_t n_msm = order.size();
  for (size_t g = 0; g < groups.size(); g++)
    if (!gm[g]) order.push_back(g);
  // size this phase's buffers BEFORE any pointer into them is taken or any launch queued:
  // a phase with more groups than phase A had grows d_fall2 (and the group buffers), and a
  // pointer saved earlier would name the freed allocation
  LSG_RC(size_state(s, s->n_sets, s->n_pks, groups.size(), n_msm, 2));
  s->cur = 0;  // the phase's kernel timers follow phase A's (lsg_last_kernel_times: the whole ticket)
  s->plan.clear();
  PhasePlan Ph;
  for (size_t k = 0; k < order.size(); k++) {
    Ph.groups.push_back(groups[order[k]]);
    Ph.groups.back().msm = gm[order[k]] != 0;
  }
  // groups of one set each (the per-job phase of single-set jobs): one-set Miller items in
  // the list form instead of four-wave fused items holding one pair
  size_t singles = 0;
  for (auto& g : groups) singles += g.len == 1 ? 1 : 0;
  const int K0 = s->K;
  if (!given && 2 * singles >= groups.size()) s->K = 1;
  if (given) {
    Ph.reuse_items = true;
    for (size_t k = 0; k < order.size(); k++) Ph.given.push_back((*given)[order[k]]);
    Ph.n_items = s->phA.n_items;
    Ph.term_base = s->phA.n_items + s->phA.groups.size();  // after phase A's own terms
  }
  const int prc = plan_phase(s, Ph);
  s->K = K0;
  LSG_RC(prc);
  LSG_RC(upload_plan(s));
  // [r_i] sig_i into d_rs2 for the sets no earlier fallback phase of this package scaled
  if (s->rs2_scaled.size() != s->n_sets) s->rs2_scaled.assign(s->n_sets, 0);
  std::vector<uint8_t> mode(s->n_sets, 0);
  bool any = false;
  for (size_t g = 0; g < groups.size(); g++) {
    if (gm[g]) continue;  // (its MSM reads the unscaled points)
    for (size_t i = groups[g].first; i < groups[g].first + groups[g].len; i++)
      if (!s->rs2_scaled[i]) {
        mode[i] = s->rs2_scaled[i] = 1;
        any = true;
      }
  }
  // the side stream needs the plan: order it after the upload on the main stream
  LSG_HIP(s, hipEventRecord(s->ev_in, s->st[0]));
  LSG_HIP(s, hipStreamWaitEvent(s->st[1], s->ev_in, 0));
  if (any) {
    s->cur = 1;
    const int n = (int)s->n_sets;
    LSG_RC(ensure_host(s, s->h_mode, (size_t)n));
    memcpy(s->h_mode.p, mode.data(), (size_t)n);
    LSG_HIP(s, hipMemcpyAsync(s->d_mode.p, s->h_mode.p, (size_t)n, hipMemcpyHostToDevice, s->st[1]));
    size_t n_scaled = 0;
    for (uint8_t m : mode) n_scaled += m;
    if (slp_items_max() > 0 && n_scaled <= 8192)  // one program per scaled set (the others exit at once)
      KL(s, "k_slp_g2_scale", lsg_slp_g2_scale(S_(s), n, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf),
                                               P_<int32_t>(s->d_seterr), P_<uint8_t>(s->d_pinf), P_<uint64_t>(s->d_rnd),
                                               P_<uint8_t>(s->d_mode), P_<uint32_t>(s->d_rs2)));
    else
      KL(s, "k_sig_scale", lsgk::sig_scale_only(S_(s), n, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf),
                                                P_<int32_t>(s->d_seterr), P_<uint8_t>(s->d_pinf), P_<uint64_t>(s->d_rnd),
                                                P_<uint8_t>(s->d_mode), P_<uint32_t>(s->d_rs2)));
  }
  s->cur = 0;
  uint32_t* fall = given ? P_<uint32_t>(s->d_fall) : P_<uint32_t>(s->d_fall2);
  if (!given) LSG_RC(launch_accum(s, Ph.n_items, Ph.item_off, fall, Ph.single_items));
  LSG_RC(launch_phase(s, Ph, P_<uint32_t>(s->d_rs2), fall, false, P_<uint32_t>(s->d_rs)));
  LSG_RC(launch_fe(s, groups.size()));
  LSG_RC(launch_readback(s, false));
  const uint64_t tf1 = trace_host() ? now_ns() : 0;
  const int dev = s->d->device;
  if (lk) lk->unlock();
  hipError_t e = event_wait(s->ev_done);
  if (lk) {
    lk->lock();
    (void)hipSetDevice(dev);
  }
  if (e != hipSuccess) return fail(s, "hipEventSynchronize", e);
  if (trace_host())
    fprintf(stderr, "lsg host: fallback groups %zu (msm %zu) given %d | plan+launch %.3f ms, device+lock %.3f ms\n",
            groups.size(), n_msm, given ? 1 : 0, (tf1 - tf0) * 1e-6, (now_ns() - tf1) * 1e-6);
  s->stats.n_final_exps += (uint32_t)groups.size();
  for (size_t k = 0; k < order.size(); k++) v[order[k]] = H_<int32_t>(s->h_verdict)[k];
  return LSG_OK;
}

// the deferred final exponentiation of the package group (pkg_part2 skip_big), synchronous
int run_big_fe(Slot* s, CtxLock* lk) {
  s->cur = 0;
  LSG_RC(launch_fe_range(s, (size_t)s->big_g, (size_t)s->big_g + 1));
  LSG_HIP(s, hipEventRecord(s->ev_done, s->st[0]));
  const int dev = s->d->device;
  if (lk) lk->unlock();
  hipError_t e = event_wait(s->ev_done);
  if (lk) {
    lk->lock();
    (void)hipSetDevice(dev);
  }
  if (e != hipSuccess) return fail(s, "hipEventSynchronize", e);
  s->big_fe_pending = false;
  return LSG_OK;
}

// The reference's verdict rules for this device's share of the package (worker.ts:30-106),
// after ev_done.  node_valid: 1 = the node-wide check of all devices' partials passed, 0 = it
// failed (this device's own package check localises), -1 = no node check (single device).
// worker.ts:41-43: deserializeSet runs over the package's jobs in caller order before any
// verification; the first bad pubkey throws out of verifyManySignatureSets.  Returns that
// key's code for this device's share (0: none) and the caller index of its job.
int32_t first_pk_error(Slot* s, size_t* job_id) {
  const int32_t* pkerr = H_<int32_t>(s->h_pkerr);
  for (size_t k = 0; k < s->jobs.size(); k++) {  // jobs[k] are in caller order (job_ids ascending)
    const JobRec& J = s->jobs[k];
    for (size_t i = J.first; i < J.first + J.count; i++)
      for (uint32_t q = 0; q < s->pk_cnt[i]; q++)
        if (const int32_t e = pkerr[s->pk_first[i] + q]) {
          *job_id = s->job_ids[k];
          return e;
        }
  }
  return 0;
}

// pkfail: the package-wide deserializeSet failure (first_pk_error over every device of the
// ticket, in caller order) -- a bad key on any device rejects every job of the package
// node_valid 2: this ticket's own node check (lsg_init_devices: the library gathered every
// device's partial itself) passed, and it decides the package group.
int pkg_resolve(Slot* s, CtxLock* lk, int node_valid, int32_t pkfail) {
  const SetStatus ss = read_status(s);
  const PhasePlan& A = s->phA;
  std::vector<int32_t> vA(H_<int32_t>(s->h_verdict), H_<int32_t>(s->h_verdict) + A.groups.size());
  s->stats.n_final_exps += (uint32_t)(A.groups.size() - (s->big_fe_pending ? 1 : 0));
  const size_t nj = s->jobs.size();
  if (pkfail) {
    for (size_t j = 0; j < nj; j++) s->results[j] = {LSG_ERROR, pkfail};
    return LSG_OK;
  }
  if (s->big_fe_pending) {
    if (node_valid == 2) {
      vA[(size_t)s->big_g] = 1;
    } else {  // the node check failed: this device's own check localises
      LSG_RC(run_big_fe(s, lk));
      vA[(size_t)s->big_g] = H_<int32_t>(s->h_verdict)[s->big_g];
      s->stats.n_final_exps++;
    }
  }
  // counters of the chunk at batch_order position q: the slot's, and its sub-package's
  auto retry_inc = [&](size_t q) {
    s->stats.batch_retries++;
    if (s->n_sub) s->sub_stats[(size_t)sub_of_pos(s, q)].batch_retries++;
  };
  auto succ_add = [&](size_t q, size_t len) {
    s->stats.batch_sigs_success += (uint32_t)len;
    if (s->n_sub) s->sub_stats[(size_t)sub_of_pos(s, q)].batch_sigs_success += (uint32_t)len;
  };
  // a coalesced launch: the deserializeSet rule per sub-package (worker.ts:41-43)
  std::vector<uint8_t> job_dead(nj, 0);
  for (int k = 0; k < s->n_sub; k++) {
    const int32_t* pkerr = H_<int32_t>(s->h_pkerr);
    int32_t e = 0;
    size_t ej = 0;
    for (size_t j = s->sub_first[k]; j < s->sub_first[k + 1] && !e; j++)
      for (size_t i = s->jobs[j].first; i < s->jobs[j].first + s->jobs[j].count && !e; i++)
        for (uint32_t q = 0; q < s->pk_cnt[i] && !e; q++)
          if (pkerr[s->pk_first[i] + q]) {
            e = pkerr[s->pk_first[i] + q];
            ej = j - s->sub_first[k];
          }
    s->sub_pkfail[k] = e;
    s->sub_stats[k].key_error = e;
    s->sub_stats[k].key_error_job = e ? (uint32_t)ej : 0;
    if (e)
      for (size_t j = s->sub_first[k]; j < s->sub_first[k + 1]; j++) {
        s->results[j] = {LSG_ERROR, e};
        job_dead[j] = 1;
      }
  }
  // non-batchable jobs: their own group (worker.ts:88-96), or the merged group (nb_g): a
  // passing one answers every such job; a failing one is localised job by job over the jobs'
  // resident phase-A items (a fallback phase), so each verdict is still the job's own
  std::vector<Grp> nbg;
  std::vector<size_t> nbj;
  std::vector<std::pair<int32_t, int32_t>> nbi;
  for (size_t j = 0; j < nj; j++) {
    const int g = s->job_group[j];
    if (g < 0 || job_dead[j]) continue;
    const int32_t e = job_error(ss, s->jobs[j].first, s->jobs[j].count);
    if (!e && g == s->nb_g && !vA[(size_t)g]) {
      Grp q;
      q.first = s->jobs[j].first;
      q.len = s->jobs[j].count;
      nbg.push_back(q);
      nbj.push_back(j);
      nbi.push_back(s->nb_items[j]);
      continue;
    }
    s->results[j] = e ? lsg_job_result{LSG_ERROR, e} : lsg_job_result{vA[(size_t)g] ? LSG_VALID : LSG_INVALID, 0};
  }
  if (!nbg.empty()) {
    std::vector<int32_t> vn;
    LSG_RC(run_fallback_phase(s, lk, nbg, &nbi, vn));
    for (size_t k = 0; k < nbj.size(); k++) s->results[nbj[k]] = {vn[k] ? LSG_VALID : LSG_INVALID, 0};
  }
  if (s->batch_order.empty()) return LSG_OK;
  // batchable jobs: chunks of >= 16 jobs (worker.ts:51-86)
  // The device's own check of its share (computed in phase A in any case) decides.  The
  // node-wide verdict is advisory: a passing node check with a failing own check (a caller
  // whose all-gather missed a rank) localises like a failing one instead of
  // accepting the package.
  (void)node_valid;
  auto chunks = slot_chunks(s);
  // the package group covering chunk c passed (a coalesced launch: its sub-package's group)
  auto pkg_ok = [&](size_t c) {
    const int g = s->n_sub ? s->sub_big[(size_t)sub_of_pos(s, chunks[c].first)] : s->big_g;
    return g < 0 || vA[(size_t)g] != 0;
  };
  std::vector<size_t> retry;  // jobs verified individually (phase C)
  std::vector<Grp> chk;       // chunks checked on their own (phase B)
  std::vector<std::pair<size_t, size_t>> chk_jobs;
  std::vector<std::pair<int32_t, int32_t>> chk_items;  // their resident phase-A items
  std::vector<uint8_t> chk_threw;                      // the chunk threw (its retry is counted)
  std::vector<uint8_t> job_err(nj, 0);                 // the job's result is its decode error
  bool any_err_chunk = false;
  std::vector<uint8_t> chunk_err(chunks.size(), 0);
  for (size_t c = 0; c < chunks.size(); c++) {
    for (size_t q = chunks[c].first; q < chunks[c].second && !chunk_err[c]; q++) {
      const JobRec& J = s->jobs[s->batch_order[q]];
      for (size_t i = J.first; i < J.first + J.count; i++)
        if (set_error(ss, i)) {
          chunk_err[c] = 1;
          break;
        }
    }
    any_err_chunk = any_err_chunk || chunk_err[c];
  }
  // a coalesced sub-package of exactly one chunk: its group has the chunk's sets and r_i
  std::vector<int> sub_nchunks((size_t)s->n_sub, 0);
  for (size_t c = 0; c < chunks.size() && s->n_sub; c++) sub_nchunks[(size_t)sub_of_pos(s, chunks[c].first)]++;
  auto group_is_chunk = [&](size_t c) {
    if (!s->n_sub) return chunks.size() == 1 && !any_err_chunk;
    return sub_nchunks[(size_t)sub_of_pos(s, chunks[c].first)] == 1;  // (chunk c has no decode error)
  };
  for (size_t c = 0; c < chunks.size(); c++) {
    if (job_dead[s->batch_order[chunks[c].first]]) continue;  // its sub-package has a bad key
    const size_t first = s->jobs[s->batch_order[chunks[c].first]].first;
    size_t len = 0;
    for (size_t q = chunks[c].first; q < chunks[c].second; q++) len += s->jobs[s->batch_order[q]].count;
    if (len == 0) {  // maybeBatch([]) throws: retried, and every job throws again
      retry_inc(chunks[c].first);
      for (size_t q = chunks[c].first; q < chunks[c].second; q++)
        s->results[s->batch_order[q]] = {LSG_ERROR, LSG_ERR_EMPTY_SET};
      continue;
    }
    if (!chunk_err[c] && s->chunk_mode) {  // the chunk's own phase-A group decides
      if (vA[(size_t)s->chunk_group[c]]) {
        for (size_t q = chunks[c].first; q < chunks[c].second; q++) s->results[s->batch_order[q]] = {LSG_VALID, 0};
        succ_add(chunks[c].first, len);
      } else {
        retry_inc(chunks[c].first);
        for (size_t q = chunks[c].first; q < chunks[c].second; q++) retry.push_back(s->batch_order[q]);
      }
    } else if (!chunk_err[c]) {
      if (pkg_ok(c)) {
        for (size_t q = chunks[c].first; q < chunks[c].second; q++) s->results[s->batch_order[q]] = {LSG_VALID, 0};
        succ_add(chunks[c].first, len);
      } else if (group_is_chunk(c)) {
        // the package (or sub-package) group is exactly this chunk: its verdict is the chunk's
        retry_inc(chunks[c].first);
        for (size_t q = chunks[c].first; q < chunks[c].second; q++) retry.push_back(s->batch_order[q]);
      } else {
        Grp g;
        g.first = first;
        g.len = len;
        chk.push_back(g);
        chk_jobs.push_back(chunks[c]);
        chk_items.push_back(c < s->chunk_items.size() ? s->chunk_items[c] : std::make_pair(-1, -1));
        chk_threw.push_back(0);
      }
    } else {  // the chunk throws (worker.ts:79-85): every job is verified on its own
      retry_inc(chunks[c].first);
      // A job's own verdict is its validity alone, so the chunk's jobs that do not throw are
      // checked as ONE group first -- the throwing sets are the identity in the chunk's items
      // and signature sums (the kernels' err rule) -- and localised only if it fails: a chunk
      // with one undecodable signature costs one group check instead of 16 per-job checks.
      // Verdicts and the batch counters are the reference's (the retry counted above, no
      // batch success for a chunk that threw).
      bool live = false;
      for (size_t q = chunks[c].first; q < chunks[c].second; q++) {
        const size_t j = s->batch_order[q];
        const int32_t e = job_error(ss, s->jobs[j].first, s->jobs[j].count);
        if (e) {
          s->results[j] = {LSG_ERROR, e};
          job_err[j] = 1;
        } else {
          live = true;
        }
      }
      if (!live) continue;
      if (!s->chunk_mode && pkg_ok(c)) {  // its sets are in the passing package group
        for (size_t q = chunks[c].first; q < chunks[c].second; q++)
          if (!job_err[s->batch_order[q]]) s->results[s->batch_order[q]] = {LSG_VALID, 0};
      } else if (s->chunk_mode) {  // the chunk's own phase-A group (throwing sets as identity)
        const bool ok = vA[(size_t)s->chunk_group[c]] != 0;
        for (size_t q = chunks[c].first; q < chunks[c].second; q++) {
          const size_t j = s->batch_order[q];
          if (job_err[j]) continue;
          if (ok)
            s->results[j] = {LSG_VALID, 0};
          else
            retry.push_back(j);
        }
      } else {
        Grp g;
        g.first = first;
        g.len = len;
        chk.push_back(g);
        chk_jobs.push_back(chunks[c]);
        chk_items.push_back(c < s->chunk_items.size() ? s->chunk_items[c] : std::make_pair(-1, -1));
        chk_threw.push_back(1);
      }
    }
  }
  std::vector<int32_t> v;
  std::vector<size_t> fail_chunks;  // phase-B chunks that failed, whose phase-A items phase C1 reuses
  bool reuse = true;
  if (!chk.empty()) {  // phase B
    for (auto& r : chk_items) reuse = reuse && r.first >= 0;
    // Phase B0: runs of consecutive chunks (adjacent sets and resident items) as one group
    // each, so that only the chunks of a failing run are checked on their own.  A run passes
    // only if every chunk in it would (the RLC check of its sets, the throwing sets the
    // identity as in the chunks' own groups), so each chunk's verdict -- and with it the batch
    // counters below -- is what its own check gives.  At 1 % corrupted sets about a fifth of
    // the runs of four fail: 2048 chunk checks of a 32k package become ~512 + ~460.
    std::vector<uint8_t> passed(chk.size(), 0);
    if (reuse && b0_min_chunks() > 0 && chk.size() >= b0_min_chunks()) {
      std::vector<Grp> rg;
      std::vector<std::pair<int32_t, int32_t>> ri;
      std::vector<std::pair<size_t, size_t>> rc;  // chk index range [a, b) of each run
      for (size_t c = 0; c < chk.size();) {
        size_t e = c + 1;
        while (e < chk.size() && e - c < b0_run() && chk[e].first == chk[e - 1].first + chk[e - 1].len &&
               chk_items[e].first == chk_items[e - 1].second)
          e++;
        if (e - c >= 2) {
          Grp g;
          g.first = chk[c].first;
          g.len = chk[e - 1].first + chk[e - 1].len - chk[c].first;
          rg.push_back(g);
          ri.push_back({chk_items[c].first, chk_items[e - 1].second});
          rc.push_back({c, e});
        }
        c = e;
      }
      if (!rg.empty()) {
        std::vector<int32_t> vr;
        LSG_RC(run_fallback_phase(s, lk, rg, &ri, vr));
        for (size_t k = 0; k < rg.size(); k++)
          if (vr[k])
            for (size_t c = rc[k].first; c < rc[k].second; c++) passed[c] = 1;
      }
    }
    std::vector<Grp> rest;
    std::vector<std::pair<int32_t, int32_t>> rest_items;
    std::vector<size_t> rest_of;
    for (size_t c = 0; c < chk.size(); c++)
      if (!passed[c]) {
        rest.push_back(chk[c]);
        rest_items.push_back(chk_items[c]);
        rest_of.push_back(c);
      }
    std::vector<int32_t> vb;
    LSG_RC(run_fallback_phase(s, lk, rest, reuse ? &rest_items : nullptr, vb));
    v.assign(chk.size(), 1);
    for (size_t k = 0; k < rest.size(); k++) v[rest_of[k]] = vb[k];
    for (size_t c = 0; c < chk.size(); c++) {
      if (v[c]) {
        for (size_t q = chk_jobs[c].first; q < chk_jobs[c].second; q++)
          if (!job_err[s->batch_order[q]]) s->results[s->batch_order[q]] = {LSG_VALID, 0};
        if (!chk_threw[c]) succ_add(chk_jobs[c].first, chk[c].len);
      } else {
        if (!chk_threw[c]) retry_inc(chk_jobs[c].first);
        if (reuse) {
          fail_chunks.push_back(c);
        } else {
          for (size_t q = chk_jobs[c].first; q < chk_jobs[c].second; q++)
            if (!job_err[s->batch_order[q]]) retry.push_back(s->batch_order[q]);
        }
      }
    }
  }
  // Phase C1: the jobs of a failing chunk, localised over its phase-A items.  A group is a
  // run of whole items ending on a job boundary (for single-set jobs: one item = four jobs),
  // checked with its resident items -- no new Miller work.  A passing group answers its jobs
  // (valid); a one-job group's verdict is that job's maybeBatch verdict (the same RLC check,
  // worker.ts:88-96); the jobs of a failing multi-job group are checked one by one (C2).
  // Per-job verdicts and the batch counters are unchanged: only the work is (a chunk with one
  // bad set costs 4 group checks + 4 one-set checks instead of 16 one-set checks).
  if (!fail_chunks.empty()) {
    const PhasePlan& A0 = s->phA;
    std::vector<Grp> g1;
    std::vector<std::pair<int32_t, int32_t>> g1_items;
    std::vector<std::pair<size_t, size_t>> g1_jobs;  // batch_order positions [a, b)
    for (size_t c : fail_chunks) {
      size_t q = chk_jobs[c].first;
      const size_t qe = chk_jobs[c].second;
      int32_t ia = chk_items[c].first;
      for (int32_t it = chk_items[c].first; it < chk_items[c].second; it++) {
        const size_t end = (size_t)A0.it_first[(size_t)it] + (size_t)A0.it_cnt[(size_t)it];
        // jobs of this group: those ending at or before `end`; close the group on a boundary
        size_t qb = q;
        while (qb < qe && s->jobs[s->batch_order[qb]].first + s->jobs[s->batch_order[qb]].count <= end) qb++;
        const bool boundary = qb > q && s->jobs[s->batch_order[qb - 1]].first + s->jobs[s->batch_order[qb - 1]].count == end;
        if (!boundary && it + 1 < chk_items[c].second) continue;
        Grp g;
        g.first = (size_t)A0.it_first[(size_t)ia];
        g.len = end - g.first;
        g1.push_back(g);
        g1_items.push_back({ia, it + 1});
        g1_jobs.push_back({q, qb});
        q = qb;
        ia = it + 1;
      }
      for (; q < qe; q++) retry.push_back(s->batch_order[q]);  // (not reached: items cover the chunk)
    }
    LSG_RC(run_fallback_phase(s, lk, g1, &g1_items, v));
    for (size_t g = 0; g < g1.size(); g++) {
      // A thrown job keeps its error.  Only its throwing sets are the identity in the group:
      // its other sets take part, so a failing group with one live job localises that job on
      // its own (C2) unless every other job of the group is live too.
      size_t nlive = 0;
      bool thrown = false;
      for (size_t q = g1_jobs[g].first; q < g1_jobs[g].second; q++) {
        nlive += job_err[s->batch_order[q]] ? 0 : 1;
        thrown = thrown || job_err[s->batch_order[q]];
      }
      for (size_t q = g1_jobs[g].first; q < g1_jobs[g].second; q++) {
        const size_t j = s->batch_order[q];
        if (job_err[j]) continue;
        if (v[g])
          s->results[j] = {LSG_VALID, 0};
        else if (nlive == 1 && !thrown)
          s->results[j] = {LSG_INVALID, 0};
        else
          retry.push_back(j);
      }
    }
  }
  if (!retry.empty()) {  // phase C2: one group per job
    std::vector<Grp> g3;
    std::vector<size_t> g3job;
    for (size_t j : retry) {
      const int32_t e = job_error(ss, s->jobs[j].first, s->jobs[j].count);
      if (e) {
        s->results[j] = {LSG_ERROR, e};
        continue;
      }
      Grp g;
      g.first = s->jobs[j].first;
      g.len = s->jobs[j].count;
      g3.push_back(g);
      g3job.push_back(j);
    }
    LSG_RC(run_fallback_phase(s, lk, g3, nullptr, v));
    for (size_t g = 0; g < g3.size(); g++) s->results[g3job[g]] = {v[g] ? LSG_VALID : LSG_INVALID, 0};
  }
  return LSG_OK;
}

}  // namespace

// ---------------------------------------------------------------------------- tickets
namespace {

// Whole jobs per device by cumulative set count (never splits a job): job j goes
// to floor(sets_before_j * n_dev / total).
void assign_jobs(const uint32_t* sizes, size_t n_jobs, int n_dev, int32_t* owner) {
  uint64_t total = 0;
  for (size_t j = 0; j < n_jobs; j++) total += sizes[j];
  uint64_t before = 0;
  for (size_t j = 0; j < n_jobs; j++) {
    owner[j] = (total == 0 || n_dev <= 1) ? 0 : (int32_t)std::min<uint64_t>((uint64_t)n_dev - 1, before * (uint64_t)n_dev / total);
    before += sizes[j];
  }
}

uint64_t make_ticket(lsg_ctx* c, int kind, int index, uint64_t* serial) {
  *serial = c->next_serial++;
  return (*serial << 16) | ((uint64_t)kind << 8) | (uint64_t)index;
}

// package index of a jobs ticket (slot `index` on every device), or -1
int ticket_pkg(lsg_ctx* c, uint64_t t) {
  const int k = (int)((t >> 8) & 255), i = (int)(t & 255);
  if (k != SLOT_JOBS || i >= LSG_SLOTS) return -1;
  const Slot& s = c->dev[0]->slots[i];
  if (s.kind != SLOT_JOBS || s.serial != (t >> 16)) return -1;
  return i;
}
Slot* ticket_final(lsg_ctx* c, uint64_t t) {
  const int k = (int)((t >> 8) & 255), i = (int)(t & 255);
  if (k != SLOT_FINAL || i >= LSG_FINALS) return nullptr;
  Slot* s = &c->dev[0]->finals[i];
  if (s->kind != SLOT_FINAL || s->serial != (t >> 16)) return nullptr;
  return s;
}

void sync_slot(Slot* s) {
  for (int k = 0; k < 2; k++)
    if (s->st[k]) (void)hipStreamSynchronize(s->st[k]);
}

bool force_exchange() { return lsg_ab_long("LSG_FORCE_EXCHANGE", 0) != 0; }

// all-gather of the devices' partials into device 0's d_gath, then the node check there
int pkg_exchange(lsg_ctx* c, int p) {
  const int n = c->n_dev;
  Slot* s0 = &c->dev[0]->slots[p];
  if (c->rccl) {
    // one collective over xGMI: every device contributes 576 bytes
    ncclResult_t r = ncclGroupStart();
    for (int d = 0; d < n && r == ncclSuccess; d++) {
      Slot* s = &c->dev[d]->slots[p];
      (void)hipSetDevice(c->dev[d]->device);
      r = ncclAllGather(pkg_partial_dev(s), s->d_gath.p, 576, ncclUint8, c->comm[d], s->st[0]);
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    (void)hipSetDevice(c->dev[0]->device);
    if (r != ncclSuccess) {
      set_err(c, std::string("ncclAllGather: ") + ncclGetErrorString(r));
      return LSG_ERR_DEVICE;
    }
  } else {
    // duplicate device list (tests): device-to-device copies on device 0's main stream
    (void)hipSetDevice(c->dev[0]->device);
    for (int d = 0; d < n; d++) {
      Slot* s = &c->dev[d]->slots[p];
      LSG_HIP(s0, hipStreamWaitEvent(s0->st[0], s->ev_part, 0));
      uint8_t* dst = P_<uint8_t>(s0->d_gath) + 576 * (size_t)d;
      if (c->dev[d]->device == c->dev[0]->device)
        LSG_HIP(s0, hipMemcpyAsync(dst, pkg_partial_dev(s), 576, hipMemcpyDeviceToDevice, s0->st[0]));
      else
        LSG_HIP(s0, hipMemcpyPeerAsync(dst, c->dev[0]->device, pkg_partial_dev(s), c->dev[d]->device, 576, s0->st[0]));
    }
  }
  return pkg_node_check(s0, n);
}

// Each device's share of a package (pkg_part1 .. pkg_part2), staged with the context lock
// released: device 0 on the calling thread, every other device on a thread of its own, so that
// a context over N GPUs spends one device's staging time per package instead of N (VERDICT r5
// item 3), and host threads submitting packages to different slots stage them side by side.
// Errors go to *err (t_err_sink), not to c->err.
int stage_pkg(lsg_ctx* c, int p, const lsg_job* jobs, size_t n_jobs, uint64_t seed, bool lone_ok, bool exch,
              std::string* err) {
  const int n = c->n_dev;
  std::vector<std::vector<size_t>> ids(n);
  {
    std::vector<uint32_t> sizes(n_jobs);
    std::vector<int32_t> owner(n_jobs);
    for (size_t j = 0; j < n_jobs; j++) sizes[j] = jobs[j].n_sets;
    assign_jobs(sizes.data(), n_jobs, n, owner.data());
    for (size_t j = 0; j < n_jobs; j++) ids[(size_t)owner[j]].push_back(j);
  }
  std::vector<int> rcs(n, LSG_OK);
  std::vector<std::string> errs(n);
  auto part1 = [&](int d) {
    t_err_sink = &errs[d];
    (void)hipSetDevice(c->dev[d]->device);
    // distinct seeds per device for tests; 0 stays 0 (OS CSPRNG on every device)
    const uint64_t sd = seed ? seed + 0x9e3779b97f4a7c15ull * (uint64_t)d : 0;
    rcs[d] = pkg_part1(&c->dev[d]->slots[p], jobs, ids[d], sd, (d == 0 && exch) ? n : 0, nullptr, lone_ok && !exch);
    t_err_sink = nullptr;
  };
  auto part2 = [&](int d) {
    t_err_sink = &errs[d];
    (void)hipSetDevice(c->dev[d]->device);
    rcs[d] = pkg_part2(&c->dev[d]->slots[p], exch);
    t_err_sink = nullptr;
  };
  // first error in device order
  auto first_rc = [&]() {
    for (int d = 0; d < n; d++)
      if (rcs[d]) {
        *err = errs[d];
        return rcs[d];
      }
    return (int)LSG_OK;
  };
  std::shared_lock<std::shared_mutex> tab(c->tab_mu);  // (the sets may name table rows)
  int rc = LSG_OK;
  // A/B build: LSG_STAGE_PAR=0 stages the devices one after another (round 5), 1 runs part 1
  // on threads and part 2 serially, 2 (shipped) both on threads
  const long par = n == 1 ? 0 : lsg_ab_long("LSG_STAGE_PAR", 2);
  if (par == 0) {
    for (int d = 0; d < n && !rc; d++) {
      part1(d);
      rc = first_rc();
    }
    if (!rc && exch) {
      std::lock_guard<std::mutex> x(c->xmu);
      t_err_sink = err;
      rc = pkg_exchange(c, p);
      t_err_sink = nullptr;
    }
    for (int d = 0; d < n && !rc; d++) {
      part2(d);
      rc = first_rc();
    }
    return rc;
  }
  // devices 1..n-1 on threads of their own: part 1, then (after the exchange, which needs every
  // device's partial) part 2
  std::mutex m;
  std::condition_variable cv;
  int n_part1 = 1;  // devices done with part 1 (device 0 counted when it is)
  int phase2 = 0;   // 1: run part 2, -1: stop (an error before the exchange or in it)
  std::vector<std::thread> th;
  for (int d = 1; d < n; d++)
    th.emplace_back([&, d] {
      part1(d);
      std::unique_lock<std::mutex> l(m);
      n_part1++;
      cv.notify_all();
      cv.wait(l, [&] { return phase2 != 0; });
      const bool go = phase2 > 0 && par >= 2;
      l.unlock();
      if (go) part2(d);
    });
  part1(0);
  {
    std::unique_lock<std::mutex> l(m);
    cv.wait(l, [&] { return n_part1 == n; });
  }
  rc = first_rc();
  if (!rc && exch) {
    std::lock_guard<std::mutex> x(c->xmu);  // one exchange at a time over the communicators
    t_err_sink = err;
    rc = pkg_exchange(c, p);
    t_err_sink = nullptr;
  }
  {
    std::lock_guard<std::mutex> l(m);
    phase2 = rc ? -1 : 1;
  }
  cv.notify_all();
  if (!rc) part2(0);
  for (int d = 1; d < n && !rc && par < 2; d++) {
    part2(d);
    rc = first_rc();
  }
  for (auto& t : th) t.join();
  if (!rc) rc = first_rc();
  return rc;
}

// A package: its slot is reserved on every device under the context lock (`lk`, held on entry
// and on return), staged with the lock released (stage_pkg), and its ticket committed under the
// lock again.  A reserved slot is SLOT_STAGING: no other call takes, reserves or waits on it.
int submit_pkg(lsg_ctx* c, CtxLock& lk, const lsg_job* jobs, size_t n_jobs, uint64_t seed, lsg_ticket* ticket,
               bool lone_ok = true) {
  int p = -1;
  for (int i = 0; i < LSG_SLOTS && p < 0; i++)
    if (c->dev[0]->slots[i].kind == SLOT_FREE) p = i;
  if (p < 0) {
    c->err = "all pipeline slots are busy (wait on an outstanding ticket first)";
    return LSG_ERR_BUSY;
  }
  const int n = c->n_dev;
  const bool exch = n > 1 || force_exchange();
  bool prio = false;
  for (size_t j = 0; j < n_jobs; j++) prio = prio || (jobs[j].flags & LSG_JOB_PRIORITY) != 0;
  for (int d = 0; d < n; d++) {
    (void)hipSetDevice(c->dev[d]->device);
    LSG_RC(slot_ready(c->dev[d], &c->dev[d]->slots[p], p));
    LSG_RC(slot_streams(&c->dev[d]->slots[p], prio));
  }
  for (int d = 0; d < n; d++) c->dev[d]->slots[p].kind = SLOT_STAGING;
  c->staging++;
  lk.unlock();
  std::string err;
  const int rc = stage_pkg(c, p, jobs, n_jobs, seed, lone_ok, exch, &err);
  lk.lock();
  (void)hipSetDevice(c->dev[0]->device);
  c->staging--;
  c->cv.notify_all();
  if (rc) {
    for (int d = 0; d < n; d++) {
      sync_slot(&c->dev[d]->slots[p]);
      c->dev[d]->slots[p].kind = SLOT_FREE;
    }
    c->err = err;
    return rc;
  }
  uint64_t serial;
  *ticket = make_ticket(c, SLOT_JOBS, p, &serial);
  for (int d = 0; d < n; d++) {
    Slot* s = &c->dev[d]->slots[p];
    s->kind = SLOT_JOBS;
    s->serial = serial;
  }
  c->dev[0]->slots[p].n_jobs = n_jobs;
  c->dev[0]->slots[p].stats.submit_us = (uint32_t)((now_ns() - c->dev[0]->slots[p].stats.start_ns) / 1000);
  return LSG_OK;
}

// resolve a package: node_valid as pkg_resolve (-2: the ticket's own node check)
int wait_pkg(lsg_ctx* c, CtxLock* lk, int p, int node_valid, lsg_job_result* results, lsg_stats* stats) {
  const int n = c->n_dev;
  int rc = LSG_OK;
  for (int d = 0; d < n && !rc; d++) {
    Slot* s = &c->dev[d]->slots[p];
    (void)hipSetDevice(c->dev[d]->device);
    if (event_wait(s->ev_done) != hipSuccess) rc = fail(s, "hipEventSynchronize", hipGetLastError());
  }
  Slot* s0 = &c->dev[0]->slots[p];
  // the ticket's own node check (lsg_init_devices) decides the package groups: 2 = passed
  if (!rc && node_valid == -2) node_valid = s0->has_node ? (H_<int32_t>(s0->h_nodeV)[0] ? 2 : 0) : -1;
  lsg_stats total;
  memset(&total, 0, sizeof(total));
  total.start_ns = s0->stats.start_ns;
  total.submit_us = s0->stats.submit_us;
  int32_t pkfail = 0;  // package-wide: the first bad key in caller job order over all devices
  size_t pkfail_job = SIZE_MAX;
  for (int d = 0; d < n && !rc; d++) {
    size_t j = SIZE_MAX;
    const int32_t e = first_pk_error(&c->dev[d]->slots[p], &j);
    if (e && j < pkfail_job) {
      pkfail = e;
      pkfail_job = j;
    }
  }
  for (int d = 0; d < n && !rc; d++) {
    Slot* s = &c->dev[d]->slots[p];
    (void)hipSetDevice(c->dev[d]->device);
    rc = pkg_resolve(s, lk, node_valid, pkfail);
    if (rc) break;
    for (size_t k = 0; k < s->jobs.size(); k++) results[s->job_ids[k]] = s->results[k];
    total.batch_retries += s->stats.batch_retries;
    total.batch_sigs_success += s->stats.batch_sigs_success;
    total.n_final_exps += s->stats.n_final_exps;
  }
  if (s0->has_node) total.n_final_exps += 1;
  total.key_error = pkfail;
  total.key_error_job = pkfail ? (uint32_t)pkfail_job : 0;
  total.end_ns = now_ns();
  if (stats) *stats = total;
  for (int d = 0; d < n; d++) {
    Slot* s = &c->dev[d]->slots[p];
    if (rc) sync_slot(s);
    s->kind = SLOT_FREE;
    keep_times(s);
  }
  (void)hipSetDevice(c->dev[0]->device);
  return rc;
}

// ---- coalesced launches (lsg_set_coalesce)
PendingPkg copy_pkg(const lsg_job* jobs, size_t n_jobs, uint64_t seed) {
  PendingPkg pk;
  pk.seed = seed;
  size_t ns = 0, nb = 0;
  for (size_t j = 0; j < n_jobs; j++)
    for (uint32_t q = 0; q < jobs[j].n_sets; q++) {
      const lsg_set& t = jobs[j].sets[q];
      ns++;
      nb += (t.pks ? (size_t)t.n_pks * (t.pk_len == LSG_PK_INDEX ? 4 : t.pk_len) : 0) + (t.msg ? t.msg_len : 0) +
            (t.sig ? t.sig_len : 0);
    }
  pk.n_sets = ns;
  pk.sets.resize(ns);
  pk.data.resize(std::max(nb, (size_t)1));
  pk.jobs.assign(jobs, jobs + n_jobs);
  size_t si = 0, off = 0;
  auto put = [&](const uint8_t* src, size_t len) -> const uint8_t* {
    if (!src) return nullptr;
    uint8_t* d = pk.data.data() + off;
    if (len) memcpy(d, src, len);
    off += len;
    return d;
  };
  for (size_t j = 0; j < n_jobs; j++) {
    pk.jobs[j].sets = pk.sets.data() + si;
    for (uint32_t q = 0; q < jobs[j].n_sets; q++, si++) {
      lsg_set t = jobs[j].sets[q];
      t.pks = put(t.pks, t.pks ? (size_t)t.n_pks * (t.pk_len == LSG_PK_INDEX ? 4 : t.pk_len) : 0);
      t.msg = put(t.msg, t.msg ? t.msg_len : 0);
      t.sig = put(t.sig, t.sig ? t.sig_len : 0);
      pk.sets[si] = t;
    }
  }
  return pk;
}

// launches still executing on the device (their completion event not reached): a launch
// whose work is done no longer holds packages back, whether or not its tickets were waited on
int launches_in_flight(lsg_ctx* c) {
  int n = 0;
  for (int i = 0; i < LSG_SLOTS; i++) {
    const Slot& s = c->dev[0]->slots[i];
    n += s.kind == SLOT_JOBS && hipEventQuery(s.ev_done) == hipErrorNotReady ? 1 : 0;
  }
  return n;
}

// the pending packages as one launch: one slot, each package a sub-package with its own
// chunks, deserialisation rule and counters (context lock held)
int flush_pending(lsg_ctx* c) {
  if (c->pending.empty()) return LSG_OK;
  int p = -1;
  for (int i = 0; i < LSG_SLOTS && p < 0; i++)
    if (c->dev[0]->slots[i].kind == SLOT_FREE) p = i;
  if (p < 0) {
    c->err = "all pipeline slots are busy (wait on an outstanding ticket first)";
    return LSG_ERR_BUSY;
  }
  Slot* s = &c->dev[0]->slots[p];
  LSG_RC(slot_ready(c->dev[0], s, p));
  LSG_RC(slot_streams(s, false));
  std::vector<lsg_job> all;
  std::vector<size_t> subs{0};
  uint64_t seed = c->pending[0].seed;
  for (auto& pk : c->pending) {
    all.insert(all.end(), pk.jobs.begin(), pk.jobs.end());
    subs.push_back(all.size());
    if (!pk.seed) seed = 0;  // any package asking for OS randomness gets it for all
  }
  std::vector<size_t> ids(all.size());
  for (size_t j = 0; j < ids.size(); j++) ids[j] = j;
  int rc = pkg_part1(s, all.data(), ids, seed, 0, &subs);
  if (!rc) rc = pkg_part2(s);
  if (rc) {
    sync_slot(s);
    // every held package's wait (or poll) reports this failure -- its code and message --
    // instead of an unknown ticket; the entry goes when its ticket is waited on
    for (auto& pk : c->pending) {
      MergeTicket& m = c->merged[pk.serial];
      m.slot = -1;
      m.rc = rc;
      m.err = c->err;
    }
    c->pending.clear();
    c->pending_sets = 0;
    return rc;
  }
  uint64_t serial;
  (void)make_ticket(c, SLOT_JOBS, p, &serial);
  s->kind = SLOT_JOBS;
  s->serial = serial;
  s->n_jobs = all.size();
  s->sub_serial.clear();
  for (size_t k = 0; k < c->pending.size(); k++) {
    s->sub_serial.push_back(c->pending[k].serial);
    c->merged[c->pending[k].serial] = MergeTicket{p, (int)k};
  }
  s->stats.submit_us = (uint32_t)((now_ns() - s->stats.start_ns) / 1000);
  c->pending.clear();
  c->pending_sets = 0;
  return LSG_OK;
}

// launch what is pending when the device has room (after a wait freed a slot)
void maybe_flush(lsg_ctx* c) {
  if (!c->pending.empty() && launches_in_flight(c) < c->co_inflight) (void)flush_pending(c);
}

int submit_merged(lsg_ctx* c, const lsg_job* jobs, size_t n_jobs, uint64_t seed, size_t n_sets, lsg_ticket* ticket) {
  if (c->pending_sets + n_sets > c->co_max_pending) LSG_RC(flush_pending(c));
  PendingPkg pk = copy_pkg(jobs, n_jobs, seed);
  uint64_t serial;
  *ticket = make_ticket(c, SLOT_MERGE, 0, &serial);
  pk.serial = serial;
  c->merged[serial] = MergeTicket{};
  c->pending.push_back(std::move(pk));
  c->pending_sets += n_sets;
  if (launches_in_flight(c) < c->co_inflight) {
    const int rc = flush_pending(c);
    if (rc && rc != LSG_ERR_BUSY) {  // (busy: it stays pending, a later wait launches it)
      c->merged.erase(serial);       // this submission fails; the others' waits report rc
      return rc;
    }
  }
  return LSG_OK;
}

int wait_merged(lsg_ctx* c, lsg_ticket t, lsg_job_result* results, lsg_stats* stats) {
  const uint64_t serial = t >> 16;
  int p, k;
  hipEvent_t ev;
  for (int spin = 0;; spin++) {
    std::unique_lock<std::mutex> lk(c->mu);
    LSG_HIPC(c, hipSetDevice(c->dev[0]->device));
    auto it = c->merged.find(serial);
    if (it == c->merged.end()) return LSG_ERR_INVALID_ARG;
    if (it->second.slot >= 0 || it->second.rc) break;  // launched (or its launch failed)
    // still held: it goes out with whatever else is pending once fewer than co_inflight launches
    // execute -- packages submitted meanwhile join it (a waiter forcing the flush at once left
    // two packages per launch on the gossip bench) -- or at once if the device is idle
    if (launches_in_flight(c) >= c->co_inflight) {
      lk.unlock();
      std::this_thread::sleep_for(std::chrono::microseconds(spin < 20 ? 50 : 200));
      continue;
    }
    const int frc = flush_pending(c);
    it = c->merged.find(serial);
    if (it == c->merged.end()) return LSG_ERR_INVALID_ARG;
    // still held (every slot busy: LSG_ERR_BUSY, c->err says so): the ticket stays live and a
    // later wait -- after the caller has waited on another ticket -- launches it
    if (frc && it->second.slot < 0 && !it->second.rc) return frc;
    break;
  }
  {
    std::lock_guard<std::mutex> lk(c->mu);
    LSG_HIPC(c, hipSetDevice(c->dev[0]->device));
    auto it = c->merged.find(serial);
    if (it == c->merged.end()) return LSG_ERR_INVALID_ARG;
    if (it->second.rc) {  // its coalesced launch failed
      const int frc = it->second.rc;
      c->err = it->second.err;
      c->merged.erase(it);
      return frc;
    }
    if (it->second.slot < 0) return LSG_ERR_INVALID_ARG;
    p = it->second.slot;
    k = it->second.sub;
    ev = c->dev[0]->slots[p].ev_done;
  }
  const hipError_t wr = event_wait(ev);
  CtxLock lk(c->mu);
  if (wr != hipSuccess) return fail_c(c, "hipEventSynchronize", wr);
  LSG_HIPC(c, hipSetDevice(c->dev[0]->device));
  Slot* s = &c->dev[0]->slots[p];
  c->cv.wait(lk, [&] { return !s->resolving; });
  if (!s->resolved) {  // the first waiter resolves every sub-package (fallback phases included)
    s->resolving = true;
    s->resolve_rc = pkg_resolve(s, &lk, -1, 0);
    s->resolved = true;
    s->resolving = false;
    c->cv.notify_all();
  }
  const int rc = s->resolve_rc;
  for (size_t j = s->sub_first[k]; j < s->sub_first[k + 1]; j++) results[j - s->sub_first[k]] = s->results[j];
  if (stats) {
    *stats = s->sub_stats[k];
    stats->start_ns = s->stats.start_ns;
    stats->submit_us = s->stats.submit_us;
    stats->n_final_exps = s->stats.n_final_exps;  // (the whole coalesced launch)
    stats->end_ns = now_ns();
  }
  c->merged.erase(serial);
  s->sub_done[k] = 1;
  bool all = true;
  for (uint8_t d : s->sub_done) all = all && d;
  if (all) {
    if (rc) sync_slot(s);
    s->kind = SLOT_FREE;
    s->n_sub = 0;
    keep_times(s);
    maybe_flush(c);
  }
  return rc;
}

#define LSG_ENTER(c)                         \
  std::lock_guard<std::mutex> _lk((c)->mu); \
  LSG_HIPC((c), hipSetDevice((c)->dev[0]->device))

// Block until a ticket's device work is done WITHOUT holding the context mutex, so a waiter
// (e.g. an N-API worker thread) never stalls submissions from another thread.  The ticket's
// slots cannot be recycled meanwhile: only the ticket's own wait call releases them.
int presync_pkg(lsg_ctx* c, lsg_ticket t, bool partial_only) {
  std::vector<std::pair<int, hipEvent_t>> evs;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    const int p = ticket_pkg(c, t);
    if (p < 0) return LSG_ERR_INVALID_ARG;
    for (int d = 0; d < c->n_dev; d++) {
      Slot* s = &c->dev[d]->slots[p];
      evs.push_back({c->dev[d]->device, partial_only ? s->ev_part : s->ev_done});
    }
  }
  for (auto& e : evs) {
    (void)hipSetDevice(e.first);
    hipError_t r = event_wait(e.second);
    if (r != hipSuccess) {
      std::lock_guard<std::mutex> lk(c->mu);
      return fail_c(c, "hipEventSynchronize", r);
    }
  }
  return LSG_OK;
}

// ---- final-exponentiation entries (device 0): ng groups of pg partials
int submit_final(Slot* s, const uint8_t* partials576, size_t ng, size_t pg, bool on_device = false) {
  timer_reset(s);
  s->plan.clear();
  const size_t n = ng * pg, np = std::max(n, (size_t)1), gq = std::max(ng, (size_t)1);
  LSG_RC(ensure_host(s, s->h_blob, 576 * np));
  LSG_RC(ensure(s, s->d_Fb, 576 * std::max(np, gq)));
  LSG_RC(ensure(s, s->d_aux, 4 * W_F12 * np));
  LSG_RC(ensure(s, s->d_F, 4 * W_F12 * gq));
  LSG_RC(ensure(s, s->d_verdict, 4 * gq));
  LSG_RC(ensure_host(s, s->h_verdict, 4 * gq));
  s->n_sets = ng;  // verdict count
  if (n) {
    std::vector<int32_t> off, len;
    for (size_t g = 0; g < ng; g++) {
      off.push_back((int32_t)(g * pg));
      len.push_back((int32_t)pg);
    }
    SegPlan P = plan_seg(s->plan, 2, off, len, false, 0, 0);
    LSG_RC(upload_plan(s));
    hipStream_t S = s->st[0];
    if (on_device) {  // the caller's device buffer (e.g. a collective's output): no host copy
      LSG_HIP(s, hipMemcpyAsync(s->d_Fb.p, partials576, 576 * n, hipMemcpyDeviceToDevice, S));
    } else {
      memcpy(s->h_blob.p, partials576, 576 * n);
      LSG_HIP(s, hipMemcpyAsync(s->d_Fb.p, s->h_blob.p, 576 * n, hipMemcpyHostToDevice, S));
    }
    KL(s, "k_blobs_to_fp12", lsgk::blobs_to_fp12(S, (int)n, P_<uint8_t>(s->d_Fb), P_<uint32_t>(s->d_aux)));
    LSG_RC(run_seg(s, 2, "fp12_product", P, P_<uint32_t>(s->d_aux), P_<uint32_t>(s->d_F)));
    KL(s, "k_fp12_to_canon", lsgk::fp12_to_canon(S, (int)ng, P_<uint32_t>(s->d_F), P_<uint8_t>(s->d_Fb)));
    KL(s, SERIAL_LABEL(final_exp), lsg_row_final_exp(S, (int)ng, P_<uint8_t>(s->d_Fb), P_<int32_t>(s->d_verdict)));
    LSG_HIP(s, hipMemcpyAsync(s->h_verdict.p, s->d_verdict.p, 4 * ng, hipMemcpyDeviceToHost, S));
  } else {
    s->n_sets = 0;
  }
  LSG_HIP(s, hipEventRecord(s->ev_done, s->st[0]));
  return LSG_OK;
}

// stage + expand + hash on the utility slot (synchronous callers only)
int util_hash(Slot* s, const uint8_t* msgs, uint32_t msg_len, size_t n, const uint8_t* dst, uint32_t dst_len) {
  std::vector<lsg_set> sets(n);
  std::vector<const lsg_set*> sp(n);
  for (size_t i = 0; i < n; i++) {
    memset(&sets[i], 0, sizeof(lsg_set));
    sets[i].msg = msgs + (size_t)msg_len * i;
    sets[i].msg_len = msg_len;
    sp[i] = &sets[i];
  }
  LSG_RC(stage_sets(s, sp.data(), n, 0, false));
  LSG_RC(size_state(s, n, 0, 1, 0));
  LSG_HIP(s, hipMemcpyAsync(s->d_dst.p, dst, dst_len, hipMemcpyHostToDevice, s->st[0]));
  const int nn = (int)n;
  KL(s, "k_expand_msg", lsgk::expand_msg(S_(s), nn, P_<uint8_t>(s->d_msg), P_<uint32_t>(s->d_msgoff),
                                         P_<uint32_t>(s->d_msglen), P_<uint8_t>(s->d_dst), dst_len, P_<uint8_t>(s->d_ub)));
  LSG_RC(launch_hash(s, nn, P_<uint32_t>(s->d_H), P_<uint8_t>(s->d_hinf)));
  // the utility slot's DST is restored for the next caller
  LSG_HIP(s, hipMemcpyAsync(s->d_dst.p, DST_POP, DST_POP_LEN, hipMemcpyHostToDevice, s->st[0]));
  return LSG_OK;
}

// keys (one "set" of n keys) into the utility slot's arena, decoded on its stream
int util_stage_keys(Slot* s, const uint8_t* pks, uint32_t pk_len, size_t n) {
  lsg_set q;
  memset(&q, 0, sizeof(q));
  q.pks = pks;
  q.pk_len = pk_len;
  q.n_pks = (uint32_t)n;
  const lsg_set* qp = &q;
  LSG_RC(stage_sets(s, &qp, 1, 0, false));
  return size_state(s, 1, n, 1, 0);
}

int dev_create(lsg_ctx* c, int ord, int device, Dev** out) {
  Dev* d = new Dev();
  *out = d;
  d->c = c;
  d->device = device;
  d->ord = ord;
  LSG_HIPC(c, hipSetDevice(device));
  LSG_HIPC(c, hipStreamCreateWithFlags(&d->s_util, hipStreamNonBlocking));
  // pipeline slots are created on first use (slot_ready): 64 x 2 streams per device up front
  // would cost init time nobody needs below a few packages in flight
  if (ord == 0) {
    for (int i = 0; i < LSG_FE_STREAMS; i++) LSG_HIPC(c, hipStreamCreateWithFlags(&d->s_fe[i], hipStreamNonBlocking));
    for (int i = 0; i < LSG_FINALS; i++) LSG_RC(slot_create(d, &d->finals[i], i, d->s_fe[i % LSG_FE_STREAMS]));
  }
  return slot_create(d, &d->util, 0, d->s_util);
}

void dev_destroy(Dev* d) {
  if (!d) return;
  (void)hipSetDevice(d->device);
  for (Slot& s : d->slots) slot_destroy(&s);
  for (Slot& s : d->finals) slot_destroy(&s);
  slot_destroy(&d->util);
  free_dev(d->d_pktab);
  free_dev(d->d_pktab_ok);
  if (d->s_util) (void)hipStreamDestroy(d->s_util);
  for (hipStream_t st : d->s_fe)
    if (st) (void)hipStreamDestroy(st);
  if (d->s_xp) (void)hipStreamDestroy(d->s_xp);
  if (d->s_nfe) (void)hipStreamDestroy(d->s_nfe);
  for (hipStream_t st : d->s_pp)
    if (st) (void)hipStreamDestroy(st);
  delete d;
}

// pubkey table rows first .. first+n-1 on one device
int dev_pktab_set(Dev* d, size_t first, const uint8_t* pks, uint32_t pk_len, size_t n, std::vector<int32_t>& pkerr) {
  lsg_ctx* c = d->c;
  Slot* s = &d->util;
  timer_reset(s);
  LSG_HIPC(c, hipSetDevice(d->device));
  const size_t need = first + n;
  // tickets in flight read the table: drain the device before moving it or rewriting rows
  // that may be read (an in-flight aggregate must never see a half-written row)
  if (need > d->pktab_cap || first < d->pktab_n) LSG_HIPC(c, hipDeviceSynchronize());
  if (need > d->pktab_cap) {
    const size_t cap = std::max(std::max(need, 2 * d->pktab_cap), (size_t)1024);
    DevBuf nt, nok;
    LSG_HIPC(c, hipMalloc(&nt.p, 4 * W_TAB * cap));
    g_allocs++;
    nt.cap = 4 * W_TAB * cap;
    hipError_t e = hipMalloc(&nok.p, cap);
    if (e != hipSuccess) {
      free_dev(nt);
      return fail_c(c, "hipMalloc", e);
    }
    g_allocs++;
    nok.cap = cap;
    LSG_HIPC(c, hipMemset(nok.p, 0, cap));
    if (d->pktab_n) {
      LSG_HIPC(c, hipMemcpy(nt.p, d->d_pktab.p, 4 * W_TAB * d->pktab_n, hipMemcpyDeviceToDevice));
      LSG_HIPC(c, hipMemcpy(nok.p, d->d_pktab_ok.p, d->pktab_n, hipMemcpyDeviceToDevice));
    }
    free_dev(d->d_pktab);
    free_dev(d->d_pktab_ok);
    d->d_pktab = nt;
    d->d_pktab_ok = nok;
    d->pktab_cap = cap;
  }
  LSG_RC(util_stage_keys(s, pks, pk_len, n));
  // decode straight into the table rows first .. first + n - 1: affine points (the first
  // level of the aggregation tree reads them as they are), row flag 1 = a finite key, 2 = the
  // infinity key, 0 = no key
  LSG_RC(ensure(s, s->d_ub, n));
  KL(s, "k_pk_gather_aff", lsgk::pk_gather_aff(S_(s), (int)n, P_<uint8_t>(s->d_pk), s->pk_stride,
                                               P_<uint32_t>(s->d_pklen), P_<uint32_t>(d->d_pktab) + W_TAB * first,
                                               P_<uint8_t>(s->d_ub), P_<int32_t>(s->d_pkerr), nullptr, nullptr, 0u));
  pkerr.assign(n, 0);
  std::vector<uint8_t> inf(n);
  LSG_HIP(s, hipMemcpyAsync(pkerr.data(), s->d_pkerr.p, 4 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipMemcpyAsync(inf.data(), s->d_ub.p, n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  std::vector<uint8_t> ok(n);
  for (size_t k = 0; k < n; k++) ok[k] = pkerr[k] != 0 ? 0 : (inf[k] ? 2 : 1);
  LSG_HIP(s, hipMemcpy(P_<uint8_t>(d->d_pktab_ok) + first, ok.data(), n, hipMemcpyHostToDevice));
  d->pktab_n = std::max(d->pktab_n, need);
  keep_times(s);
  return LSG_OK;
}

}  // namespace

// ---------------------------------------------------------------------------- C ABI
extern "C" {

int lsg_init_devices(const int* device_ids, int n_devices, lsg_ctx** out) {
  if (!out || !device_ids || n_devices < 1 || n_devices > LSG_MAX_DEVICES) return LSG_ERR_INVALID_ARG;
  *out = nullptr;
  // A package keeps two streams busy and up to LSG_SLOTS packages are in flight: HIP's default
  // of 4 hardware queues per process serialises them (profiles/r05_hwq_ab.txt).  The library
  // owns this setting: before its first HIP call it sets GPU_MAX_HW_QUEUES to LSG_HW_QUEUES
  // (1..32, default LSG_DEFAULT_HW_QUEUES), overriding a process-wide default such as the
  // GPU_MAX_HW_QUEUES=4 some hosts export.  It takes effect when HIP is not yet initialised --
  // the first lsg_init of a Node process; INTEGRATION.md section 5.
  // setenv is not safe against getenv on other threads: a host calls lsg_init before it
  // starts threads that read the environment.  A value already in the
  // environment is replaced, and said so once: if HIP was initialised before (by another
  // library), the replacement comes too late to take effect.
  static std::once_flag hwq_once;
  std::call_once(hwq_once, [] {
    const char* want = getenv("LSG_HW_QUEUES");
    const int q = want ? atoi(want) : 0;
    const char* v = (q >= 1 && q <= 32) ? want : LSG_DEFAULT_HW_QUEUES;
    const char* had = getenv("GPU_MAX_HW_QUEUES");
    if (had && strcmp(had, v) != 0)
      fprintf(stderr, "lodestar_bls: GPU_MAX_HW_QUEUES=%s replaced by %s (LSG_HW_QUEUES); effective unless HIP was "
                      "initialised earlier in this process\n", had, v);
    setenv("GPU_MAX_HW_QUEUES", v, 1);
  });
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return LSG_ERR_NO_DEVICE;
  bool distinct = true;
  for (int i = 0; i < n_devices; i++) {
    const int dev = device_ids[i];
    if (dev < 0 || dev >= count) return LSG_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return LSG_ERR_NO_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return LSG_ERR_NO_DEVICE;
    for (int j = 0; j < i; j++)
      if (device_ids[j] == dev) distinct = false;
  }
  lsg_ctx* c = new lsg_ctx();
  c->n_dev = n_devices;
  int rc = LSG_OK;
  for (int i = 0; i < n_devices && !rc; i++) rc = dev_create(c, i, device_ids[i], &c->dev[i]);
  if (!rc && distinct && (n_devices > 1 || force_exchange())) {
    // the partial exchange of SURVEY.md 8e: one RCCL communicator per device, owned here
    ncclResult_t r = ncclCommInitAll(c->comm, n_devices, device_ids);
    if (r != ncclSuccess) {
      c->err = std::string("ncclCommInitAll: ") + ncclGetErrorString(r);
      rc = LSG_ERR_DEVICE;
    } else {
      c->rccl = true;
    }
  }
  (void)hipSetDevice(device_ids[0]);
  if (rc) {
    lsg_destroy(c);
    return rc;
  }
  *out = c;
  return LSG_OK;
}

int lsg_init(int device_ordinal, lsg_ctx** out) {
  const int dev = device_ordinal < 0 ? 0 : device_ordinal;
  return lsg_init_devices(&dev, 1, out);
}

int lsg_destroy(lsg_ctx* c) {
  if (!c) return LSG_ERR_INVALID_ARG;
  for (int d = 0; d < c->n_dev; d++) dev_destroy(c->dev[d]);
  if (c->rccl)
    for (int d = 0; d < c->n_dev; d++)
      if (c->comm[d]) (void)ncclCommDestroy(c->comm[d]);
  delete c;
  return LSG_OK;
}

int lsg_device_count(lsg_ctx* c, int32_t* n) {
  if (!c || !n) return LSG_ERR_INVALID_ARG;
  *n = c->n_dev;
  return LSG_OK;
}

// a copy per calling thread: another thread's failing call may replace c->err meanwhile
const char* lsg_last_error(lsg_ctx* c) {
  if (!c) return "null context";
  thread_local std::string copy;
  std::lock_guard<std::mutex> lk(c->mu);
  copy = c->err;
  return copy.c_str();
}

int lsg_device_name(lsg_ctx* c, char* buf, size_t len) {
  if (!c || !buf || !len) return LSG_ERR_INVALID_ARG;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->dev[0]->device) != hipSuccess) return LSG_ERR_DEVICE;
  snprintf(buf, len, "%s (%s, %d CUs)%s", prop.name, prop.gcnArchName, prop.multiProcessorCount,
           c->n_dev > 1 ? " x several" : "");
  return LSG_OK;
}

int lsg_reserve(lsg_ctx* c, size_t max_sets, size_t max_pks, size_t max_msg_bytes, int32_t n_slots) {
  if (!c || n_slots < 0) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  const int ns = std::min(n_slots == 0 ? LSG_SLOTS : n_slots, LSG_SLOTS);
  if (c->n_dev > 1) {
    // a device stages its share of a package: whole jobs by cumulative set count (assign_jobs),
    // so at most 1/n of the sets plus one job's -- reserved with a job's worth of slack (a larger
    // share grows its slot's buffers when it comes)
    const size_t n = (size_t)c->n_dev;
    max_sets = std::min(max_sets, max_sets / n + 4096);
    max_pks = std::min(max_pks, max_pks / n + 4096 * 512);
    max_msg_bytes = std::min(max_msg_bytes, max_msg_bytes / n + 4096 * 32);
  }
  for (int d = 0; d < c->n_dev; d++) {
    LSG_HIPC(c, hipSetDevice(c->dev[d]->device));
    for (int i = 0; i < ns; i++) {
      Slot* s = &c->dev[d]->slots[i];
      if (s->kind != SLOT_FREE) continue;
      LSG_RC(slot_ready(c->dev[d], s, i));
      LSG_RC(size_inputs(s, max_sets, max_pks, max_msg_bytes));
      // groups: as many as sets (the per-job phase of a failing package of single-set jobs)
      LSG_RC(size_state(s, max_sets, max_pks, max_sets, max_sets / 256 + 1, 1));
      LSG_RC(ensure_host(s, s->h_mode, std::max(max_sets, (size_t)1)));
      const size_t plan_words = 16 * max_sets + 4 * max_pks + 64 * 1024;
      LSG_RC(ensure_host(s, s->h_plan, 4 * plan_words));
      LSG_RC(ensure(s, s->d_plan, 4 * plan_words));
      s->plan.reserve(plan_words);
      for (int u = 0; u < 3; u++) {
        const size_t W = u == 0 ? W_G1P : (u == 1 ? W_G2P : W_F12);
        const size_t items = std::max(max_sets / 8 + 64, std::max(max_pks, max_sets) / 8 + 64);
        for (int k = 0; k < 2; k++) LSG_RC(ensure(s, s->seg_tmp[u][k], 4 * W * items));
      }
      // timing events for a full submission, created up front
      while (s->timers.size() < 192) {
        Timer t;
        LSG_HIPC(c, hipEventCreate(&t.a));
        LSG_HIPC(c, hipEventCreate(&t.b));
        s->timers.push_back(t);
      }
    }
  }
  LSG_HIPC(c, hipSetDevice(c->dev[0]->device));
  return LSG_OK;
}

int lsg_allocation_count(lsg_ctx* c, uint64_t* n) {
  if (!c || !n) return LSG_ERR_INVALID_ARG;
  *n = g_allocs.load();
  return LSG_OK;
}

int lsg_submit_jobs(lsg_ctx* c, const lsg_job* jobs, size_t n_jobs, uint64_t seed, lsg_ticket* ticket) {
  if (!c || !ticket || (n_jobs && !jobs)) return LSG_ERR_INVALID_ARG;
  for (size_t j = 0; j < n_jobs; j++)
    if (jobs[j].n_sets && !jobs[j].sets) return LSG_ERR_INVALID_ARG;
  CtxLock lk(c->mu);
  LSG_HIPC(c, hipSetDevice(c->dev[0]->device));
  bool prio = false;
  for (size_t j = 0; j < n_jobs; j++) prio = prio || (jobs[j].flags & LSG_JOB_PRIORITY) != 0;
  if (c->co_max_sets && c->n_dev == 1 && !prio) {  // (a priority package is never held back)
    size_t ns = 0;
    for (size_t j = 0; j < n_jobs; j++) ns += jobs[j].n_sets;
    if (ns <= c->co_max_sets) return submit_merged(c, jobs, n_jobs, seed, ns, ticket);
  }
  return submit_pkg(c, lk, jobs, n_jobs, seed, ticket);
}

int lsg_set_coalesce(lsg_ctx* c, uint32_t max_sets, int32_t max_inflight) {
  if (!c || max_inflight < 1) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  LSG_RC(flush_pending(c));
  c->co_max_sets = max_sets;
  c->co_inflight = max_inflight;
  return LSG_OK;
}

int lsg_wait_jobs_node(lsg_ctx* c, lsg_ticket ticket, int32_t node_valid, lsg_job_result* results, lsg_stats* stats) {
  if (!c) return LSG_ERR_INVALID_ARG;
  if (((ticket >> 8) & 255) == SLOT_MERGE) {
    if (node_valid != -1) {
      c->err = "lsg_wait_jobs_node: a coalesced package has no node check of its own";
      return LSG_ERR_INVALID_ARG;
    }
    if (!results) return LSG_ERR_INVALID_ARG;
    return wait_merged(c, ticket, results, stats);
  }
  if (int prc = presync_pkg(c, ticket, false)) return prc;
  CtxLock lk(c->mu);
  LSG_HIPC(c, hipSetDevice(c->dev[0]->device));
  const int p = ticket_pkg(c, ticket);
  if (p < 0) return LSG_ERR_INVALID_ARG;
  const size_t nj = c->dev[0]->slots[p].n_jobs;
  if (nj && !results) return LSG_ERR_INVALID_ARG;
  if (node_valid != -1 && c->n_dev > 1) {
    c->err = "lsg_wait_jobs_node: a multi-device context runs its own node check";
    return LSG_ERR_INVALID_ARG;
  }
  const int rc = wait_pkg(c, &lk, p, node_valid == -1 ? -2 : (node_valid ? 1 : 0), results, stats);
  maybe_flush(c);
  return rc;
}

int lsg_wait_jobs(lsg_ctx* c, lsg_ticket ticket, lsg_job_result* results, lsg_stats* stats) {
  return lsg_wait_jobs_node(c, ticket, -1, results, stats);
}

int lsg_jobs_partial(lsg_ctx* c, lsg_ticket ticket, uint8_t* out576, int32_t* has_batch) {
  if (!c || !out576) return LSG_ERR_INVALID_ARG;
  if (c->n_dev > 1) {
    c->err = "lsg_jobs_partial: a multi-device context exchanges its partials itself";
    return LSG_ERR_INVALID_ARG;
  }
  if (int prc = presync_pkg(c, ticket, true)) return prc;
  LSG_ENTER(c);
  const int p = ticket_pkg(c, ticket);
  if (p < 0) return LSG_ERR_INVALID_ARG;
  Slot* s = &c->dev[0]->slots[p];
  const bool has = !s->phA.groups.empty() && s->big_g >= 0;
  if (has && s->lone_unscaled) {
    const uint8_t* src;
    LSG_RC(export_partial_dev(s, &src));
    LSG_RC(ensure_host(s, s->h_xport, 576));
    LSG_HIP(s, hipMemcpyAsync(s->h_xport.p, src, 576, hipMemcpyDeviceToHost, s->st[0]));
    LSG_HIP(s, hipStreamSynchronize(s->st[0]));
    memcpy(out576, s->h_xport.p, 576);
  } else if (has) {
    memcpy(out576, H_<uint8_t>(s->h_blob) + 576 * (size_t)s->big_g, 576);
  } else {
    memcpy(out576, fp12_one_blob(), 576);
  }
  if (has_batch) *has_batch = has ? 1 : 0;
  return LSG_OK;
}

int lsg_jobs_partial_device(lsg_ctx* c, lsg_ticket ticket, void* dev_out576, int32_t* has_batch) {
  if (!c || !dev_out576) return LSG_ERR_INVALID_ARG;
  if (c->n_dev > 1) {
    c->err = "lsg_jobs_partial_device: a multi-device context exchanges its partials itself";
    return LSG_ERR_INVALID_ARG;
  }
  if (int prc = presync_pkg(c, ticket, true)) return prc;
  hipEvent_t xev;
  bool has;
  {
    LSG_ENTER(c);
    const int p = ticket_pkg(c, ticket);
    if (p < 0) return LSG_ERR_INVALID_ARG;
    Slot* s = &c->dev[0]->slots[p];
    has = !s->phA.groups.empty() && s->big_g >= 0;
    // the copy goes out on a high-priority stream (the node final exponentiations'): on the
    // package's own stream it would queue behind other packages' kernels sharing its hardware
    // queue, and the node's next verdicts wait on it (ev_part is complete: presync_pkg)
    LSG_RC(prio_stream(c, c->dev[0], &c->dev[0]->s_xp));
    hipStream_t xs = c->dev[0]->s_xp;
    if (has) {
      const uint8_t* src;
      LSG_RC(export_partial_dev(s, &src, xs));  // f^r (a lone unscaled set) runs on xs too
      LSG_HIP(s, hipMemcpyAsync(dev_out576, src, 576, hipMemcpyDeviceToDevice, xs));
    } else {
      LSG_HIP(s, hipMemcpyAsync(dev_out576, fp12_one_blob(), 576, hipMemcpyHostToDevice, xs));
    }
    LSG_HIP(s, hipEventRecord(s->ev_xp, xs));
    xev = s->ev_xp;  // (the slot stays this ticket's until it is waited on)
  }
  // the copy completes without the context lock held: submissions and resolutions of other
  // packages go on meanwhile
  (void)hipSetDevice(c->dev[0]->device);
  if (hipError_t e = event_wait(xev)) {
    std::lock_guard<std::mutex> lk(c->mu);  // (c->err is written under the lock)
    return fail_c(c, "hipEventSynchronize", e);
  }
  if (has_batch) *has_batch = has ? 1 : 0;
  return LSG_OK;
}

int lsg_verify_jobs(lsg_ctx* c, const lsg_job* jobs, size_t n_jobs, uint64_t seed, lsg_job_result* results,
                    lsg_stats* stats) {
  if (!c || (n_jobs && (!jobs || !results))) return LSG_ERR_INVALID_ARG;
  lsg_ticket t;
  int rc = lsg_submit_jobs(c, jobs, n_jobs, seed, &t);
  if (rc) return rc;
  return lsg_wait_jobs(c, t, results, stats);
}

int lsg_verify_sets(lsg_ctx* c, const lsg_set* sets, size_t n_sets, uint64_t seed, lsg_job_result* result) {
  if (!c || !result || (n_sets && !sets)) return LSG_ERR_INVALID_ARG;
  lsg_job job;
  job.sets = sets;
  job.n_sets = (uint32_t)n_sets;
  job.flags = 0;
  return lsg_verify_jobs(c, &job, 1, seed, result, nullptr);
}

int lsg_pipeline_slots(lsg_ctx* c, int32_t* n) {
  if (!c || !n) return LSG_ERR_INVALID_ARG;
  *n = LSG_SLOTS;
  return LSG_OK;
}

int lsg_poll(lsg_ctx* c, lsg_ticket ticket, int32_t* done) {
  if (!c || !done) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  std::vector<hipEvent_t> evs;
  if (Slot* f = ticket_final(c, ticket)) {
    evs.push_back(f->ev_done);
  } else if (((ticket >> 8) & 255) == SLOT_MERGE) {
    auto it = c->merged.find(ticket >> 16);
    if (it == c->merged.end()) return LSG_ERR_INVALID_ARG;
    if (it->second.rc) {  // its launch failed: done (the wait reports the failure)
      *done = 1;
      return LSG_OK;
    }
    if (it->second.slot < 0) {  // not launched: launch when the device has room
      maybe_flush(c);
      it = c->merged.find(ticket >> 16);
      if (it == c->merged.end()) return LSG_ERR_INVALID_ARG;
      if (it->second.slot < 0) {
        *done = it->second.rc ? 1 : 0;
        return LSG_OK;
      }
    }
    evs.push_back(c->dev[0]->slots[it->second.slot].ev_done);
  } else {
    const int p = ticket_pkg(c, ticket);
    if (p < 0) return LSG_ERR_INVALID_ARG;
    for (int d = 0; d < c->n_dev; d++) evs.push_back(c->dev[d]->slots[p].ev_done);
  }
  *done = 1;
  for (hipEvent_t e : evs) {
    hipError_t r = hipEventQuery(e);
    if (r == hipErrorNotReady) {
      *done = 0;
      return LSG_OK;
    }
    if (r != hipSuccess) return fail_c(c, "hipEventQuery", r);
  }
  return LSG_OK;
}

// one shard's partial (sync): all sets as one batchable job
int lsg_batch_partial(lsg_ctx* c, const lsg_set* sets, size_t n_sets, uint64_t seed, uint8_t* out576,
                      int32_t* set_err, int32_t* any_error) {
  if (!c || !out576 || !any_error || (n_sets && !sets)) return LSG_ERR_INVALID_ARG;
  if (c->n_dev > 1) {
    c->err = "lsg_batch_partial: single-device contexts only";
    return LSG_ERR_INVALID_ARG;
  }
  lsg_ticket t;
  {
    CtxLock lk(c->mu);
    LSG_HIPC(c, hipSetDevice(c->dev[0]->device));
    lsg_job job;
    job.sets = sets;
    job.n_sets = (uint32_t)n_sets;
    job.flags = LSG_JOB_BATCHABLE;
    int rc = submit_pkg(c, lk, &job, 1, seed, &t, false);  // the partial leaves: every r_i random
    if (rc) return rc;
  }
  const int prc = presync_pkg(c, t, false);
  LSG_ENTER(c);
  const int p = ticket_pkg(c, t);
  if (p < 0) return LSG_ERR_INVALID_ARG;
  Slot* s = &c->dev[0]->slots[p];
  if (prc) {  // the internal ticket cannot be waited on again: give its slot back
    sync_slot(s);
    s->kind = SLOT_FREE;
    return prc;
  }
  const SetStatus ss = read_status(s);
  *any_error = 0;
  for (size_t i = 0; i < n_sets; i++) {
    const int32_t e = set_error(ss, i);
    if (set_err) set_err[i] = e;
    if (e) *any_error = 1;
  }
  for (size_t k = 0; k < s->n_pks; k++)
    if (ss.pkerr[k]) *any_error = 1;
  if (s->big_g >= 0)
    memcpy(out576, H_<uint8_t>(s->h_blob) + 576 * (size_t)s->big_g, 576);
  else
    memcpy(out576, fp12_one_blob(), 576);
  s->kind = SLOT_FREE;
  keep_times(s);
  return LSG_OK;
}

int lsg_final_submit_groups(lsg_ctx* c, const uint8_t* partials576, size_t n_groups, size_t per_group,
                            lsg_ticket* ticket) {
  if (!c || !ticket || (n_groups && per_group && !partials576) || (n_groups && !per_group)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = nullptr;
  for (int i = 0; i < LSG_FINALS && !s; i++)
    if (c->dev[0]->finals[i].kind == SLOT_FREE) s = &c->dev[0]->finals[i];
  if (!s) {
    c->err = "all final-exponentiation entries are busy";
    return LSG_ERR_BUSY;
  }
  // a node verdict waits on this one program: the greatest stream priority (the entry is free)
  LSG_RC(prio_stream(c, c->dev[0], &c->dev[0]->s_nfe));
  s->st[0] = s->st[1] = c->dev[0]->s_nfe;
  int rc = submit_final(s, partials576, n_groups, per_group);
  if (rc) {
    sync_slot(s);
    return rc;
  }
  uint64_t serial;
  *ticket = make_ticket(c, SLOT_FINAL, s->index, &serial);
  s->kind = SLOT_FINAL;
  s->serial = serial;
  return LSG_OK;
}

int lsg_final_submit_device(lsg_ctx* c, const void* dev_partials576, size_t n_partials, lsg_ticket* ticket) {
  if (!c || !ticket || (n_partials && !dev_partials576)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = nullptr;
  for (int i = 0; i < LSG_FINALS && !s; i++)
    if (c->dev[0]->finals[i].kind == SLOT_FREE) s = &c->dev[0]->finals[i];
  if (!s) {
    c->err = "all final-exponentiation entries are busy";
    return LSG_ERR_BUSY;
  }
  LSG_RC(prio_stream(c, c->dev[0], &c->dev[0]->s_nfe));
  s->st[0] = s->st[1] = c->dev[0]->s_nfe;
  int rc = submit_final(s, (const uint8_t*)dev_partials576, n_partials ? 1 : 0, n_partials, true);
  if (rc) {
    sync_slot(s);
    return rc;
  }
  uint64_t serial;
  *ticket = make_ticket(c, SLOT_FINAL, s->index, &serial);
  s->kind = SLOT_FINAL;
  s->serial = serial;
  return LSG_OK;
}

int lsg_final_submit(lsg_ctx* c, const uint8_t* partials576, size_t n_partials, lsg_ticket* ticket) {
  if (!c || !ticket || (n_partials && !partials576)) return LSG_ERR_INVALID_ARG;
  return lsg_final_submit_groups(c, partials576, n_partials ? 1 : 0, n_partials, ticket);
}

static int final_wait(lsg_ctx* c, lsg_ticket ticket, int32_t* valid, bool single) {
  if (!c || !valid) return LSG_ERR_INVALID_ARG;
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    Slot* s = ticket_final(c, ticket);
    if (!s) return LSG_ERR_INVALID_ARG;
    ev = s->ev_done;
  }
  (void)hipSetDevice(c->dev[0]->device);
  hipError_t e = event_wait(ev);
  LSG_ENTER(c);
  if (e != hipSuccess) return fail_c(c, "hipEventSynchronize", e);
  Slot* s = ticket_final(c, ticket);
  if (!s) return LSG_ERR_INVALID_ARG;
  if (single && s->n_sets > 1) {
    c->err = "ticket carries several groups: use lsg_final_wait_groups";
    return LSG_ERR_INVALID_ARG;
  }
  if (!s->n_sets) valid[0] = 0;
  for (size_t g = 0; g < s->n_sets; g++) valid[g] = H_<int32_t>(s->h_verdict)[g];
  s->kind = SLOT_FREE;
  keep_times(s);
  return LSG_OK;
}

int lsg_final_wait_groups(lsg_ctx* c, lsg_ticket ticket, int32_t* valid) { return final_wait(c, ticket, valid, false); }
int lsg_final_wait(lsg_ctx* c, lsg_ticket ticket, int32_t* valid) { return final_wait(c, ticket, valid, true); }

int lsg_final_verify(lsg_ctx* c, const uint8_t* partials576, size_t n_partials, int32_t* valid) {
  if (!c || !valid || (n_partials && !partials576)) return LSG_ERR_INVALID_ARG;
  lsg_ticket t;
  int rc = lsg_final_submit(c, partials576, n_partials, &t);
  if (rc) return rc;
  return lsg_final_wait(c, t, valid);
}

int lsg_aggregate_pubkeys(lsg_ctx* c, const uint8_t* pks, uint32_t pk_len, size_t n, uint8_t* out96,
                          int32_t* err_code) {
  if (!c || !out96 || !err_code || (n && !pks)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Dev* d = c->dev[0];
  Slot* s = &d->util;
  timer_reset(s);
  *err_code = 0;
  if (n == 0) {
    *err_code = LSG_ERR_EMPTY_AGGREGATE;
    return LSG_OK;
  }
  s->plan.clear();
  LSG_RC(util_stage_keys(s, pks, pk_len, n));
  std::vector<int32_t> off{0}, len{(int32_t)n};
  SegPlan P = plan_seg(s->plan, 0, off, len, false, 0, 0);
  LSG_RC(upload_plan(s));
  const int np = (int)n;
  KL(s, "k_pk_decode", lsgk::pk_decode(S_(s), np, P_<uint8_t>(s->d_pk), s->pk_stride, P_<uint32_t>(s->d_pklen),
                                       P_<uint32_t>(s->d_pkp), P_<int32_t>(s->d_pkerr), P_<uint32_t>(d->d_pktab),
                                       P_<uint8_t>(d->d_pktab_ok), (uint32_t)d->pktab_n));
  LSG_RC(run_seg(s, 0, "g1_aggregate", P, P_<uint32_t>(s->d_pkp), P_<uint32_t>(s->d_agg)));
  KL(s, "k_g1p_to_bytes", lsgk::g1p_to_bytes(S_(s), 1, P_<uint32_t>(s->d_agg), P_<uint8_t>(s->d_Fb)));
  std::vector<int32_t> pkerr(n);
  LSG_HIP(s, hipMemcpyAsync(pkerr.data(), s->d_pkerr.p, 4 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipMemcpyAsync(out96, s->d_Fb.p, 96, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  keep_times(s);
  for (size_t k = 0; k < n; k++)
    if (pkerr[k]) {
      *err_code = pkerr[k];
      break;
    }
  return LSG_OK;
}

int lsg_aggregate_pubkeys_multi(lsg_ctx* c, const lsg_set* sets, size_t n_sets, uint8_t* out96, int32_t* err) {
  if (!c || (n_sets && (!sets || !out96 || !err)) || n_sets > 0x7fffffffull) return LSG_ERR_INVALID_ARG;
  for (size_t i = 0; i < n_sets; i++)
    if (sets[i].n_pks && (!sets[i].pks || (sets[i].pk_len != 48 && sets[i].pk_len != 96 && sets[i].pk_len != LSG_PK_INDEX)))
      return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Dev* d = c->dev[0];
  Slot* s = &d->util;
  timer_reset(s);
  if (n_sets == 0) return LSG_OK;
  std::vector<lsg_set> ks(n_sets);
  std::vector<const lsg_set*> sp(n_sets);
  for (size_t i = 0; i < n_sets; i++) {
    memset(&ks[i], 0, sizeof(lsg_set));
    ks[i].pks = sets[i].pks;
    ks[i].pk_len = sets[i].pk_len;
    ks[i].n_pks = sets[i].n_pks;
    sp[i] = &ks[i];
  }
  LSG_RC(stage_sets(s, sp.data(), n_sets, 0, false));
  const size_t np = s->n_pks;
  LSG_RC(size_state(s, n_sets, np, 1, 0));
  s->plan.clear();
  const bool tree = np >= AGG_TREE_MIN_KEYS && agg_tree_on();
  s->single_keys = false;
  if (tree)
    s->agg = plan_agg_tree(s);
  else
    s->pkagg = plan_pk_agg(s);
  LSG_RC(upload_plan(s));
  if (tree) {
    LSG_RC(launch_agg_tree(s, s->agg, P_<uint32_t>(s->d_agg)));
  } else if (np) {
    LSG_RC(run_pk_seg(s, s->pkagg, P_<uint32_t>(s->d_agg)));
  }
  LSG_RC(ensure(s, s->d_aux, 96 * n_sets));
  KL(s, "k_g1p_to_bytes", lsgk::g1p_to_bytes(S_(s), (int)n_sets, P_<uint32_t>(s->d_agg), P_<uint8_t>(s->d_aux)));
  std::vector<int32_t> pkerr(std::max(np, (size_t)1));
  if (np) LSG_HIP(s, hipMemcpyAsync(pkerr.data(), s->d_pkerr.p, 4 * np, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipMemcpyAsync(out96, s->d_aux.p, 96 * n_sets, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  keep_times(s);
  for (size_t i = 0; i < n_sets; i++) {
    err[i] = s->pk_cnt[i] == 0 ? LSG_ERR_EMPTY_AGGREGATE : 0;
    for (uint32_t q = 0; q < s->pk_cnt[i] && !err[i]; q++) err[i] = pkerr[s->pk_first[i] + q];
  }
  return LSG_OK;
}

int lsg_pubkey_table_set(lsg_ctx* c, size_t first, const uint8_t* pks, uint32_t pk_len, size_t n, int32_t* err) {
  if (!c || (n && !pks) || (pk_len != 48 && pk_len != 96) || first + n > 0xffffffffull) return LSG_ERR_INVALID_ARG;
  std::unique_lock<std::shared_mutex> tab(c->tab_mu);  // no package is being staged from the table
  LSG_ENTER(c);
  if (n == 0) return LSG_OK;
  std::vector<int32_t> pkerr;
  for (int d = 0; d < c->n_dev; d++) LSG_RC(dev_pktab_set(c->dev[d], first, pks, pk_len, n, pkerr));
  (void)hipSetDevice(c->dev[0]->device);
  if (err)
    for (size_t k = 0; k < n; k++) err[k] = pkerr[k];
  return LSG_OK;
}

int lsg_pubkey_table_size(lsg_ctx* c, size_t* n) {
  if (!c || !n) return LSG_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  *n = c->dev[0]->pktab_n;
  return LSG_OK;
}

int lsg_pubkey_validate(lsg_ctx* c, const uint8_t* pks, uint32_t pk_len, size_t n, uint8_t* out96, int32_t* err) {
  if (!c || !err || (n && !pks) || (pk_len != 48 && pk_len != 96) || n > 0x7fffffffull) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Dev* d = c->dev[0];
  Slot* s = &d->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  LSG_RC(util_stage_keys(s, pks, pk_len, n));
  LSG_RC(ensure(s, s->d_ub, 96 * n));
  KL(s, "k_pk_validate", lsgk::pk_validate(S_(s), (int)n, P_<uint8_t>(s->d_pk), pk_len, P_<uint32_t>(s->d_pkp),
                                           P_<int32_t>(s->d_pkerr)));
  LSG_HIP(s, hipMemcpyAsync(err, s->d_pkerr.p, 4 * n, hipMemcpyDeviceToHost, s->st[0]));
  if (out96) {
    KL(s, "k_g1p_to_bytes", lsgk::g1p_to_bytes(S_(s), (int)n, P_<uint32_t>(s->d_pkp), P_<uint8_t>(s->d_ub)));
    LSG_HIP(s, hipMemcpyAsync(out96, s->d_ub.p, 96 * n, hipMemcpyDeviceToHost, s->st[0]));
  }
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  keep_times(s);
  return LSG_OK;
}

int lsg_hash_to_g2(lsg_ctx* c, const uint8_t* msgs, uint32_t msg_len, size_t n, const uint8_t* dst,
                   uint32_t dst_len, uint8_t* out192) {
  if (!c || !out192 || (n && msg_len && !msgs) || dst_len > 255 || (dst_len && !dst)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Dev* d = c->dev[0];
  Slot* s = &d->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  LSG_RC(util_hash(s, msgs, msg_len, n, dst, dst_len));
  LSG_RC(ensure(s, s->d_aux, 192 * n));
  const int nn = (int)n;
  KL(s, "k_g2a_to_bytes",
     lsgk::g2a_to_bytes(S_(s), nn, P_<uint32_t>(s->d_H), P_<uint8_t>(s->d_hinf), P_<uint8_t>(s->d_aux)));
  LSG_HIP(s, hipMemcpyAsync(out192, s->d_aux.p, 192 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  keep_times(s);
  return LSG_OK;
}

// Signature.fromBytes(sig, affine, validate) for n signatures (subgroup check when validate)
static int sig_decode_impl(lsg_ctx* c, const uint8_t* sigs, uint32_t sig_len, size_t n, bool validate, Slot** out) {
  Dev* d = c->dev[0];
  Slot* s = &d->util;
  *out = s;
  std::vector<lsg_set> sets(n);
  std::vector<const lsg_set*> sp(n);
  for (size_t i = 0; i < n; i++) {
    memset(&sets[i], 0, sizeof(lsg_set));
    sets[i].sig = sigs + (size_t)sig_len * i;
    sets[i].sig_len = sig_len;
    sp[i] = &sets[i];
  }
  LSG_RC(stage_sets(s, sp.data(), n, 0, false));
  LSG_RC(size_state(s, n, 0, 1, 0));
  const int nn = (int)n;
  KL(s, "k_sig_decode", lsgk::sig_decode(S_(s), nn, P_<uint8_t>(s->d_sig), P_<uint32_t>(s->d_siglen),
                                         P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf), P_<int32_t>(s->d_seterr)));
  if (validate)
    KL(s, "k_sig_subgroup", lsgk::sig_subgroup(S_(s), nn, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf),
                                               P_<int32_t>(s->d_seterr)));
  return LSG_OK;
}

int lsg_sig_decode(lsg_ctx* c, const uint8_t* sigs, uint32_t sig_len, size_t n, uint8_t* out192, int32_t* err) {
  if (!c || !out192 || !err || (n && !sigs)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  timer_reset(&c->dev[0]->util);
  if (n == 0) return LSG_OK;
  Slot* s;
  LSG_RC(sig_decode_impl(c, sigs, sig_len, n, true, &s));
  LSG_RC(ensure(s, s->d_aux, 192 * n));
  KL(s, "k_g2a_to_bytes", lsgk::g2a_to_bytes(S_(s), (int)n, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf),
                                             P_<uint8_t>(s->d_aux)));
  LSG_HIP(s, hipMemcpyAsync(out192, s->d_aux.p, 192 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipMemcpyAsync(err, s->d_seterr.p, 4 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  keep_times(s);
  return LSG_OK;
}

// G2 signature aggregation for the op pools: n_groups Signature.aggregate
// calls in one pass -- decode without the subgroup check (signatureFromBytesNoCheck,
// opPools/utils.ts:32-34), one segmented reduction, one compression per group
int lsg_aggregate_signatures(lsg_ctx* c, const uint8_t* sigs, uint32_t sig_len, const uint32_t* offsets,
                             size_t n_groups, uint8_t* out96, int32_t* err) {
  if (!c || !offsets || (n_groups && (!out96 || !err)) || offsets[0] != 0 || n_groups > 0x7fffffffull)
    return LSG_ERR_INVALID_ARG;
  for (size_t g = 0; g < n_groups; g++)
    if (offsets[g + 1] < offsets[g]) return LSG_ERR_INVALID_ARG;
  const size_t n = offsets[n_groups];
  if (n && !sigs) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  timer_reset(&c->dev[0]->util);
  for (size_t g = 0; g < n_groups; g++) {
    err[g] = offsets[g + 1] == offsets[g] ? LSG_ERR_EMPTY_AGGREGATE : 0;
    memset(out96 + 96 * g, 0, 96);
  }
  if (n == 0) return LSG_OK;
  Slot* s;
  LSG_RC(sig_decode_impl(c, sigs, sig_len, n, false, &s));
  LSG_RC(size_state(s, n, 0, n_groups, 0));
  s->plan.clear();
  std::vector<int32_t> off(n_groups), len(n_groups);
  for (size_t g = 0; g < n_groups; g++) {
    off[g] = (int32_t)offsets[g];
    len[g] = (int32_t)(offsets[g + 1] - offsets[g]);
  }
  SegPlan P = plan_seg(s->plan, 1, off, len, false, 0, 0);
  LSG_RC(upload_plan(s));
  LSG_RC(ensure(s, s->d_aux, 96 * n_groups));
  const int nn = (int)n;
  KL(s, "k_sig_prep", lsgk::sig_prep(S_(s), nn, P_<uint32_t>(s->d_sigaff), P_<uint8_t>(s->d_siginf),
                                     P_<int32_t>(s->d_seterr), nullptr, nullptr, nullptr, P_<uint32_t>(s->d_rs)));
  LSG_RC(run_seg(s, 1, "g2_aggregate", P, P_<uint32_t>(s->d_rs), P_<uint32_t>(s->d_S)));
  KL(s, "k_g2p_compress",
     lsgk::g2p_compress(S_(s), (int)n_groups, P_<uint32_t>(s->d_S), P_<uint8_t>(s->d_aux)));
  std::vector<int32_t> serr(n);
  std::vector<uint8_t> blob(96 * n_groups);
  LSG_HIP(s, hipMemcpyAsync(serr.data(), s->d_seterr.p, 4 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipMemcpyAsync(blob.data(), s->d_aux.p, 96 * n_groups, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  keep_times(s);
  // Signature.aggregate throws on the first signature that fails to deserialize
  for (size_t g = 0; g < n_groups; g++) {
    if (offsets[g + 1] == offsets[g]) continue;
    for (uint32_t i = offsets[g]; i < offsets[g + 1] && !err[g]; i++) err[g] = serr[i];
    if (!err[g]) memcpy(out96 + 96 * g, blob.data() + 96 * g, 96);
  }
  return LSG_OK;
}

// SSZ signing roots; kind 0: object roots given, 1: AttestationData bytes
static int signing_roots(lsg_ctx* c, int kind, const uint8_t* objs, size_t n, const uint8_t* domain, uint32_t dstride,
                         uint8_t* out32) {
  const size_t ob = kind ? 128 : 32;
  if (!c || !domain || (dstride != 0 && dstride != 32) || (n && (!objs || !out32)) || n > 0x7fffffffull)
    return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Dev* d = c->dev[0];
  Slot* s = &d->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  const size_t nd = dstride ? n : 1;
  LSG_RC(ensure(s, s->d_aux, ob * n + 32 * nd));
  LSG_RC(ensure(s, s->d_Fb, 32 * n));
  uint8_t* d_obj = P_<uint8_t>(s->d_aux);
  uint8_t* d_dom = d_obj + ob * n;
  LSG_HIP(s, hipMemcpyAsync(d_obj, objs, ob * n, hipMemcpyHostToDevice, s->st[0]));
  LSG_HIP(s, hipMemcpyAsync(d_dom, domain, 32 * nd, hipMemcpyHostToDevice, s->st[0]));
  const int nn = (int)n;
  if (kind)
    KL(s, "k_attestation_signing_root",
       lsgk::attestation_signing_root(S_(s), nn, d_obj, d_dom, dstride, P_<uint8_t>(s->d_Fb)));
  else
    KL(s, "k_signing_root", lsgk::signing_root(S_(s), nn, d_obj, d_dom, dstride, P_<uint8_t>(s->d_Fb)));
  LSG_HIP(s, hipMemcpyAsync(out32, s->d_Fb.p, 32 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  keep_times(s);
  return LSG_OK;
}

int lsg_signing_roots(lsg_ctx* c, const uint8_t* roots32, size_t n, const uint8_t* domain32, uint32_t domain_stride,
                      uint8_t* out32) {
  return signing_roots(c, 0, roots32, n, domain32, domain_stride, out32);
}

int lsg_attestation_signing_roots(lsg_ctx* c, const uint8_t* data128, size_t n, const uint8_t* domain32,
                                  uint32_t domain_stride, uint8_t* out32) {
  return signing_roots(c, 1, data128, n, domain32, domain_stride, out32);
}

int lsg_sign(lsg_ctx* c, const uint8_t* sks32, const uint8_t* msgs, uint32_t msg_len, size_t n, uint8_t* out96) {
  if (!c || !out96 || (n && (!sks32 || !msgs))) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->dev[0]->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  LSG_RC(util_hash(s, msgs, msg_len, n, DST_POP, DST_POP_LEN));
  LSG_RC(ensure(s, s->d_aux, 96 * n));
  LSG_RC(ensure(s, s->d_Fb, 32 * n));
  LSG_HIP(s, hipMemcpyAsync(s->d_Fb.p, sks32, 32 * n, hipMemcpyHostToDevice, s->st[0]));
  KL(s, "k_sign", lsgk::sign(S_(s), (int)n, P_<uint8_t>(s->d_Fb), P_<uint32_t>(s->d_H), P_<uint8_t>(s->d_aux)));
  LSG_HIP(s, hipMemcpyAsync(out96, s->d_aux.p, 96 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  return LSG_OK;
}

int lsg_sk_to_pk(lsg_ctx* c, const uint8_t* sks32, size_t n, uint8_t* out96) {
  if (!c || !out96 || (n && !sks32)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->dev[0]->util;
  timer_reset(s);
  if (n == 0) return LSG_OK;
  LSG_RC(ensure(s, s->d_aux, 96 * n));
  LSG_RC(ensure(s, s->d_Fb, 32 * n));
  LSG_HIP(s, hipMemcpyAsync(s->d_Fb.p, sks32, 32 * n, hipMemcpyHostToDevice, s->st[0]));
  KL(s, "k_sk_to_pk", lsgk::sk_to_pk(S_(s), (int)n, P_<uint8_t>(s->d_Fb), P_<uint8_t>(s->d_aux)));
  LSG_HIP(s, hipMemcpyAsync(out96, s->d_aux.p, 96 * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  return LSG_OK;
}

int lsg_check_fp2_mul(lsg_ctx* c, const uint32_t* in, size_t n, uint32_t* out) {
  if (!c || (n && (!in || !out)) || n > 0x7fffffffull / (4 * W_FP)) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  if (n == 0) return LSG_OK;
  Slot* s = &c->dev[0]->util;
  timer_reset(s);
  LSG_RC(ensure(s, s->d_aux, 4 * 4 * W_FP * n));
  LSG_RC(ensure(s, s->d_Fb, 4 * 2 * W_FP * n));
  LSG_HIP(s, hipMemcpyAsync(s->d_aux.p, in, 4 * 4 * W_FP * n, hipMemcpyHostToDevice, s->st[0]));
  KL(s, "k_check_fp2_mul", lsgk::check_fp2_mul(S_(s), (int)n, P_<uint32_t>(s->d_aux), P_<uint32_t>(s->d_Fb)));
  LSG_HIP(s, hipMemcpyAsync(out, s->d_Fb.p, 4 * 2 * W_FP * n, hipMemcpyDeviceToHost, s->st[0]));
  LSG_HIP(s, hipStreamSynchronize(s->st[0]));
  return LSG_OK;
}

int lsg_probe_fp_mul_rate(lsg_ctx* c, double* fp_mul_per_s, double* mad_per_s) {
  if (!c || !fp_mul_per_s || !mad_per_s) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->dev[0]->util;
  hipDeviceProp_t prop;
  LSG_HIP(s, hipGetDeviceProperties(&prop, c->dev[0]->device));
  const int items = prop.multiProcessorCount * 32 * 32;  // 32 waves per CU, 32 pair items each
  LSG_RC(ensure(s, s->d_aux, 4 * W_FP * (size_t)items));
  std::vector<uint32_t> init(W_FP * (size_t)items, 0);
  for (size_t i = 0; i < init.size(); i += 4) init[i] = (uint32_t)(i * 2654435761u) & 0x1fffffffu;  // small values < p
  LSG_HIP(s, hipMemcpy(s->d_aux.p, init.data(), 4 * init.size(), hipMemcpyHostToDevice));
  const int iters = 64;
  hipStream_t S = s->st[0];
  LSG_HIP(s, lsgk::probe_fp_mul(S, items, 2, P_<uint32_t>(s->d_aux)));
  hipEvent_t a, b;
  LSG_HIP(s, hipEventCreate(&a));
  LSG_HIP(s, hipEventCreate(&b));
  LSG_HIP(s, hipEventRecord(a, S));
  LSG_HIP(s, lsgk::probe_fp_mul(S, items, iters, P_<uint32_t>(s->d_aux)));
  LSG_HIP(s, hipEventRecord(b, S));
  LSG_HIP(s, hipEventSynchronize(b));
  float ms = 0;
  LSG_HIP(s, hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *fp_mul_per_s = (double)items * iters * 4.0 / (ms * 1e-3);
  *mad_per_s = *fp_mul_per_s * 300.0;
  return LSG_OK;
}

int lsg_probe_mad_peak(lsg_ctx* c, double* mad_per_s) {
  if (!c || !mad_per_s) return LSG_ERR_INVALID_ARG;
  LSG_ENTER(c);
  Slot* s = &c->dev[0]->util;
  hipDeviceProp_t prop;
  LSG_HIP(s, hipGetDeviceProperties(&prop, c->dev[0]->device));
  const int blocks = prop.multiProcessorCount * 32;  // 32 waves per CU (8 per SIMD)
  const size_t threads = (size_t)blocks * 256;
  LSG_RC(ensure(s, s->d_aux, 8 * threads));
  hipStream_t S = s->st[0];
  const int iters = 4096;
  LSG_HIP(s, lsgk::probe_mad(S, blocks, 16, 3u, P_<uint64_t>(s->d_aux)));
  hipEvent_t a, b;
  LSG_HIP(s, hipEventCreate(&a));
  LSG_HIP(s, hipEventCreate(&b));
  LSG_HIP(s, hipEventRecord(a, S));
  LSG_HIP(s, lsgk::probe_mad(S, blocks, iters, 5u, P_<uint64_t>(s->d_aux)));
  LSG_HIP(s, hipEventRecord(b, S));
  LSG_HIP(s, hipEventSynchronize(b));
  float ms = 0;
  LSG_HIP(s, hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *mad_per_s = (double)threads * iters * 16.0 / (ms * 1e-3);
  return LSG_OK;
}

int lsg_last_kernel_times(lsg_ctx* c, const char** names, double* ms, int max) {
  if (!c) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  const auto& v = c->dev[0]->last_times;
  int n = 0;
  for (size_t i = 0; i < v.size() && n < max; i++, n++) {
    if (names) names[n] = v[i].first;
    if (ms) ms[n] = v[i].second;
  }
  return n;
}

int lsg_assign_jobs(const uint32_t* job_sets, size_t n_jobs, int32_t n_devices, int32_t* owner) {
  if ((n_jobs && (!job_sets || !owner)) || n_devices < 1) return LSG_ERR_INVALID_ARG;
  assign_jobs(job_sets, n_jobs, n_devices, owner);
  return LSG_OK;
}

}  // extern "C"
