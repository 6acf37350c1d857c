/*
 * lsg_napi.c -- thin N-API addon over the C ABI (include/lodestar_bls.h).
 *
 * This is the native half of BlsGpuVerifier (lodestar_amd/js/blsGpuVerifier.js), which
 * stands in for BlsMultiThreadWorkerPool
 * (/root/reference/packages/beacon-node/src/chain/bls/multithread/index.ts).  Where the
 * reference posts BlsWorkReq[] packages to @chainsafe/threads workers running
 * @chainsafe/blst (multithread/worker.ts:30-106), the verifier hands each package to
 * verifyPacked(): one of the context's own package threads submits it (lsg_submit_jobs copies
 * the inputs into pinned staging) and blocks in lsg_wait_jobs; the verdicts return to the JS
 * thread through a napi_threadsafe_function.  Neither the JS main thread nor libuv's thread
 * pool (the beacon node's file and DB I/O runs there) ever blocks on the GPU.  Nothing here
 * does arithmetic.
 *
 * JS surface (all synchronous unless noted):
 *   open(device | devices[]) -> ctx         lsg_init / lsg_init_devices (one context over the
 *                                           node's GPUs: chain.ts:195-198 builds one verifier)
 *   reserve(ctx, maxSets, maxPks, maxMsgBytes, nSlots)                  lsg_reserve
 *   deviceCount(ctx) -> n                   lsg_device_count
 *   close(ctx)                              lsg_destroy
 *   slots(ctx) -> n                         packages in flight: min(lsg_pipeline_slots, 16 threads)
 *   deviceName(ctx) -> string               lsg_device_name
 *   verifyPacked(ctx, arena, setDesc, jobDesc, seed[, priority]) -> Promise<{status: Uint8Array,
 *       errCode: Int32Array, batchRetries, batchSigsSuccess, startNs, endNs, finalExps,
 *       submitUs, keyError, workerId}>     lsg_submit_jobs + lsg_wait_jobs on a package thread
 *       (layout below, at js_verify_packed).  startNs / endNs are CLOCK_MONOTONIC nanoseconds
 *       (process.hrtime.bigint()'s clock); workerId is the pipeline slot that ran the package
 *       (the reference's workerId label).  priority = true (verifyOnMainThread): the package
 *       goes ahead of every queued one, onto the addon's priority thread
 *   sign(ctx, sks, msgs) / skToPk(ctx, sks)  test and bench input generation
 *   verifySets(ctx, sets, seed) -> {status, errCode}                   lsg_verify_sets
 *   aggregatePubkeys(ctx, pubkeys[]) -> {errCode, bytes: Uint8Array(96)} lsg_aggregate_pubkeys
 *   pubkeyTableSet(ctx, firstIndex, pubkeys[]) -> errCodes[]          lsg_pubkey_table_set
 *       (a set may then carry pubkeyIndices: Uint32Array instead of pubkeys)
 *   hashToG2(ctx, message, dst) -> Uint8Array(192)                     lsg_hash_to_g2
 * Failures of the library itself (not verdicts) throw an Error carrying lsg_last_error().
 */
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lodestar_bls.h"

#define LSG_NAPI_THREADS 16 /* package threads per context: one outstanding package each */

#define NAPI_CALL(env, call)                                              \
  do {                                                                    \
    if ((call) != napi_ok) {                                              \
      napi_throw_error((env), NULL, "lsg_napi: N-API call failed: " #call); \
      return NULL;                                                        \
    }                                                                     \
  } while (0)

static napi_value throw_lsg(napi_env env, lsg_ctx* ctx, const char* what, int rc) {
  char msg[512];
  snprintf(msg, sizeof msg, "%s failed (status %d): %s", what, rc, ctx ? lsg_last_error(ctx) : "");
  napi_throw_error(env, NULL, msg);
  return NULL;
}

/* the external of a context is an addon_ctx (defined with the package engine below) whose
 * first member is the lsg_ctx (NULL once closed) */
static lsg_ctx* get_ctx(napi_env env, napi_value v) {
  void* p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, NULL, "lsg_napi: expected a context from open()");
    return NULL;
  }
  lsg_ctx* c = *(lsg_ctx**)p;
  if (!c) napi_throw_error(env, NULL, "lsg_napi: the context is closed");
  return c;
}

/* Uint8Array (or Buffer) -> pointer + length; returns 0 on success */
static int get_bytes(napi_env env, napi_value v, const uint8_t** data, size_t* len) {
  bool is_ta = false;
  if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return -1;
  napi_typedarray_type t;
  size_t n;
  void* d;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, &n, &d, &ab, &off) != napi_ok || t != napi_uint8_array) return -1;
  *data = (const uint8_t*)d;
  *len = n;
  return 0;
}

/* Uint32Array -> pointer + element count; returns 0 on success */
static int get_u32s(napi_env env, napi_value v, const uint32_t** data, size_t* n) {
  bool is_ta = false;
  if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return -1;
  napi_typedarray_type t;
  void* d;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, n, &d, &ab, &off) != napi_ok || t != napi_uint32_array) return -1;
  *data = (const uint32_t*)d;
  return 0;
}

static napi_value get_prop(napi_env env, napi_value obj, const char* name) {
  napi_value v = NULL;
  if (napi_get_named_property(env, obj, name, &v) != napi_ok) return NULL;
  return v;
}

static uint32_t array_len(napi_env env, napi_value arr) {
  uint32_t n = 0;
  bool is_arr = false;
  if (napi_is_array(env, arr, &is_arr) != napi_ok || !is_arr) return UINT32_MAX;
  napi_get_array_length(env, arr, &n);
  return n;
}

/* Flattened host view of JS signature sets.  Pubkeys of an aggregate set are packed into
 * one owned buffer (lsg_set wants n_pks keys back to back); everything else points at the
 * JS buffers, which stay alive for the duration of the synchronous call. */
typedef struct {
  lsg_set* sets;
  uint8_t** owned;
  size_t n_sets, n_owned;
} set_view;

static void view_free(set_view* v) {
  for (size_t i = 0; i < v->n_owned; i++) free(v->owned[i]);
  free(v->owned);
  free(v->sets);
  memset(v, 0, sizeof *v);
}

/* returns 0 on success, else throws and returns -1 */
static int view_sets(napi_env env, napi_value arr, set_view* out) {
  memset(out, 0, sizeof *out);
  uint32_t n = array_len(env, arr);
  if (n == UINT32_MAX) {
    napi_throw_type_error(env, NULL, "lsg_napi: sets must be an array");
    return -1;
  }
  out->sets = (lsg_set*)calloc(n ? n : 1, sizeof(lsg_set));
  out->owned = (uint8_t**)calloc(n ? n : 1, sizeof(uint8_t*));
  out->n_sets = n;
  for (uint32_t i = 0; i < n; i++) {
    napi_value s;
    napi_get_element(env, arr, i, &s);
    lsg_set* q = &out->sets[i];
    const uint8_t* d;
    size_t len;
    napi_value m = get_prop(env, s, "message"), g = get_prop(env, s, "signature"), pk = get_prop(env, s, "pubkeys");
    if (!m || get_bytes(env, m, &d, &len)) goto bad;
    q->msg = d;
    q->msg_len = (uint32_t)len;
    if (!g || get_bytes(env, g, &d, &len)) goto bad;
    q->sig = d;
    q->sig_len = (uint32_t)len;
    /* signers by validator index into the device pubkey table (lsg_pubkey_table_set) */
    napi_value pki = get_prop(env, s, "pubkeyIndices");
    napi_valuetype pkit = napi_undefined;
    if (pki) napi_typeof(env, pki, &pkit);
    if (pki && pkit != napi_undefined) {
      const uint32_t* ix;
      size_t nix;
      if (get_u32s(env, pki, &ix, &nix)) goto bad;
      q->pks = (const uint8_t*)ix;
      q->pk_len = LSG_PK_INDEX;
      q->n_pks = (uint32_t)nix;
      continue;
    }
    uint32_t npk = pk ? array_len(env, pk) : UINT32_MAX;
    if (npk == UINT32_MAX) goto bad;
    q->n_pks = npk;
    q->pk_len = 96;
    if (npk == 0) {
      q->pks = NULL;
    } else {
      napi_value k0;
      napi_get_element(env, pk, 0, &k0);
      if (get_bytes(env, k0, &d, &len)) goto bad;
      q->pk_len = (uint32_t)len;
      if (npk == 1) {
        q->pks = d;
      } else {
        uint8_t* buf = (uint8_t*)malloc((size_t)npk * len);
        out->owned[out->n_owned++] = buf;
        for (uint32_t k = 0; k < npk; k++) {
          napi_value kk;
          const uint8_t* dk;
          size_t lk;
          napi_get_element(env, pk, k, &kk);
          if (get_bytes(env, kk, &dk, &lk) || lk != len) {
            napi_throw_type_error(env, NULL, "lsg_napi: every pubkey of a set must have the same encoding");
            view_free(out);
            return -1;
          }
          memcpy(buf + (size_t)k * len, dk, len);
        }
        q->pks = buf;
      }
    }
  }
  return 0;
bad:
  view_free(out);
  napi_throw_type_error(env, NULL,
                        "lsg_napi: a set is {pubkeys: Uint8Array[] | pubkeyIndices: Uint32Array, message: Uint8Array, "
                        "signature: Uint8Array}");
  return -1;
}

static napi_value make_int(napi_env env, int64_t x) {
  napi_value v;
  napi_create_double(env, (double)x, &v);
  return v;
}

static void set_int(napi_env env, napi_value obj, const char* name, int64_t x) {
  napi_set_named_property(env, obj, name, make_int(env, x));
}

static napi_value make_result(napi_env env, const lsg_job_result* r) {
  napi_value o;
  napi_create_object(env, &o);
  set_int(env, o, "status", r->status);
  set_int(env, o, "errCode", r->err_code);
  return o;
}

static napi_value js_reserve(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  double v[4] = {0, 0, 0, 0};
  for (size_t k = 1; k < argc && k < 5; k++) napi_get_value_double(env, argv[k], &v[k - 1]);
  int rc = lsg_reserve(ctx, (size_t)v[0], (size_t)v[1], (size_t)v[2], (int32_t)v[3]);
  if (rc) return throw_lsg(env, ctx, "lsg_reserve", rc);
  return NULL;
}

static napi_value js_device_count(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  int32_t n = 0;
  int rc = lsg_device_count(ctx, &n);
  if (rc) return throw_lsg(env, ctx, "lsg_device_count", rc);
  return make_int(env, n);
}

/* the packages this addon keeps in flight per context: one per package thread, at most the
 * library's pipeline slots (BlsGpuVerifier's poolSize, the reference's worker count) */
static napi_value js_slots(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  int32_t n = 0;
  int rc = lsg_pipeline_slots(ctx, &n);
  if (rc) return throw_lsg(env, ctx, "lsg_pipeline_slots", rc);
  return make_int(env, n < LSG_NAPI_THREADS ? n : LSG_NAPI_THREADS);
}

static napi_value js_device_name(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  char buf[256];
  int rc = lsg_device_name(ctx, buf, sizeof buf);
  if (rc) return throw_lsg(env, ctx, "lsg_device_name", rc);
  napi_value s;
  NAPI_CALL(env, napi_create_string_utf8(env, buf, NAPI_AUTO_LENGTH, &s));
  return s;
}

/* ------------------------------------------------------------------ packages (async engine)
 * verifyPacked(ctx, arena, setDesc, jobDesc, seed) -> Promise<result>
 *   arena    Uint8Array: every byte of the package's sets (keys, messages, signatures)
 *   setDesc  Uint32Array, 7 words per set: pkOff, pkLen (48|96|4 = index), nPks, msgOff,
 *            msgLen, sigOff, sigLen (offsets into arena; sets in job order)
 *   jobDesc  Uint32Array, 2 words per job: nSets, flags (LSG_JOB_*)
 *   result   {status: Uint8Array(nJobs), errCode: Int32Array(nJobs), batchRetries,
 *             batchSigsSuccess, startNs, endNs, finalExps, submitUs, keyError, workerId}
 * The call returns at once.  One of the context's package threads (native, not libuv's pool)
 * builds the lsg_job list over the arena, calls lsg_submit_jobs (the inputs are copied into
 * pinned staging there) and blocks in lsg_wait_jobs; the verdicts come back to the JS thread
 * through a napi_threadsafe_function, which resolves the promise.  The JS buffers are held by
 * references until then and must not be modified by the caller.  The JS thread never blocks
 * on the GPU and never stages bytes: it only packs the arena (the role of the structured
 * clone of multithread/index.ts:335) and resolves per-job promises. */
#include <pthread.h>


typedef struct pkg_req {
  struct pkg_req* next;
  napi_deferred deferred;
  napi_ref refs[3]; /* arena, setDesc, jobDesc: kept alive until the promise settles */
  const uint8_t* arena;
  size_t arena_len;
  const uint32_t* sdesc;
  const uint32_t* jdesc;
  uint32_t n_sets, n_jobs;
  uint64_t seed;
  lsg_ticket ticket;
  lsg_job_result* results;
  lsg_stats stats;
  int rc;
  char err[320];
} pkg_req;

typedef struct addon_ctx addon_ctx;
typedef struct {
  addon_ctx* a;
  int prio_only; /* the priority thread: serves only the priority queue */
} engine_arg;

struct addon_ctx {
  lsg_ctx* c;
  /* engine (started by the first verifyPacked): LSG_NAPI_THREADS package threads plus one
   * priority thread, so that a priority package (verifyOnMainThread) never waits for a
   * package thread blocked on an earlier package */
  int started, stop, n_threads;
  pthread_t th[LSG_NAPI_THREADS + 1];
  engine_arg targ[LSG_NAPI_THREADS + 1];
  pthread_mutex_t mu;
  pthread_cond_t cv;
  pkg_req *head, *tail;   /* packages, FIFO */
  pkg_req *phead, *ptail; /* priority packages, FIFO, served first by every thread */
  napi_threadsafe_function tsfn;
  uint32_t pending; /* promises not yet settled (JS thread only) */
};

static addon_ctx* get_actx(napi_env env, napi_value v) {
  void* p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, NULL, "lsg_napi: expected a context from open()");
    return NULL;
  }
  return (addon_ctx*)p;
}

/* the sets of a package over the arena; returns 0 or an LSG_ERR_* (bounds are checked here:
 * a descriptor naming bytes outside the arena is an argument error, never a wild read) */
static int build_jobs(pkg_req* r, lsg_set** sets_out, lsg_job** jobs_out) {
  lsg_set* sets = (lsg_set*)calloc(r->n_sets ? r->n_sets : 1, sizeof(lsg_set));
  lsg_job* jobs = (lsg_job*)calloc(r->n_jobs ? r->n_jobs : 1, sizeof(lsg_job));
  if (!sets || !jobs) {
    free(sets);
    free(jobs);
    return LSG_ERR_NOMEM;
  }
  const uint64_t L = r->arena_len;
  for (uint32_t i = 0; i < r->n_sets; i++) {
    const uint32_t* d = r->sdesc + 7 * (size_t)i;
    lsg_set* q = &sets[i];
    const uint64_t pk_bytes = (uint64_t)d[1] * d[2];
    if ((uint64_t)d[0] + pk_bytes > L || (uint64_t)d[3] + d[4] > L || (uint64_t)d[5] + d[6] > L) {
      free(sets);
      free(jobs);
      return LSG_ERR_INVALID_ARG;
    }
    q->pks = r->arena + d[0];
    q->pk_len = d[1];
    q->n_pks = d[2];
    q->msg = r->arena + d[3];
    q->msg_len = d[4];
    q->sig = r->arena + d[5];
    q->sig_len = d[6];
  }
  uint64_t pos = 0;
  for (uint32_t j = 0; j < r->n_jobs; j++) {
    jobs[j].n_sets = r->jdesc[2 * (size_t)j];
    jobs[j].flags = r->jdesc[2 * (size_t)j + 1];
    jobs[j].sets = sets + pos;
    pos += jobs[j].n_sets;
  }
  if (pos != r->n_sets) {
    free(sets);
    free(jobs);
    return LSG_ERR_INVALID_ARG;
  }
  *sets_out = sets;
  *jobs_out = jobs;
  return LSG_OK;
}

static void* engine_main(void* arg) {
  addon_ctx* a = ((engine_arg*)arg)->a;
  const int prio_only = ((engine_arg*)arg)->prio_only;
  for (;;) {
    pthread_mutex_lock(&a->mu);
    while (!a->phead && (prio_only || !a->head) && !a->stop) pthread_cond_wait(&a->cv, &a->mu);
    pkg_req* r = a->phead;
    if (r) {
      a->phead = r->next;
      if (!a->phead) a->ptail = NULL;
    } else if (!prio_only && a->head) {
      r = a->head;
      a->head = r->next;
      if (!a->head) a->tail = NULL;
    }
    if (!r) { /* stopping and drained */
      pthread_mutex_unlock(&a->mu);
      break;
    }
    pthread_mutex_unlock(&a->mu);
    lsg_set* sets = NULL;
    lsg_job* jobs = NULL;
    r->rc = build_jobs(r, &sets, &jobs);
    if (r->rc == LSG_OK) {
      /* at most n_threads (the package threads plus the priority thread) <= lsg_pipeline_slots
       * packages are outstanding per context (engine_start), so BUSY only means another host
       * thread of this process shares the context: back off */
      for (int tries = 0;; tries++) {
        r->rc = lsg_submit_jobs(a->c, jobs, r->n_jobs, r->seed, &r->ticket);
        if (r->rc != LSG_ERR_BUSY || tries > 100000) break;
        struct timespec ts = {0, 200000};
        nanosleep(&ts, NULL);
      }
      /* a coalesced ticket still held while every slot is busy waits with LSG_ERR_BUSY until
       * another package's wait frees one (lsg_host.hip wait_merged): back off and wait again */
      for (int tries = 0; r->rc == LSG_OK; tries++) {
        const int wrc = lsg_wait_jobs(a->c, r->ticket, r->results, &r->stats);
        if (wrc != LSG_ERR_BUSY || tries > 100000) {
          r->rc = wrc;
          break;
        }
        struct timespec ts = {0, 200000};
        nanosleep(&ts, NULL);
      }
    }
    if (r->rc) snprintf(r->err, sizeof r->err, "lsg_submit_jobs/lsg_wait_jobs failed (status %d): %s", r->rc, lsg_last_error(a->c));
    free(sets);
    free(jobs);
    napi_call_threadsafe_function(a->tsfn, r, napi_tsfn_blocking);
  }
  return NULL;
}

/* JS thread: settle one package's promise */
static void engine_deliver(napi_env env, napi_value js_cb, void* context, void* data) {
  (void)js_cb;
  addon_ctx* a = (addon_ctx*)context;
  pkg_req* r = (pkg_req*)data;
  if (env) {
    if (r->rc != LSG_OK) {
      napi_value msg, err;
      napi_create_string_utf8(env, r->err, NAPI_AUTO_LENGTH, &msg);
      napi_create_error(env, NULL, msg, &err);
      napi_reject_deferred(env, r->deferred, err);
    } else {
      napi_value o, st, ec, ab;
      void* p;
      napi_create_object(env, &o);
      napi_create_arraybuffer(env, r->n_jobs ? r->n_jobs : 1, &p, &ab);
      for (uint32_t i = 0; i < r->n_jobs; i++) ((uint8_t*)p)[i] = (uint8_t)r->results[i].status;
      napi_create_typedarray(env, napi_uint8_array, r->n_jobs, ab, 0, &st);
      napi_create_arraybuffer(env, 4 * (size_t)(r->n_jobs ? r->n_jobs : 1), &p, &ab);
      for (uint32_t i = 0; i < r->n_jobs; i++) ((int32_t*)p)[i] = r->results[i].err_code;
      napi_create_typedarray(env, napi_int32_array, r->n_jobs, ab, 0, &ec);
      napi_set_named_property(env, o, "status", st);
      napi_set_named_property(env, o, "errCode", ec);
      set_int(env, o, "batchRetries", r->stats.batch_retries);
      set_int(env, o, "batchSigsSuccess", r->stats.batch_sigs_success);
      set_int(env, o, "startNs", (int64_t)r->stats.start_ns);
      set_int(env, o, "endNs", (int64_t)r->stats.end_ns);
      set_int(env, o, "finalExps", r->stats.n_final_exps);
      set_int(env, o, "submitUs", r->stats.submit_us);
      set_int(env, o, "keyError", r->stats.key_error);
      set_int(env, o, "workerId", (int64_t)(r->ticket & 0xff));
      napi_resolve_deferred(env, r->deferred, o);
    }
    for (int k = 0; k < 3; k++)
      if (r->refs[k]) napi_delete_reference(env, r->refs[k]);
    if (a->pending && --a->pending == 0) napi_unref_threadsafe_function(env, a->tsfn);
  }
  free(r->results);
  free(r);
}

static int engine_start(napi_env env, addon_ctx* a) {
  if (a->started) return 0;
  napi_value name;
  if (napi_create_string_utf8(env, "lsg_packages", NAPI_AUTO_LENGTH, &name) != napi_ok) return -1;
  if (napi_create_threadsafe_function(env, NULL, NULL, name, 0, 1, NULL, NULL, a, engine_deliver, &a->tsfn) != napi_ok)
    return -1;
  napi_unref_threadsafe_function(env, a->tsfn); /* an idle verifier does not keep node alive */
  pthread_mutex_init(&a->mu, NULL);
  pthread_cond_init(&a->cv, NULL);
  int32_t slots = LSG_NAPI_THREADS;
  lsg_pipeline_slots(a->c, &slots);
  /* package threads: min(slots - 1, LSG_NAPI_THREADS), so that the priority thread always finds
   * a free slot (with fewer slots than threads it would spin on BUSY behind the packages).  One
   * slot: one thread, which serves the priority queue first like every package thread. */
  int pkg_threads = slots - 1 < LSG_NAPI_THREADS ? slots - 1 : LSG_NAPI_THREADS;
  const int prio_thread = pkg_threads >= 1;
  if (pkg_threads < 1) pkg_threads = 1;
  a->n_threads = pkg_threads + prio_thread;
  a->started = 1;
  for (int i = 0; i < a->n_threads; i++) {
    a->targ[i].a = a;
    a->targ[i].prio_only = prio_thread && i == a->n_threads - 1;
    pthread_create(&a->th[i], NULL, engine_main, &a->targ[i]);
  }
  return 0;
}

/* join the package threads (every promise has settled: BlsGpuVerifier.close awaits them) */
static void engine_stop(addon_ctx* a) {
  if (!a->started) return;
  pthread_mutex_lock(&a->mu);
  a->stop = 1;
  pthread_cond_broadcast(&a->cv);
  pthread_mutex_unlock(&a->mu);
  for (int i = 0; i < a->n_threads; i++) pthread_join(a->th[i], NULL);
  napi_release_threadsafe_function(a->tsfn, napi_tsfn_release);
  pthread_mutex_destroy(&a->mu);
  pthread_cond_destroy(&a->cv);
  a->started = 0;
}

static int typed_info(napi_env env, napi_value v, napi_typedarray_type want, void** data, size_t* n) {
  bool is_ta = false;
  napi_typedarray_type t;
  napi_value ab;
  size_t off;
  if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return -1;
  if (napi_get_typedarray_info(env, v, &t, n, data, &ab, &off) != napi_ok || t != want) return -1;
  return 0;
}

static napi_value js_verify_packed(napi_env env, napi_callback_info info) {
  size_t argc = 6;
  napi_value argv[6];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* a = get_actx(env, argv[0]);
  if (!a) return NULL;
  void *arena, *sd, *jd;
  size_t na, ns, nj;
  if (argc < 4 || typed_info(env, argv[1], napi_uint8_array, &arena, &na) ||
      typed_info(env, argv[2], napi_uint32_array, &sd, &ns) || typed_info(env, argv[3], napi_uint32_array, &jd, &nj) ||
      ns % 7 || nj % 2) {
    napi_throw_type_error(env, NULL, "lsg_napi: verifyPacked(ctx, arena: Uint8Array, setDesc: Uint32Array(7n), jobDesc: Uint32Array(2m), seed)");
    return NULL;
  }
  double seedd = 0;
  if (argc >= 5) napi_get_value_double(env, argv[4], &seedd);
  bool prio = false;
  if (argc >= 6) napi_get_value_bool(env, argv[5], &prio);
  if (engine_start(env, a)) {
    napi_throw_error(env, NULL, "lsg_napi: could not start the package threads");
    return NULL;
  }
  pkg_req* r = (pkg_req*)calloc(1, sizeof(pkg_req));
  r->arena = (const uint8_t*)arena;
  r->arena_len = na;
  r->sdesc = (const uint32_t*)sd;
  r->jdesc = (const uint32_t*)jd;
  r->n_sets = (uint32_t)(ns / 7);
  r->n_jobs = (uint32_t)(nj / 2);
  r->seed = (uint64_t)seedd;
  r->results = (lsg_job_result*)calloc(r->n_jobs ? r->n_jobs : 1, sizeof(lsg_job_result));
  for (int k = 0; k < 3; k++) napi_create_reference(env, argv[1 + k], 1, &r->refs[k]);
  napi_value promise;
  NAPI_CALL(env, napi_create_promise(env, &r->deferred, &promise));
  if (a->pending++ == 0) napi_ref_threadsafe_function(env, a->tsfn);
  pthread_mutex_lock(&a->mu);
  if (prio) {
    if (a->ptail)
      a->ptail->next = r;
    else
      a->phead = r;
    a->ptail = r;
    pthread_cond_broadcast(&a->cv); /* the priority thread may be the only one free */
  } else {
    if (a->tail)
      a->tail->next = r;
    else
      a->head = r;
    a->tail = r;
    /* broadcast, not signal: one wakeup could go to the priority thread, which does not
     * take this package, and the package threads would sleep on */
    pthread_cond_broadcast(&a->cv);
  }
  pthread_mutex_unlock(&a->mu);
  return promise;
}

/* ------------------------------------------------------------------ open / close */
static void engine_stop(addon_ctx* a);
static void finalize_actx(napi_env env, void* data, void* hint) {
  (void)env;
  (void)hint;
  addon_ctx* a = (addon_ctx*)data;
  if (!a->c && !a->started) free(a); /* an unclosed context lives until the process exits */
}

static napi_value js_open(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = NULL;
  int rc;
  bool is_arr = false;
  /* the package threads sleep on the completion events instead of spinning (the library's
   * LSG_BLOCKING_WAITS; an explicit setting in the environment wins) */
  setenv("LSG_BLOCKING_WAITS", "1", 0);
  if (argc >= 1) napi_is_array(env, argv[0], &is_arr);
  if (is_arr) {
    uint32_t n = array_len(env, argv[0]);
    if (n == 0 || n > 64) {
      napi_throw_range_error(env, NULL, "lsg_napi: open() expects 1..64 device ids");
      return NULL;
    }
    int ids[64];
    for (uint32_t k = 0; k < n; k++) {
      napi_value e;
      napi_get_element(env, argv[0], k, &e);
      int32_t d = 0;
      napi_get_value_int32(env, e, &d);
      ids[k] = d;
    }
    rc = lsg_init_devices(ids, (int)n, &ctx);
  } else {
    int32_t dev = 0;
    if (argc >= 1) napi_get_value_int32(env, argv[0], &dev);
    rc = lsg_init(dev, &ctx);
  }
  if (rc != LSG_OK) return throw_lsg(env, NULL, "lsg_init (no gfx950 device?)", rc);
  addon_ctx* a = (addon_ctx*)calloc(1, sizeof(addon_ctx));
  a->c = ctx;
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, a, finalize_actx, NULL, &ext));
  return ext;
}

static napi_value js_close(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* a = get_actx(env, argv[0]);
  if (!a || !a->c) return NULL;
  engine_stop(a);
  lsg_destroy(a->c);
  a->c = NULL;
  return NULL;
}

static napi_value js_verify_sets(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  double seedd = 0;
  if (argc >= 3) napi_get_value_double(env, argv[2], &seedd);
  set_view v;
  if (view_sets(env, argv[1], &v)) return NULL;
  lsg_job_result r;
  int rc = lsg_verify_sets(ctx, v.sets, v.n_sets, (uint64_t)seedd, &r);
  view_free(&v);
  if (rc) return throw_lsg(env, ctx, "lsg_verify_sets", rc);
  return make_result(env, &r);
}

/* ------------------------------------------------------------------ parity exports */
static napi_value js_aggregate_pubkeys(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  uint32_t n = array_len(env, argv[1]);
  if (n == UINT32_MAX) {
    napi_throw_type_error(env, NULL, "lsg_napi: pubkeys must be an array");
    return NULL;
  }
  size_t len = 96;
  uint8_t* buf = NULL;
  for (uint32_t k = 0; k < n; k++) {
    napi_value kk;
    const uint8_t* d;
    size_t l;
    napi_get_element(env, argv[1], k, &kk);
    if (get_bytes(env, kk, &d, &l) || (k > 0 && l != len)) {
      free(buf);
      napi_throw_type_error(env, NULL, "lsg_napi: pubkeys must be Uint8Arrays of one encoding");
      return NULL;
    }
    if (k == 0) {
      len = l;
      buf = (uint8_t*)malloc((size_t)n * len);
    }
    memcpy(buf + (size_t)k * len, d, len);
  }
  void* outp;
  napi_value ab, out, o;
  NAPI_CALL(env, napi_create_arraybuffer(env, 96, &outp, &ab));
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, 96, ab, 0, &out));
  int32_t err = 0;
  int rc = lsg_aggregate_pubkeys(ctx, buf, (uint32_t)len, n, (uint8_t*)outp, &err);
  free(buf);
  if (rc) return throw_lsg(env, ctx, "lsg_aggregate_pubkeys", rc);
  NAPI_CALL(env, napi_create_object(env, &o));
  set_int(env, o, "errCode", err);
  napi_set_named_property(env, o, "bytes", out);
  return o;
}

/* pubkeyTableSet(ctx, firstIndex, pubkeys: Uint8Array[]) -> errCodes: number[]  (8f(1)) */
static napi_value js_pubkey_table_set(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  int64_t first = 0;
  uint32_t n = array_len(env, argv[2]);
  if (napi_get_value_int64(env, argv[1], &first) != napi_ok || first < 0 || n == UINT32_MAX) {
    napi_throw_type_error(env, NULL, "lsg_napi: pubkeyTableSet(ctx, firstIndex, pubkeys: Uint8Array[])");
    return NULL;
  }
  size_t len = 96;
  uint8_t* buf = NULL;
  for (uint32_t k = 0; k < n; k++) {
    napi_value kk;
    const uint8_t* d;
    size_t l;
    napi_get_element(env, argv[2], k, &kk);
    if (get_bytes(env, kk, &d, &l) || (k > 0 && l != len)) {
      free(buf);
      napi_throw_type_error(env, NULL, "lsg_napi: pubkeys must be Uint8Arrays of one encoding");
      return NULL;
    }
    if (k == 0) {
      len = l;
      buf = (uint8_t*)malloc((size_t)n * len);
    }
    memcpy(buf + (size_t)k * len, d, len);
  }
  int32_t* err = (int32_t*)calloc(n ? n : 1, sizeof(int32_t));
  int rc = n ? lsg_pubkey_table_set(ctx, (size_t)first, buf, (uint32_t)len, n, err) : LSG_OK;
  free(buf);
  if (rc) {
    free(err);
    return throw_lsg(env, ctx, "lsg_pubkey_table_set", rc);
  }
  napi_value out;
  NAPI_CALL(env, napi_create_array_with_length(env, n, &out));
  for (uint32_t k = 0; k < n; k++) napi_set_element(env, out, k, make_int(env, err[k]));
  free(err);
  return out;
}

static napi_value js_hash_to_g2(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  const uint8_t *m, *d;
  size_t ml, dl;
  if (get_bytes(env, argv[1], &m, &ml) || get_bytes(env, argv[2], &d, &dl)) {
    napi_throw_type_error(env, NULL, "lsg_napi: hashToG2(ctx, message: Uint8Array, dst: Uint8Array)");
    return NULL;
  }
  void* outp;
  napi_value ab, out;
  NAPI_CALL(env, napi_create_arraybuffer(env, 192, &outp, &ab));
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, 192, ab, 0, &out));
  int rc = lsg_hash_to_g2(ctx, m, (uint32_t)ml, 1, d, (uint32_t)dl, (uint8_t*)outp);
  if (rc) return throw_lsg(env, ctx, "lsg_hash_to_g2", rc);
  return out;
}

/* aggregateSignatures(ctx, groups: Uint8Array[][]) -> [{signature: Uint8Array(96) | null, err}]
 * -- the op pools' bls.Signature.aggregate(sigs.map(signatureFromBytesNoCheck)).toBytes()
 * for every group in one device pass (8f(4), lsg_aggregate_signatures). */
static napi_value js_aggregate_signatures(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  uint32_t ng = array_len(env, argv[1]);
  if (ng == UINT32_MAX) {
    napi_throw_type_error(env, NULL, "lsg_napi: aggregateSignatures(ctx, groups: Uint8Array[][])");
    return NULL;
  }
  uint32_t* offs = (uint32_t*)calloc((size_t)ng + 1, sizeof(uint32_t));
  size_t total = 0, len = 0;
  for (uint32_t g = 0; g < ng; g++) {
    napi_value grp;
    napi_get_element(env, argv[1], g, &grp);
    uint32_t n = array_len(env, grp);
    if (n == UINT32_MAX) {
      free(offs);
      napi_throw_type_error(env, NULL, "lsg_napi: each group must be an array of signatures");
      return NULL;
    }
    total += n;
    offs[g + 1] = (uint32_t)total;
  }
  uint8_t* buf = (uint8_t*)malloc(total ? total * 192 : 1);
  size_t k = 0;
  for (uint32_t g = 0; g < ng; g++) {
    napi_value grp;
    napi_get_element(env, argv[1], g, &grp);
    for (uint32_t i = 0; i < offs[g + 1] - offs[g]; i++, k++) {
      napi_value sv;
      const uint8_t* d;
      size_t l;
      napi_get_element(env, grp, i, &sv);
      if (get_bytes(env, sv, &d, &l) || (k > 0 && l != len) || l > 192) {
        free(buf);
        free(offs);
        napi_throw_type_error(env, NULL, "lsg_napi: signatures must be Uint8Arrays of one encoding");
        return NULL;
      }
      len = l;
      memcpy(buf + k * len, d, len);
    }
  }
  uint8_t* out = (uint8_t*)calloc(ng ? (size_t)ng * 96 : 1, 1);
  int32_t* err = (int32_t*)calloc(ng ? ng : 1, sizeof(int32_t));
  int rc = ng ? lsg_aggregate_signatures(ctx, buf, (uint32_t)(total ? len : 96), offs, ng, out, err) : LSG_OK;
  free(buf);
  free(offs);
  if (rc) {
    free(out);
    free(err);
    return throw_lsg(env, ctx, "lsg_aggregate_signatures", rc);
  }
  napi_value res;
  NAPI_CALL(env, napi_create_array_with_length(env, ng, &res));
  for (uint32_t g = 0; g < ng; g++) {
    napi_value o, sig;
    napi_create_object(env, &o);
    if (err[g] == 0) {
      void* p;
      napi_value ab;
      napi_create_arraybuffer(env, 96, &p, &ab);
      memcpy(p, out + 96 * (size_t)g, 96);
      napi_create_typedarray(env, napi_uint8_array, 96, ab, 0, &sig);
    } else {
      napi_get_null(env, &sig);
    }
    napi_set_named_property(env, o, "signature", sig);
    set_int(env, o, "err", err[g]);
    napi_set_element(env, res, g, o);
  }
  free(out);
  free(err);
  return res;
}

/* attestationSigningRoots(ctx, data: Uint8Array (n x 128 B SSZ AttestationData), domain: Uint8Array
 * (32 B shared, or n x 32 B)) -> Uint8Array(n x 32): getAttestationDataSigningRoot for n objects
 * (8f(3), lsg_attestation_signing_roots) */
static napi_value js_attestation_signing_roots(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  const uint8_t *d, *dom;
  size_t dl, doml;
  if (get_bytes(env, argv[1], &d, &dl) || get_bytes(env, argv[2], &dom, &doml) || dl % 128 ||
      (doml != 32 && doml != 32 * (dl / 128))) {
    napi_throw_type_error(env, NULL, "lsg_napi: attestationSigningRoots(ctx, data: n x 128 B, domain: 32 B | n x 32 B)");
    return NULL;
  }
  const size_t n = dl / 128;
  void* outp;
  napi_value ab, out;
  NAPI_CALL(env, napi_create_arraybuffer(env, 32 * n, &outp, &ab));
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, 32 * n, ab, 0, &out));
  uint32_t stride = doml == 32 ? 0 : 32;
  int rc = n ? lsg_attestation_signing_roots(ctx, d, n, dom, stride, (uint8_t*)outp) : LSG_OK;
  if (rc) return throw_lsg(env, ctx, "lsg_attestation_signing_roots", rc);
  return out;
}

/* sign(ctx, sks: Uint8Array(32n, big-endian), msgs: Uint8Array(32n)) -> Uint8Array(96n) and
 * skToPk(ctx, sks) -> Uint8Array(96n): test/bench input generation on the GPU (lsg_sign,
 * lsg_sk_to_pk), not on the verify path */
static napi_value js_sign(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  const uint8_t *k, *m;
  size_t kl, ml;
  if (argc < 3 || get_bytes(env, argv[1], &k, &kl) || get_bytes(env, argv[2], &m, &ml) || kl % 32 || ml != kl) {
    napi_throw_type_error(env, NULL, "lsg_napi: sign(ctx, sks: 32n bytes, msgs: 32n bytes)");
    return NULL;
  }
  const size_t n = kl / 32;
  void* outp;
  napi_value ab, out;
  NAPI_CALL(env, napi_create_arraybuffer(env, 96 * (n ? n : 1), &outp, &ab));
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, 96 * n, ab, 0, &out));
  int rc = n ? lsg_sign(ctx, k, m, 32, n, (uint8_t*)outp) : LSG_OK;
  if (rc) return throw_lsg(env, ctx, "lsg_sign", rc);
  return out;
}

static napi_value js_sk_to_pk(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  const uint8_t* k;
  size_t kl;
  if (argc < 2 || get_bytes(env, argv[1], &k, &kl) || kl % 32) {
    napi_throw_type_error(env, NULL, "lsg_napi: skToPk(ctx, sks: 32n bytes)");
    return NULL;
  }
  const size_t n = kl / 32;
  void* outp;
  napi_value ab, out;
  NAPI_CALL(env, napi_create_arraybuffer(env, 96 * (n ? n : 1), &outp, &ab));
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, 96 * n, ab, 0, &out));
  int rc = n ? lsg_sk_to_pk(ctx, k, n, (uint8_t*)outp) : LSG_OK;
  if (rc) return throw_lsg(env, ctx, "lsg_sk_to_pk", rc);
  return out;
}

/* ------------------------------------------------------------------ module */
static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"open", NULL, js_open, NULL, NULL, NULL, napi_enumerable, NULL},
      {"close", NULL, js_close, NULL, NULL, NULL, napi_enumerable, NULL},
      {"slots", NULL, js_slots, NULL, NULL, NULL, napi_enumerable, NULL},
      {"reserve", NULL, js_reserve, NULL, NULL, NULL, napi_enumerable, NULL},
      {"deviceCount", NULL, js_device_count, NULL, NULL, NULL, napi_enumerable, NULL},
      {"deviceName", NULL, js_device_name, NULL, NULL, NULL, napi_enumerable, NULL},
      {"verifyPacked", NULL, js_verify_packed, NULL, NULL, NULL, napi_enumerable, NULL},
      {"sign", NULL, js_sign, NULL, NULL, NULL, napi_enumerable, NULL},
      {"skToPk", NULL, js_sk_to_pk, NULL, NULL, NULL, napi_enumerable, NULL},
      {"verifySets", NULL, js_verify_sets, NULL, NULL, NULL, napi_enumerable, NULL},
      {"aggregatePubkeys", NULL, js_aggregate_pubkeys, NULL, NULL, NULL, napi_enumerable, NULL},
      {"hashToG2", NULL, js_hash_to_g2, NULL, NULL, NULL, napi_enumerable, NULL},
      {"pubkeyTableSet", NULL, js_pubkey_table_set, NULL, NULL, NULL, napi_enumerable, NULL},
      {"aggregateSignatures", NULL, js_aggregate_signatures, NULL, NULL, NULL, napi_enumerable, NULL},
      {"attestationSigningRoots", NULL, js_attestation_signing_roots, NULL, NULL, NULL, napi_enumerable, NULL},
  };
  NAPI_CALL(env, napi_define_properties(env, exports, sizeof props / sizeof props[0], props));
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
