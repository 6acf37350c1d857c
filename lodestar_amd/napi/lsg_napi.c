/*
 * lsg_napi.c -- thin N-API addon over the C ABI (include/lodestar_bls.h).
 *
 * This is the native half of BlsGpuVerifier (lodestar_amd/js/blsGpuVerifier.js), which
 * stands in for BlsMultiThreadWorkerPool
 * (/root/reference/packages/beacon-node/src/chain/bls/multithread/index.ts).  Where the
 * reference posts BlsWorkReq[] packages to @chainsafe/threads workers running
 * @chainsafe/blst (multithread/worker.ts:30-106), the verifier hands each package to
 * submitJobs() (inputs copied into pinned staging memory before it returns) and awaits
 * waitJobs(), whose blocking part runs on a libuv pool thread (napi_create_async_work), so
 * the JS main thread never blocks on the GPU.  Nothing here does arithmetic.
 *
 * JS surface (all synchronous unless noted):
 *   open(device | devices[]) -> ctx         lsg_init / lsg_init_devices (one context over the
 *                                           node's GPUs: chain.ts:195-198 builds one verifier)
 *   reserve(ctx, maxSets, maxPks, maxMsgBytes, nSlots)                  lsg_reserve
 *   deviceCount(ctx) -> n                   lsg_device_count
 *   close(ctx)                              lsg_destroy
 *   slots(ctx) -> n                         lsg_pipeline_slots
 *   deviceName(ctx) -> string               lsg_device_name
 *   submitJobs(ctx, jobs, seed) -> ticket | null (every slot busy)     lsg_submit_jobs
 *       jobs = [{sets: [{pubkeys: Uint8Array[], message: Uint8Array, signature: Uint8Array}],
 *                flags: number}]
 *   waitJobs(ctx, ticket) -> Promise<{results: [{status, errCode}], batchRetries,
 *                                     batchSigsSuccess, startNs, endNs, finalExps,
 *                                     workerId}>   lsg_wait_jobs
 *       startNs / endNs are CLOCK_MONOTONIC nanoseconds (process.hrtime.bigint()'s clock);
 *       workerId is the pipeline slot that ran the package (the reference's workerId label)
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

static lsg_ctx* get_ctx(napi_env env, napi_value v) {
  void* p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, NULL, "lsg_napi: expected a context from open()");
    return NULL;
  }
  return (lsg_ctx*)p;
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

/* ------------------------------------------------------------------ open / close */
static void finalize_noop(napi_env env, void* data, void* hint) {
  (void)env;
  (void)data;
  (void)hint;
}

static napi_value js_open(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = NULL;
  int rc;
  bool is_arr = false;
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
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, ctx, finalize_noop, NULL, &ext));
  return ext;
}

static napi_value js_close(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  lsg_destroy(ctx);
  return NULL;
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

static napi_value js_slots(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  int32_t n = 0;
  int rc = lsg_pipeline_slots(ctx, &n);
  if (rc) return throw_lsg(env, ctx, "lsg_pipeline_slots", rc);
  return make_int(env, n);
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

/* ------------------------------------------------------------------ jobs */
static napi_value js_submit_jobs(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  uint32_t nj = array_len(env, argv[1]);
  if (nj == UINT32_MAX) {
    napi_throw_type_error(env, NULL, "lsg_napi: jobs must be an array");
    return NULL;
  }
  double seedd = 0;
  if (argc >= 3) napi_get_value_double(env, argv[2], &seedd);
  lsg_job* jobs = (lsg_job*)calloc(nj ? nj : 1, sizeof(lsg_job));
  set_view* views = (set_view*)calloc(nj ? nj : 1, sizeof(set_view));
  napi_value ret = NULL;
  uint32_t built = 0;
  for (; built < nj; built++) {
    napi_value j;
    napi_get_element(env, argv[1], built, &j);
    napi_value sets = get_prop(env, j, "sets"), flags = get_prop(env, j, "flags");
    uint32_t f = 0;
    if (flags) napi_get_value_uint32(env, flags, &f);
    if (!sets || view_sets(env, sets, &views[built])) goto out;
    jobs[built].sets = views[built].sets;
    jobs[built].n_sets = (uint32_t)views[built].n_sets;
    jobs[built].flags = f;
  }
  {
    lsg_ticket t = 0;
    int rc = lsg_submit_jobs(ctx, jobs, nj, (uint64_t)seedd, &t);
    if (rc == LSG_ERR_BUSY) {
      napi_get_null(env, &ret);
    } else if (rc != LSG_OK) {
      throw_lsg(env, ctx, "lsg_submit_jobs", rc);
    } else {
      /* tickets are serial << 16 | kind << 8 | slot: exact in a double for 2^37 submissions */
      napi_value o;
      napi_create_object(env, &o);
      set_int(env, o, "ticket", (int64_t)t);
      set_int(env, o, "nJobs", nj);
      ret = o;
    }
  }
out:
  for (uint32_t k = 0; k < built && k < nj; k++) view_free(&views[k]);
  free(views);
  free(jobs);
  return ret;
}

typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  lsg_ctx* ctx;
  lsg_ticket ticket;
  uint32_t n;
  lsg_job_result* results;
  lsg_stats stats;
  int rc;
  char err[256];
} wait_req;

static void wait_execute(napi_env env, void* data) {
  (void)env;
  wait_req* w = (wait_req*)data;
  w->rc = lsg_wait_jobs(w->ctx, w->ticket, w->results, &w->stats);
  if (w->rc) snprintf(w->err, sizeof w->err, "lsg_wait_jobs failed (status %d): %s", w->rc, lsg_last_error(w->ctx));
}

static void wait_complete(napi_env env, napi_status status, void* data) {
  wait_req* w = (wait_req*)data;
  if (status != napi_ok || w->rc != LSG_OK) {
    napi_value msg, err;
    napi_create_string_utf8(env, w->rc ? w->err : "lsg_napi: async wait cancelled", NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, w->deferred, err);
  } else {
    napi_value o, arr;
    napi_create_object(env, &o);
    napi_create_array_with_length(env, w->n, &arr);
    for (uint32_t i = 0; i < w->n; i++) napi_set_element(env, arr, i, make_result(env, &w->results[i]));
    napi_set_named_property(env, o, "results", arr);
    set_int(env, o, "batchRetries", w->stats.batch_retries);
    set_int(env, o, "batchSigsSuccess", w->stats.batch_sigs_success);
    set_int(env, o, "startNs", (int64_t)w->stats.start_ns);
    set_int(env, o, "endNs", (int64_t)w->stats.end_ns);
    set_int(env, o, "finalExps", w->stats.n_final_exps);
    set_int(env, o, "workerId", (int64_t)(w->ticket & 0xff));
    napi_resolve_deferred(env, w->deferred, o);
  }
  napi_delete_async_work(env, w->work);
  free(w->results);
  free(w);
}

static napi_value js_wait_jobs(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  lsg_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  napi_value tv = get_prop(env, argv[1], "ticket"), nv = get_prop(env, argv[1], "nJobs");
  double t = 0;
  uint32_t n = 0;
  if (!tv || !nv || napi_get_value_double(env, tv, &t) != napi_ok || napi_get_value_uint32(env, nv, &n) != napi_ok) {
    napi_throw_type_error(env, NULL, "lsg_napi: waitJobs expects the object submitJobs returned");
    return NULL;
  }
  wait_req* w = (wait_req*)calloc(1, sizeof(wait_req));
  w->ctx = ctx;
  w->ticket = (lsg_ticket)t;
  w->n = n;
  w->results = (lsg_job_result*)calloc(n ? n : 1, sizeof(lsg_job_result));
  napi_value promise, name;
  NAPI_CALL(env, napi_create_promise(env, &w->deferred, &promise));
  NAPI_CALL(env, napi_create_string_utf8(env, "lsg_wait_jobs", NAPI_AUTO_LENGTH, &name));
  NAPI_CALL(env, napi_create_async_work(env, NULL, name, wait_execute, wait_complete, w, &w->work));
  NAPI_CALL(env, napi_queue_async_work(env, w->work));
  return promise;
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

/* ------------------------------------------------------------------ module */
static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"open", NULL, js_open, NULL, NULL, NULL, napi_enumerable, NULL},
      {"close", NULL, js_close, NULL, NULL, NULL, napi_enumerable, NULL},
      {"slots", NULL, js_slots, NULL, NULL, NULL, napi_enumerable, NULL},
      {"reserve", NULL, js_reserve, NULL, NULL, NULL, napi_enumerable, NULL},
      {"deviceCount", NULL, js_device_count, NULL, NULL, NULL, napi_enumerable, NULL},
      {"deviceName", NULL, js_device_name, NULL, NULL, NULL, napi_enumerable, NULL},
      {"submitJobs", NULL, js_submit_jobs, NULL, NULL, NULL, napi_enumerable, NULL},
      {"waitJobs", NULL, js_wait_jobs, NULL, NULL, NULL, napi_enumerable, NULL},
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
