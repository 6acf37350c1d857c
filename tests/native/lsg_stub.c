/*
 * lsg_stub.c -- a host-only stand-in for liblodestar_bls.so, for the sanitizer build of the
 * N-API addon (tests/test_napi_sanitizers.py).  TEST INFRASTRUCTURE ONLY: it does no BLS
 * arithmetic.  It keeps the library's contract where the addon depends on it --
 *   - lsg_submit_jobs copies every byte of the package before returning (the addon's
 *     package threads then free their lsg_set / lsg_job arrays), and lsg_wait_jobs may run on
 *     another thread, later (a small delay so that packages overlap);
 *   - per-job results follow the reference's error precedence (an empty job throws "Empty
 *     signature set", a wrong-size signature BLST_INVALID_SIZE, a wrong-size key
 *     BLST_BAD_ENCODING) and a toy verdict rule for the rest: a set is valid iff
 *     signature[0] == message[0] (tests/js/test_verifier_host.js uses the same rule);
 *   - a context is thread-safe (one mutex) and reports errors through lsg_last_error --
 * so AddressSanitizer / UBSan see the addon's real marshalling (verifyPacked's arena and
 * descriptors, threadsafe completion, close with packages in flight) under traffic.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lodestar_bls.h"

#define STUB_SLOTS 64

typedef struct {
  int used;
  uint64_t serial;
  uint32_t n_jobs;
  lsg_job_result* res;
  uint64_t start_ns;
  uint8_t* copy; /* the package's bytes, as the library's pinned staging holds them */
} stub_pkg;

struct lsg_ctx {
  pthread_mutex_t mu;
  char err[256];
  int n_dev;
  uint64_t next;
  stub_pkg pk[STUB_SLOTS];
};

static uint64_t now_ns(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

int lsg_init_devices(const int* ids, int n, lsg_ctx** out) {
  if (!ids || n < 1 || !out) return LSG_ERR_INVALID_ARG;
  lsg_ctx* c = (lsg_ctx*)calloc(1, sizeof(lsg_ctx));
  pthread_mutex_init(&c->mu, NULL);
  c->n_dev = n;
  c->next = 1;
  *out = c;
  return LSG_OK;
}
int lsg_init(int dev, lsg_ctx** out) { return lsg_init_devices(&dev, 1, out); }
int lsg_destroy(lsg_ctx* c) {
  if (!c) return LSG_ERR_INVALID_ARG;
  for (int i = 0; i < STUB_SLOTS; i++) {
    free(c->pk[i].res);
    free(c->pk[i].copy);
  }
  pthread_mutex_destroy(&c->mu);
  free(c);
  return LSG_OK;
}
int lsg_device_count(lsg_ctx* c, int32_t* n) {
  if (!c || !n) return LSG_ERR_INVALID_ARG;
  *n = c->n_dev;
  return LSG_OK;
}
const char* lsg_last_error(lsg_ctx* c) { return c ? c->err : "null context"; }
int lsg_device_name(lsg_ctx* c, char* buf, size_t len) {
  if (!c || !buf || !len) return LSG_ERR_INVALID_ARG;
  snprintf(buf, len, "host stub (no device)");
  return LSG_OK;
}
int lsg_reserve(lsg_ctx* c, size_t a, size_t b, size_t d, int32_t n) {
  (void)a, (void)b, (void)d;
  return c && n >= 0 ? LSG_OK : LSG_ERR_INVALID_ARG;
}
int lsg_pipeline_slots(lsg_ctx* c, int32_t* n) {
  if (!c || !n) return LSG_ERR_INVALID_ARG;
  *n = STUB_SLOTS;
  return LSG_OK;
}

static lsg_job_result job_verdict(const lsg_job* J) {
  lsg_job_result r = {LSG_INVALID, 0};
  if (J->n_sets == 0) return (lsg_job_result){LSG_ERROR, LSG_ERR_EMPTY_SET};
  int ok = 1;
  for (uint32_t q = 0; q < J->n_sets; q++) {
    const lsg_set* s = &J->sets[q];
    if (s->sig_len != 96 && s->sig_len != 192) return (lsg_job_result){LSG_ERROR, LSG_BLST_INVALID_SIZE};
    if (s->pk_len != 48 && s->pk_len != 96 && s->pk_len != LSG_PK_INDEX) return (lsg_job_result){LSG_ERROR, LSG_BLST_BAD_ENCODING};
    if (s->n_pks == 0) return (lsg_job_result){LSG_ERROR, LSG_ERR_EMPTY_AGGREGATE};
    ok = ok && s->msg_len > 0 && s->sig[0] == s->msg[0];
  }
  r.status = ok ? LSG_VALID : LSG_INVALID;
  return r;
}

int lsg_submit_jobs(lsg_ctx* c, const lsg_job* jobs, size_t n_jobs, uint64_t seed, lsg_ticket* t) {
  (void)seed;
  if (!c || !t || (n_jobs && !jobs)) return LSG_ERR_INVALID_ARG;
  size_t bytes = 0;
  for (size_t j = 0; j < n_jobs; j++) {
    if (jobs[j].n_sets && !jobs[j].sets) return LSG_ERR_INVALID_ARG;
    for (uint32_t q = 0; q < jobs[j].n_sets; q++) {
      const lsg_set* s = &jobs[j].sets[q];
      bytes += (size_t)s->n_pks * s->pk_len + s->msg_len + s->sig_len;
    }
  }
  /* read every byte now, as the library stages the package before returning */
  uint8_t* copy = (uint8_t*)malloc(bytes ? bytes : 1);
  size_t off = 0;
  lsg_job_result* res = (lsg_job_result*)calloc(n_jobs ? n_jobs : 1, sizeof(lsg_job_result));
  for (size_t j = 0; j < n_jobs; j++) {
    for (uint32_t q = 0; q < jobs[j].n_sets; q++) {
      const lsg_set* s = &jobs[j].sets[q];
      if (s->n_pks && s->pk_len) memcpy(copy + off, s->pks, (size_t)s->n_pks * s->pk_len), off += (size_t)s->n_pks * s->pk_len;
      if (s->msg_len) memcpy(copy + off, s->msg, s->msg_len), off += s->msg_len;
      if (s->sig_len) memcpy(copy + off, s->sig, s->sig_len), off += s->sig_len;
    }
    res[j] = job_verdict(&jobs[j]);
  }
  pthread_mutex_lock(&c->mu);
  int p = -1;
  for (int i = 0; i < STUB_SLOTS && p < 0; i++)
    if (!c->pk[i].used) p = i;
  if (p < 0) {
    snprintf(c->err, sizeof c->err, "all pipeline slots are busy");
    pthread_mutex_unlock(&c->mu);
    free(copy);
    free(res);
    return LSG_ERR_BUSY;
  }
  stub_pkg* k = &c->pk[p];
  free(k->res);
  free(k->copy);
  k->used = 1;
  k->serial = c->next++;
  k->n_jobs = (uint32_t)n_jobs;
  k->res = res;
  k->copy = copy;
  k->start_ns = now_ns();
  *t = (k->serial << 16) | (1u << 8) | (uint64_t)p;
  pthread_mutex_unlock(&c->mu);
  return LSG_OK;
}

int lsg_wait_jobs(lsg_ctx* c, lsg_ticket t, lsg_job_result* results, lsg_stats* stats) {
  if (!c) return LSG_ERR_INVALID_ARG;
  const int p = (int)(t & 255);
  struct timespec d = {0, 300000}; /* "device time": packages overlap */
  nanosleep(&d, NULL);
  pthread_mutex_lock(&c->mu);
  stub_pkg* k = p < STUB_SLOTS ? &c->pk[p] : NULL;
  if (!k || !k->used || k->serial != (t >> 16)) {
    pthread_mutex_unlock(&c->mu);
    return LSG_ERR_INVALID_ARG;
  }
  if (k->n_jobs && !results) {
    pthread_mutex_unlock(&c->mu);
    return LSG_ERR_INVALID_ARG;
  }
  memcpy(results, k->res, sizeof(lsg_job_result) * k->n_jobs);
  if (stats) {
    memset(stats, 0, sizeof *stats);
    stats->start_ns = k->start_ns;
    stats->end_ns = now_ns();
    stats->n_final_exps = 1;
  }
  k->used = 0;
  pthread_mutex_unlock(&c->mu);
  return LSG_OK;
}

int lsg_verify_sets(lsg_ctx* c, const lsg_set* sets, size_t n, uint64_t seed, lsg_job_result* r) {
  (void)seed;
  if (!c || !r || (n && !sets)) return LSG_ERR_INVALID_ARG;
  lsg_job J = {sets, (uint32_t)n, 0};
  *r = job_verdict(&J);
  return LSG_OK;
}

/* byte-level stand-ins of the utilities the addon exposes (every input byte is read, every
 * output byte written, so the sanitizers check the addon's buffer sizes) */
static uint8_t fold(const uint8_t* p, size_t n) {
  uint8_t x = 0;
  for (size_t i = 0; i < n; i++) x ^= p[i];
  return x;
}
int lsg_aggregate_pubkeys(lsg_ctx* c, const uint8_t* pks, uint32_t pk_len, size_t n, uint8_t* out96, int32_t* err) {
  if (!c || !out96 || !err || (n && !pks)) return LSG_ERR_INVALID_ARG;
  memset(out96, fold(pks, (size_t)n * pk_len), 96);
  *err = n ? 0 : LSG_ERR_EMPTY_AGGREGATE;
  return LSG_OK;
}
int lsg_pubkey_table_set(lsg_ctx* c, size_t first, const uint8_t* pks, uint32_t pk_len, size_t n, int32_t* err) {
  (void)first;
  if (!c || (n && !pks)) return LSG_ERR_INVALID_ARG;
  for (size_t k = 0; k < n; k++) {
    const uint8_t v = fold(pks + k * pk_len, pk_len);
    if (err) err[k] = (pk_len == 48 || pk_len == 96) && v != 0xff ? 0 : LSG_BLST_BAD_ENCODING;
  }
  return LSG_OK;
}
int lsg_hash_to_g2(lsg_ctx* c, const uint8_t* msgs, uint32_t msg_len, size_t n, const uint8_t* dst, uint32_t dst_len,
                   uint8_t* out192) {
  if (!c || !out192) return LSG_ERR_INVALID_ARG;
  for (size_t i = 0; i < n; i++) memset(out192 + 192 * i, fold(msgs + (size_t)msg_len * i, msg_len) ^ fold(dst, dst_len), 192);
  return LSG_OK;
}
int lsg_aggregate_signatures(lsg_ctx* c, const uint8_t* sigs, uint32_t sig_len, const uint32_t* offsets, size_t ng,
                             uint8_t* out96, int32_t* err) {
  if (!c || !offsets || (ng && (!out96 || !err))) return LSG_ERR_INVALID_ARG;
  for (size_t g = 0; g < ng; g++) {
    const size_t a = offsets[g], b = offsets[g + 1];
    err[g] = b == a ? LSG_ERR_EMPTY_AGGREGATE : (sig_len == 96 || sig_len == 192 ? 0 : LSG_BLST_INVALID_SIZE);
    memset(out96 + 96 * g, b > a ? fold(sigs + a * sig_len, (b - a) * sig_len) : 0, 96);
  }
  return LSG_OK;
}
int lsg_attestation_signing_roots(lsg_ctx* c, const uint8_t* data128, size_t n, const uint8_t* domain32, uint32_t stride,
                                  uint8_t* out32) {
  if (!c || !domain32 || (n && (!data128 || !out32))) return LSG_ERR_INVALID_ARG;
  for (size_t i = 0; i < n; i++) memset(out32 + 32 * i, fold(data128 + 128 * i, 128) ^ fold(domain32 + stride * i, 32), 32);
  return LSG_OK;
}
int lsg_sign(lsg_ctx* c, const uint8_t* sks32, const uint8_t* msgs, uint32_t msg_len, size_t n, uint8_t* out96) {
  if (!c || !out96 || (n && (!sks32 || !msgs))) return LSG_ERR_INVALID_ARG;
  for (size_t i = 0; i < n; i++) {
    memset(out96 + 96 * i, fold(sks32 + 32 * i, 32), 96);
    out96[96 * i] = msgs[(size_t)msg_len * i]; /* valid under the toy rule */
  }
  return LSG_OK;
}
int lsg_sk_to_pk(lsg_ctx* c, const uint8_t* sks32, size_t n, uint8_t* out96) {
  if (!c || !out96 || (n && !sks32)) return LSG_ERR_INVALID_ARG;
  for (size_t i = 0; i < n; i++) memset(out96 + 96 * i, fold(sks32 + 32 * i, 32), 96);
  return LSG_OK;
}
