/*
 * lodestar_bls.h -- C ABI of the MI355X (gfx950) BLS12-381 signature-set verifier.
 *
 * Drop-in boundary for Lodestar's IBlsVerifier hot path
 * (/root/reference/packages/beacon-node/src/chain/bls/interface.ts:20-51).  It replaces
 * the worker threads of BlsMultiThreadWorkerPool together with the crypto library they
 * call (@chainsafe/bls@7.1.1 -> @chainsafe/blst@0.2.8 -> supranational blst):
 *
 *   lsg_verify_jobs        <- multithread/worker.ts:30-106 verifyManySignatureSets
 *                             (+ maybeBatch.ts:16-39 verifySignatureSetsMaybeBatch,
 *                                worker.ts:108-114 deserializeSet)
 *   lsg_verify_sets        <- maybeBatch.ts:16-39 for one call (BlsSingleThreadVerifier,
 *                             singleThread.ts:14-35; verifyOnMainThread, index.ts:155-168)
 *   lsg_aggregate_pubkeys  <- utils.ts:11 PublicKey.aggregate (+ toBytes, index.ts:177)
 *   lsg_hash_to_g2         <- blst Hash_to_G2 inside Pairing.mul_n_aggregate
 *   lsg_sig_decode         <- maybeBatch.ts:23,36 Signature.fromBytes(bytes, affine, true)
 *   lsg_aggregate_signatures <- opPools Signature.aggregate
 *   lsg_*signing_roots     <- util/signingRoot.ts:7-13 computeSigningRoot
 *   lsg_submit_jobs /      <- the asynchronous lsg_submit / lsg_wait pair of SURVEY.md 8b:
 *   lsg_wait_jobs             one BlsWorkReq[] package in flight per pipeline slot
 *   lsg_init_devices       <- the node-wide pool (chain.ts:195-198, multithread/poolSize.ts:7):
 *                             one context over every GPU of the node
 *   lsg_jobs_partial /     <- the per-GPU half of a package for one-process-per-GPU hosts
 *   lsg_wait_jobs_node        (SURVEY.md 8e): Miller-loop product of the package group,
 *   lsg_batch_partial /       all-gathered by the caller, one final exponentiation
 *   lsg_final_*               (lsg_final_*), then the verdicts resolved with it
 *
 * Plain pointers and sizes only; every call returns an int status (LSG_OK = 0) and never
 * throws.  Verdicts and error codes follow blst's numbering (BLST_* below).  All compute
 * runs in HIP kernels on the context's device; there is no CPU fallback -- lsg_init fails
 * with LSG_ERR_NO_DEVICE when no gfx950 device is present.
 */
#ifndef LODESTAR_BLS_H
#define LODESTAR_BLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- call status */
#define LSG_OK 0
#define LSG_ERR_INVALID_ARG 1
#define LSG_ERR_NO_DEVICE 2
#define LSG_ERR_DEVICE 3
#define LSG_ERR_NOMEM 4
#define LSG_ERR_CLOSED 5
#define LSG_ERR_BUSY 6 /* every pipeline slot holds an outstanding ticket (canAcceptWork false) */
#define LSG_ERR_ENTROPY 7 /* the OS CSPRNG (getrandom) failed: no RLC randomizers, nothing verified */

/* ---- blst error codes (blst.h BLST_ERROR) + @chainsafe/blst's size error */
#define LSG_BLST_SUCCESS 0
#define LSG_BLST_BAD_ENCODING 1
#define LSG_BLST_POINT_NOT_ON_CURVE 2
#define LSG_BLST_POINT_NOT_IN_GROUP 3
#define LSG_BLST_AGGR_TYPE_MISMATCH 4
#define LSG_BLST_VERIFY_FAIL 5
#define LSG_BLST_PK_IS_INFINITY 6
#define LSG_BLST_BAD_SCALAR 7
#define LSG_BLST_INVALID_SIZE 10
/* non-blst job errors */
#define LSG_ERR_EMPTY_SET 100        /* maybeBatch.ts:29-31 "Empty signature set" */
#define LSG_ERR_EMPTY_AGGREGATE 101  /* PublicKey.aggregate([]) "EMPTY_AGGREGATE_ARRAY" */
#define LSG_ERR_BAD_INDEX 102        /* a pubkey index outside the loaded table (index2pubkey[i] undefined) */

/* lsg_set.pk_len value for keys given by validator index into the context's pubkey table
 * (lsg_pubkey_table_set): pks then points at n_pks uint32 indices (host byte order). */
#define LSG_PK_INDEX 4u

/* ---- job verdicts (WorkResult<boolean>, multithread/types.ts:21-24) */
#define LSG_INVALID 0 /* {code: success, result: false} */
#define LSG_VALID 1   /* {code: success, result: true}  */
#define LSG_ERROR 2   /* {code: error, error}           */

/* ---- job flags (VerifySignatureOpts, interface.ts:3-18; priority/same-message are extensions) */
#define LSG_JOB_BATCHABLE 1u
/* A package with a priority job (verifyOnMainThread, BlsGpuSingleThreadVerifier) is never held
 * by coalescing and runs on its slot's high-priority streams: its kernels are dispatched ahead
 * of the packages in flight.  Verdicts are unaffected. */
#define LSG_JOB_PRIORITY 2u

typedef struct lsg_ctx lsg_ctx;
typedef uint64_t lsg_ticket; /* handle of an in-flight submission */

/* One signature set (ISignatureSet, state-transition/src/util/signatureSets.ts:10-22).
 * Pubkeys are the set's n_pks keys back to back, each pk_len bytes (48 compressed or
 * 96 uncompressed, ZCash encoding).  n_pks == 1 is a "single" set, > 1 an "aggregate"
 * set whose keys are summed on the GPU.  sig_len other than 96/192 yields
 * BLST_INVALID_SIZE for the set, exactly as Signature.fromBytes does. */
typedef struct {
  const uint8_t* pks;
  uint32_t pk_len;
  uint32_t n_pks;
  const uint8_t* msg;
  uint32_t msg_len;
  const uint8_t* sig;
  uint32_t sig_len;
} lsg_set;

/* One job = one BlsWorkReq (multithread/types.ts:14-17): the sets of one
 * verifySignatureSets chunk (<= 128 sets) plus its options. */
typedef struct {
  const lsg_set* sets;
  uint32_t n_sets;
  uint32_t flags;
} lsg_job;

typedef struct {
  int32_t status;   /* LSG_VALID / LSG_INVALID / LSG_ERROR */
  int32_t err_code; /* BLST_* or LSG_ERR_EMPTY_* when status == LSG_ERROR */
} lsg_job_result;

/* BlsWorkResult counters (multithread/types.ts:26-38) */
typedef struct {
  uint32_t batch_retries;
  uint32_t batch_sigs_success;
  uint64_t start_ns;      /* CLOCK_MONOTONIC ns (process.hrtime's clock): submit entered */
  uint64_t end_ns;        /* CLOCK_MONOTONIC ns: verdicts resolved */
  uint32_t n_final_exps;  /* final exponentiations run (package, chunk and job groups; node check) */
  uint32_t submit_us;     /* host time inside lsg_submit_jobs (staging, randomizers, plans, launches) */
  int32_t key_error;      /* deserializeSet failure that rejected the whole package (BLST_*), 0: none */
  uint32_t key_error_job; /* caller index of the job holding that first bad key */
} lsg_stats;

/* A context over one or more devices.  Per device it owns 16 pipeline slots (each: a main
 * and a side HIP stream plus its own device buffers; lsg_pipeline_slots), and device 0 owns
 * 64 final-exponentiation entries on 8 streams (lsg_final_*).  Calls are serialised by an
 * internal mutex; waits block without holding it.
 *   lsg_init(d)              one device (d < 0: device 0)
 *   lsg_init_devices(ids, n) the node's GPUs (chain.ts:195-198 builds ONE verifier per node;
 *                            its pool spans every core, multithread/poolSize.ts:7).  A package
 *                            is split into whole jobs by cumulative set count; each device
 *                            reduces its share to one Fp12 partial, the partials are
 *                            all-gathered over RCCL (communicators owned by the context) and
 *                            one final exponentiation on device 0 checks the node; on failure
 *                            every device localises with its own check.
 *                            Duplicate ids (tests) exchange by device copies instead. */
int lsg_init(int device_ordinal, lsg_ctx** out);
int lsg_init_devices(const int* device_ids, int n_devices, lsg_ctx** out);
int lsg_destroy(lsg_ctx* ctx);
int lsg_device_count(lsg_ctx* ctx, int32_t* n);
const char* lsg_last_error(lsg_ctx* ctx);
int lsg_device_name(lsg_ctx* ctx, char* buf, size_t len);
/* Preallocate every device and pinned buffer of the first n_slots pipeline slots (0 = all) of
 * every device for packages of up to max_sets sets, max_pks keys and max_msg_bytes message
 * bytes, so that submissions within those bounds allocate nothing.  A context over n devices
 * reserves each device for its share: 1/n of each bound plus one 4,096-set job's worth.
 * lsg_submit_jobs stages a package with the context lock released (several host threads may
 * stage packages at once; the devices of a multi-device context are staged in parallel). */
int lsg_reserve(lsg_ctx* ctx, size_t max_sets, size_t max_pks, size_t max_msg_bytes, int32_t n_slots);
/* Device + pinned allocations made by this process so far (steady-state checks). */
int lsg_allocation_count(lsg_ctx* ctx, uint64_t* n);

/* worker.ts:30-106 for one work package (BlsWorkReq[] -> BlsWorkResult), asynchronous:
 * submit copies the jobs into pinned staging memory, draws the RLC randomizers, launches every
 * stage and returns a ticket (LSG_ERR_BUSY when all slots are outstanding: back-pressure as in
 * canAcceptWork, multithread/index.ts:143-149).  All batchable sets of the package form ONE
 * RLC group (one final exponentiation); only if it fails are the reference's 16-job chunks
 * and then the jobs of failing chunks checked (on the resident per-set values), so verdicts
 * and the batch_retries / batch_sigs_success counters are those of worker.ts.  wait blocks on
 * the ticket and applies those rules.  seed != 0 makes the randomizers deterministic (tests);
 * seed == 0 draws them from getrandom (LSG_ERR_ENTROPY if that fails).
 * A key that does not deserialize anywhere in the package (any device of the context) rejects
 * every job with the code of the first bad key in caller job order (worker.ts:41-43).
 * On a multi-device context the 16-job chunks are formed per device, so batch_retries /
 * batch_sigs_success can differ from a single device's; per-job verdicts never do.
 * A wait that fails before resolving (a device error while blocking) leaves the ticket
 * outstanding: it may be waited on again. */
int lsg_submit_jobs(lsg_ctx* ctx, const lsg_job* jobs, size_t n_jobs, uint64_t seed, lsg_ticket* ticket);
int lsg_wait_jobs(lsg_ctx* ctx, lsg_ticket ticket, lsg_job_result* results /* [n_jobs] */, lsg_stats* stats);
/* One process per GPU (SURVEY.md 8e over torch.distributed / any host collective), on a
 * single-device context: lsg_jobs_partial blocks until the package group's Miller product is
 * ready and writes it (576 bytes, canonical; the identity when the package has no batchable
 * set; *has_batch says which).  The caller all-gathers the partials, checks their product with
 * lsg_final_*, and resolves the ticket with that node verdict (1 passed, 0 failed: this GPU's
 * own package check then localises).  lsg_wait_jobs == lsg_wait_jobs_node(..., -1, ...).
 * The node verdict is advisory: this GPU's own check of its share is computed in any case and
 * decides, so a caller whose exchange went wrong (node_valid 1 but this share invalid) gets
 * the localised per-job verdicts, never a wrongly accepted package. */
int lsg_jobs_partial(lsg_ctx* ctx, lsg_ticket ticket, uint8_t* out576, int32_t* has_batch);
/* The same partial copied device-to-device into dev_out576 (576 bytes of device memory on the
 * context's device, e.g. the send buffer of an RCCL all-gather): the exchange never leaves the
 * GPU.  Returns once the copy is done. */
int lsg_jobs_partial_device(lsg_ctx* ctx, lsg_ticket ticket, void* dev_out576, int32_t* has_batch);
int lsg_wait_jobs_node(lsg_ctx* ctx, lsg_ticket ticket, int32_t node_valid, lsg_job_result* results,
                       lsg_stats* stats);
/* Coalescing of small packages (single-device contexts; off by default).  From this call on,
 * a package of at most max_sets sets submitted with lsg_submit_jobs is copied (the caller's
 * buffers are free on return) and, while max_inflight launches are on the device, held back;
 * the held packages go out together as ONE launch when the device has room (a wait frees a
 * slot) or when one of them is waited on.  Every package keeps the reference's semantics on
 * its own (multithread/index.ts:335 one package per worker; worker.ts:30-106): its
 * batchable jobs in 16-job chunks each checked as one RLC batch, per-job retry, the
 * deserializeSet rule over its jobs, its own counters (n_final_exps counts the whole launch).
 * Such tickets have no node protocol: lsg_jobs_partial* and lsg_wait_jobs_node with
 * node_valid != -1 reject them.  This fills the GPU with many small packages (gossip-sized)
 * without one launch -- and one chain of dependent kernels -- per package.  max_sets = 0 turns
 * coalescing off (held packages are launched first). */
int lsg_set_coalesce(lsg_ctx* ctx, uint32_t max_sets, int32_t max_inflight);
/* Whole-job assignment of lsg_init_devices (host only, no device needed): owner[j] = device of
 * job j = floor(sets before j * n_devices / total sets). */
int lsg_assign_jobs(const uint32_t* job_sets, size_t n_jobs, int32_t n_devices, int32_t* owner);
/* Number of pipeline slots (packages that may be outstanding at once): the back-pressure
 * bound of canAcceptWork (multithread/index.ts:143-149 workersBusy < poolSize). */
int lsg_pipeline_slots(lsg_ctx* ctx, int32_t* n);
/* *done = 1 once the ticket's device work has finished (any ticket kind). */
int lsg_poll(lsg_ctx* ctx, lsg_ticket ticket, int32_t* done);
/* submit + wait */
int lsg_verify_jobs(lsg_ctx* ctx, const lsg_job* jobs, size_t n_jobs, uint64_t seed, lsg_job_result* results,
                    lsg_stats* stats);

/* maybeBatch.ts:16-39 over one list of sets (no retry): *result = one lsg_job_result. */
int lsg_verify_sets(lsg_ctx* ctx, const lsg_set* sets, size_t n_sets, uint64_t seed, lsg_job_result* result);

/* PublicKey.aggregate(pks).toBytes(uncompressed): out96 receives the 96-byte affine sum.
 * *err_code = BLST_* for a bad input key, LSG_ERR_EMPTY_AGGREGATE for n == 0.  With
 * pk_len == LSG_PK_INDEX, pks holds n uint32 indices into the pubkey table. */
int lsg_aggregate_pubkeys(lsg_ctx* ctx, const uint8_t* pks, uint32_t pk_len, size_t n, uint8_t* out96,
                          int32_t* err_code);
/* PublicKey.aggregate for n_sets sets in one device pass (utils.ts:11 getAggregatedPubkey over
 * a block's aggregate sets, indexedAttestation.ts:21-47): set i's keys are sets[i].pks /
 * pk_len / n_pks (bytes or table indices; msg and sig are ignored).  out96[96 i..] = set i's
 * uncompressed sum; err[i] = its first bad key's BLST_* / LSG_ERR_BAD_INDEX, or
 * LSG_ERR_EMPTY_AGGREGATE for no keys.  Every input size runs the jobs path's fused gather +
 * mixed-addition fold (k_pk_agg_seg); the batch-affine aggregation tree exists only in the
 * A/B build (liblodestar_bls_ab.so, LSG_AGG_TREE=1), where it was measured slower. */
int lsg_aggregate_pubkeys_multi(lsg_ctx* ctx, const lsg_set* sets, size_t n_sets, uint8_t* out96, int32_t* err);

/* hash_to_G2(msg_i, DST) for n messages of msg_len bytes each -> n x 192-byte uncompressed points. */
int lsg_hash_to_g2(lsg_ctx* ctx, const uint8_t* msgs, uint32_t msg_len, size_t n, const uint8_t* dst,
                   uint32_t dst_len, uint8_t* out192);

/* Signature.fromBytes(sig, affine, validate=true) for n signatures of sig_len bytes:
 * out192[i] = uncompressed affine point, err[i] = BLST_* (0 = ok). */
int lsg_sig_decode(lsg_ctx* ctx, const uint8_t* sigs, uint32_t sig_len, size_t n, uint8_t* out192, int32_t* err);

/* One shard's sets -> its un-exponentiated Miller product (576 bytes: 12 canonical big-endian
 * Fp in tower order) over the sets that decode, and per-set error codes (synchronous;
 * single-device contexts).  *any_error != 0 means the shard cannot be batched as a whole. */
int lsg_batch_partial(lsg_ctx* ctx, const lsg_set* sets, size_t n_sets, uint64_t seed, uint8_t* out576,
                      int32_t* set_err, int32_t* any_error);
/* prod(partials) -> final exponentiation on the GPU -> *valid = (result == 1).  The
 * submit/wait pair runs on device 0's final-exponentiation entries, overlapping packages. */
int lsg_final_verify(lsg_ctx* ctx, const uint8_t* partials576, size_t n_partials, int32_t* valid);
int lsg_final_submit(lsg_ctx* ctx, const uint8_t* partials576, size_t n_partials, lsg_ticket* ticket);
/* lsg_final_submit over partials in device memory of device 0 (an all-gather's output); the
 * caller's writes to them must be complete (e.g. its stream synchronised). */
int lsg_final_submit_device(lsg_ctx* ctx, const void* dev_partials576, size_t n_partials, lsg_ticket* ticket);
int lsg_final_wait(lsg_ctx* ctx, lsg_ticket ticket, int32_t* valid);
/* Several RLC batches' final checks in one ticket (one launch per stage instead of one
 * ticket per batch): n_groups groups of per_group partials each, group g being partials
 * g*per_group .. g*per_group+per_group-1 (e.g. one per rank); lsg_final_wait_groups writes
 * n_groups verdicts.  lsg_final_submit(p, n) is lsg_final_submit_groups(p, 1, n). */
int lsg_final_submit_groups(lsg_ctx* ctx, const uint8_t* partials576, size_t n_groups, size_t per_group,
                            lsg_ticket* ticket);
int lsg_final_wait_groups(lsg_ctx* ctx, lsg_ticket ticket, int32_t* valid /* [n_groups] */);

/* ---- Validator pubkey table resident in HBM.  Replaces the per-call
 * PublicKey -> bytes hand-off of the pool (multithread/index.ts:177, utils.ts:11) with the
 * node's index2pubkey cache held on the GPU (state-transition/src/cache/pubkeyCache.ts:60-75
 * syncPubkeys, cache/epochContext.ts:701-704 addPubkey): keys are decoded once, as
 * PublicKey.fromBytes(pk, jacobian) does there (on-curve check, no subgroup check: cached
 * keys were validated at deposit time), and sets then name their keys by index
 * (lsg_set.pk_len = LSG_PK_INDEX); aggregation gathers them on the device.
 *   lsg_pubkey_table_set  keys first_index .. first_index+n-1 <- pks (48 or 96 bytes each);
 *                         the table grows as needed (growth waits for in-flight work).
 *                         err[k] (may be NULL) = BLST_* of key k; a key that does not decode
 *                         leaves its index unset, and a set naming an unset index fails
 *                         its package with LSG_ERR_BAD_INDEX (as deserializeSet throws).
 *   lsg_pubkey_table_size number of indices (highest set index + 1). */
int lsg_pubkey_table_set(lsg_ctx* ctx, size_t first_index, const uint8_t* pks, uint32_t pk_len, size_t n,
                         int32_t* err);
int lsg_pubkey_table_size(lsg_ctx* ctx, size_t* n);

/* Batched KeyValidate: PublicKey.fromBytes(pk, affine, validate=true) of
 * processDeposit.ts:57-65 for n keys of pk_len (48/96) bytes -- decode, not the point at
 * infinity (BLST_PK_IS_INFINITY), in the r-torsion subgroup (BLST_POINT_NOT_IN_GROUP).
 * err[i] = BLST_* (0 = valid); out96 (may be NULL) = the uncompressed affine key. */
int lsg_pubkey_validate(lsg_ctx* ctx, const uint8_t* pks, uint32_t pk_len, size_t n, uint8_t* out96, int32_t* err);

/* G2 signature aggregation for the op pools:
 *   bls.Signature.aggregate(sigs.map(signatureFromBytesNoCheck)).toBytes()
 * of opPools/attestationPool.ts:195, syncCommitteeMessagePool.ts:139,
 * aggregatedAttestationPool.ts:322 and syncContributionAndProofPool.ts:185, with the decode of
 * opPools/utils.ts:32-34 (Signature.fromBytes(sig, affine, validate=false): size, encoding and
 * on-curve checks, no subgroup check).  n_groups independent aggregations in one call: group g
 * is signatures offsets[g] .. offsets[g+1]-1 (offsets has n_groups+1 entries, offsets[0] = 0),
 * each sig_len (96 or 192) bytes.  out96[g] = the compressed sum (zeros unless err[g] == 0);
 * err[g] = BLST_* of the group's first signature that does not decode, or
 * LSG_ERR_EMPTY_AGGREGATE for an empty group ("EMPTY_AGGREGATE_ARRAY"). */
int lsg_aggregate_signatures(lsg_ctx* ctx, const uint8_t* sigs, uint32_t sig_len, const uint32_t* offsets,
                             size_t n_groups, uint8_t* out96, int32_t* err);

/* Signing roots on the GPU: computeSigningRoot(type, obj, domain) of
 * state-transition/src/util/signingRoot.ts:7-13 = hash_tree_root(SigningData{objectRoot, domain}).
 *   lsg_signing_roots              objectRoot given: roots32 = n x 32 bytes;
 *   lsg_attestation_signing_roots  getAttestationDataSigningRoot (signatureSets/indexedAttestation.ts:11-19):
 *                                  data128 = n SSZ-serialized phase0.AttestationData (128 bytes each:
 *                                  slot, index, beaconBlockRoot, source{epoch, root}, target{epoch, root}).
 * domain_stride 0: one 32-byte domain for every object; 32: one per object.  out32 = n x 32 bytes,
 * the 32-byte messages lsg_set.msg carries. */
int lsg_signing_roots(lsg_ctx* ctx, const uint8_t* roots32, size_t n, const uint8_t* domain32, uint32_t domain_stride,
                      uint8_t* out32);
int lsg_attestation_signing_roots(lsg_ctx* ctx, const uint8_t* data128, size_t n, const uint8_t* domain32,
                                  uint32_t domain_stride, uint8_t* out32);

/* Test/bench input generation (not on the verify path): sig_i = sk_i * H(m_i) compressed,
 * pk_i = sk_i * G1 uncompressed; sks are 32-byte big-endian secret keys. */
int lsg_sign(lsg_ctx* ctx, const uint8_t* sks32, const uint8_t* msgs, uint32_t msg_len, size_t n, uint8_t* out96);
int lsg_sk_to_pk(lsg_ctx* ctx, const uint8_t* sks32, size_t n, uint8_t* out96);

/* Parity hook of the device Fp2 product (tests only): for n items of four field elements
 * (a0, a1, b0, b1) in the pair layout -- 14 signed radix-2^29 limbs each, word k of element e
 * of item i at in[(4 i + e) * 14 + 2 (k mod 7) + k / 7] -- writes c0, c1 with
 * c0 + c1 u = (a0 + a1 u)(b0 + b1 u) / 2^406 mod p, raw (lazy, not canonical), same layout, 2
 * elements per item.  Not on the verification path. */
int lsg_check_fp2_mul(lsg_ctx* ctx, const uint32_t* in, size_t n, uint32_t* out);
/* Integer-VALU roofline probe: runs a throughput kernel of dependent-free 381-bit
 * Montgomery multiplications; reports Fp-mul/s and v_mad_u64_u32/s (x300 per mul). */
int lsg_probe_fp_mul_rate(lsg_ctx* ctx, double* fp_mul_per_s, double* mad_per_s);

/* Integer-VALU peak probe: issue rate of v_mad_u64_u32 (16 independent accumulators per lane,
 * 8 waves per SIMD) -- the roofline denominator bench.py reports. */
int lsg_probe_mad_peak(lsg_ctx* ctx, double* mad_per_s);

/* Per-kernel timing of the most recently completed ticket (or synchronous call), from HIP
 * events on the streams the kernels ran on: names[i] / ms[i] for up to max entries;
 * returns the count. */
int lsg_last_kernel_times(lsg_ctx* ctx, const char** names, double* ms, int max);

#ifdef __cplusplus
}
#endif
#endif /* LODESTAR_BLS_H */
