"use strict";
/**
 * BlsGpuVerifier -- IBlsVerifier on one MI355X (gfx950), a drop-in for Lodestar's
 * BlsMultiThreadWorkerPool (/root/reference/packages/beacon-node/src/chain/bls/multithread/
 * index.ts) and BlsSingleThreadVerifier (chain/bls/singleThread.ts:14-35).
 *
 * What is kept from the reference, name for name (the file:line is the reference code each
 * method restates):
 *   verifySignatureSets   index.ts:151-191  verifyOnMainThread shortcut, chunks of <= 128
 *                         sets, AND over the chunks, empty chunk list -> throw
 *   canAcceptWork         index.ts:143-149  back-pressure: packages in flight < pipeline
 *                         slots (the reference's workersBusy < poolSize) and jobs < 512
 *   close                 index.ts:193-217  pending jobs reject with QueueError
 *                         QUEUE_ERROR_QUEUE_ABORTED
 *   _queueBlsWork         index.ts:255-302  batchable jobs buffered until > 32 sigs or
 *                         100 ms; others queued and run on the next macrotask
 *   _runJob/_prepareWork  index.ts:307-420  one package of <= 128 sigs per free slot;
 *                         per-job resolve/reject; metrics
 *   _runBufferedJobs      index.ts:425-431
 *   chunkifyMaximizeChunkSize  multithread/utils.ts:4-19
 * What replaces the worker threads and @chainsafe/blst: the N-API addon
 * (lodestar_amd/napi/lsg_napi.c) over the C ABI (include/lodestar_bls.h).  A package is
 * submitted with addon.submitJobs (inputs copied to pinned memory before it returns) and
 * awaited with addon.waitJobs (blocking part on a libuv pool thread).  The GPU applies the
 * worker's batch + per-job retry rules (worker.ts:30-106) itself, so one package costs one
 * round trip.  Aggregate sets send all their pubkeys; the GPU sums them (utils.ts:11).
 *
 * Node-wide: chain.ts:195-198 builds ONE verifier per node, its pool spanning every core
 * (multithread/poolSize.ts:7).  options.devices = [0, 1, ...] opens one context over all the
 * node's GPUs (lsg_init_devices): a package is split into whole jobs per GPU, the GPUs'
 * partials are all-gathered over RCCL and checked by one final exponentiation (SURVEY 8e).
 *
 * BlsGpuSingleThreadVerifier restates BlsSingleThreadVerifier (singleThread.ts:14-35): one
 * synchronous maybeBatch call per verifySignatureSets, no queue, no retry, opts ignored.
 * createBlsVerifier picks between the two as chain.ts:196-198 does (blsVerifyAllMainThread).
 *
 * Metrics: the reference's names and observation points (metrics/metrics/lodestar.ts:350-430,
 * multithread/index.ts:319-381): jobWaitTime, totalJobsGroupsStarted, totalJobsStarted,
 * totalSigSetsStarted, timePerSigSet, jobsWorkerTime{workerId}, latencyToWorker,
 * latencyFromWorker, successJobsSignatureSetsCount, errorJobsSignatureSetsCount,
 * batchRetries, batchSigsSuccess, mainThreadDurationInThreadPool, bls.aggregatedPubkeys.
 * "Worker" times are the GPU package's start/end (lsg_stats, CLOCK_MONOTONIC = the clock of
 * process.hrtime.bigint()); workerId is the pipeline slot that ran the package.
 *
 * Extensions required by the north star (SURVEY.md 8b, not in the reference snapshot):
 *   opts.priority                  queue at the head instead of the tail
 *   verifySignatureSetsSameMessage per-set verdicts for sets sharing one message
 */

const MAX_SIGNATURE_SETS_PER_JOB = 128;
const MAX_BUFFERED_SIGS = 32;
const MAX_BUFFER_WAIT_MS = 100;
const MAX_JOBS_CAN_ACCEPT_WORK = 512;

const JOB_BATCHABLE = 1;
const JOB_PRIORITY = 2;

const LSG_INVALID = 0;
const LSG_VALID = 1;
const LSG_ERROR = 2;

/** blst error names (blst.h BLST_ERROR) + @chainsafe/blst's size error */
const BLST_NAMES = {
  0: "BLST_SUCCESS",
  1: "BLST_BAD_ENCODING",
  2: "BLST_POINT_NOT_ON_CURVE",
  3: "BLST_POINT_NOT_IN_GROUP",
  4: "BLST_AGGR_TYPE_MISMATCH",
  5: "BLST_VERIFY_FAIL",
  6: "BLST_PK_IS_INFINITY",
  7: "BLST_BAD_SCALAR",
  10: "BLST_INVALID_SIZE",
};

/** Error text for a job error code, in the form the reference's callers match on: the BLST
 * code name is a substring (multithread.test.ts:97 "BLST_INVALID_SIZE"). */
function errorMessage(code) {
  if (code === 100) return "Empty signature set"; // maybeBatch.ts:29-31
  if (code === 101) return "EMPTY_AGGREGATE_ARRAY"; // PublicKey.aggregate([])
  return "BLST_ERROR: " + (BLST_NAMES[code] || "BLST_UNKNOWN_" + code);
}

/** util/queue/errors.ts:3-16 */
const QueueErrorCode = {
  QUEUE_ABORTED: "QUEUE_ERROR_QUEUE_ABORTED",
  QUEUE_MAX_LENGTH: "QUEUE_ERROR_QUEUE_MAX_LENGTH",
};

class QueueError extends Error {
  constructor(type) {
    super(type.code);
    this.type = type;
    this.code = type.code;
  }
}

/** state-transition/src/util/signatureSets.ts:5-8 */
const SignatureSetType = {single: "single", aggregate: "aggregate"};

/**
 * Splits an array into an array of arrays maximizing the size of the smallest chunk
 * (multithread/utils.ts:4-19).
 */
function chunkifyMaximizeChunkSize(arr, minPerChunk) {
  const chunkCount = Math.floor(arr.length / minPerChunk);
  if (chunkCount <= 1) {
    return [arr];
  }
  const perChunk = Math.ceil(arr.length / chunkCount);
  const arrArr = [];
  for (let i = 0; i < arr.length; i += perChunk) {
    arrArr.push(arr.slice(i, i + perChunk));
  }
  return arrArr;
}

/** PublicKey -> bytes.  Accepts raw Uint8Arrays (96 B uncompressed / 48 B compressed) or
 * @chainsafe/bls PublicKey objects (toBytes(format)). */
function pubkeyBytes(pk) {
  if (pk instanceof Uint8Array) return pk;
  if (pk && typeof pk.toBytes === "function") return pk.toBytes("uncompressed");
  throw Error("Unknown public key type");
}

/** ISignatureSet -> the addon's set (utils.ts:5-17 getAggregatedPubkey, with the sum done on
 * the GPU instead of the main thread). */
function serializeSet(set) {
  // signers named by validator index into the device pubkey table (SURVEY 8f(1)):
  // loadPubkeys() mirrors index2pubkey; the set carries its attesting indices
  if (set.pubkeyIndices !== undefined) {
    const ix = set.pubkeyIndices instanceof Uint32Array ? set.pubkeyIndices : Uint32Array.from(set.pubkeyIndices);
    return {pubkeyIndices: ix, message: set.signingRoot, signature: set.signature};
  }
  let pubkeys;
  switch (set.type) {
    case SignatureSetType.single:
      pubkeys = [pubkeyBytes(set.pubkey)];
      break;
    case SignatureSetType.aggregate:
      pubkeys = set.pubkeys.map(pubkeyBytes);
      break;
    default:
      throw Error("Unknown signature set type");
  }
  return {pubkeys, message: set.signingRoot, signature: set.signature};
}

/** utils.ts:19-26 */
function getAggregatedPubkeysCount(sets) {
  let n = 0;
  for (const set of sets) {
    if (set.pubkeyIndices !== undefined) n += set.pubkeyIndices.length;
    else if (set.type === SignatureSetType.aggregate) n += set.pubkeys.length;
  }
  return n;
}

function loadAddon() {
  // eslint-disable-next-line global-require
  return require("../napi/lsg_napi.node");
}

class BlsGpuVerifier {
  /**
   * @param {{blsVerifyAllMultiThread?: boolean, device?: number, devices?: number[], seed?: number,
   *          maxSigsPerPackage?: number, reserveSets?: number, reservePubkeys?: number}} options
   * @param {{logger?: object, metrics?: object|null, addon?: object}} modules  addon is
   *        injectable (tests drive the queue logic with a mock of the addon's surface)
   */
  constructor(options = {}, modules = {}) {
    this.logger = modules.logger || null;
    this.metrics = modules.metrics || null;
    this.blsVerifyAllMultiThread = options.blsVerifyAllMultiThread === true;
    this.seed = options.seed || 0; // 0: randomizers from the OS CSPRNG (production)
    // sigs of queued jobs drained into one GPU package (prepareWork, index.ts:400-418).  The
    // reference's 128 suits a CPU worker; one GPU launch wants thousands of sets, so a
    // production node sets e.g. 4096.  Per-job verdicts do not depend on it.
    this.maxSigsPerPackage = options.maxSigsPerPackage || MAX_SIGNATURE_SETS_PER_JOB;
    this.addon = modules.addon || loadAddon();
    // throws loudly without a gfx950 device
    this.ctx = this.addon.open(Array.isArray(options.devices) ? options.devices : options.device || 0);
    this.poolSize = this.addon.slots(this.ctx);
    if (options.reserveSets && this.addon.reserve) {
      // preallocate every pipeline slot for packages of up to reserveSets sets (lsg_reserve)
      const pks = options.reservePubkeys || options.reserveSets;
      this.addon.reserve(this.ctx, options.reserveSets, pks, 32 * options.reserveSets, 0);
    }
    this.jobs = [];
    this.bufferedJobs = null;
    this.closed = false;
    this.workersBusy = 0; // packages in flight (the reference's busy workers)
    this.inflight = new Set();
    this._runJob = this._runJob.bind(this);
    this._runBufferedJobs = this._runBufferedJobs.bind(this);
  }

  /** Mirror index2pubkey[firstIndex ..] into the device pubkey table (SURVEY 8f(1); call next
   * to pubkeyCache.ts syncPubkeys / epochContext.ts addPubkey).  Sets may then carry
   * `pubkeyIndices` instead of PublicKeys.  Returns per-key BLST codes (0 = loaded). */
  loadPubkeys(firstIndex, pubkeys) {
    return this.addon.pubkeyTableSet(this.ctx, firstIndex, pubkeys.map(pubkeyBytes));
  }

  /** Op-pool aggregation (SURVEY 8f(4)): bls.Signature.aggregate(sigs.map(signatureFromBytesNoCheck))
   * .toBytes() of opPools/attestationPool.ts:195, syncCommitteeMessagePool.ts:139,
   * aggregatedAttestationPool.ts:322 and syncContributionAndProofPool.ts:185, for many groups in
   * one device pass.  Returns [{signature: Uint8Array(96) | null, err}] per group; err is the
   * BLST code of the group's first undecodable signature (101 = EMPTY_AGGREGATE_ARRAY). */
  aggregateSignatures(groups) {
    return this.addon.aggregateSignatures(this.ctx, groups);
  }

  canAcceptWork() {
    return this.workersBusy < this.poolSize && this.jobs.length < MAX_JOBS_CAN_ACCEPT_WORK;
  }

  async verifySignatureSets(sets, opts = {}) {
    if (this.metrics && this.metrics.bls) this.metrics.bls.aggregatedPubkeys.inc(getAggregatedPubkeysCount(sets));

    if (opts.verifyOnMainThread && !this.blsVerifyAllMultiThread) {
      // verifySignatureSetsMaybeBatch on the calling thread: no retry, errors propagate
      const m = this.metrics && this.metrics.blsThreadPool;
      const timer = m ? m.mainThreadDurationInThreadPool.startTimer() : null;
      try {
        const r = this.addon.verifySets(this.ctx, sets.map(serializeSet), this.seed);
        if (r.status === LSG_ERROR) throw Error(errorMessage(r.errCode));
        return r.status === LSG_VALID;
      } finally {
        if (timer) timer();
      }
    }

    const results = await Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map((setsWorker) =>
        this._queueBlsWork({opts, sets: setsWorker.map(serializeSet)})
      )
    );
    // .every on an empty array returns true
    if (results.length === 0) {
      throw Error("Empty results array");
    }
    return results.every((isValid) => isValid === true);
  }

  /**
   * Per-set verdicts for sets that share one message (north-star extension).  The sets go
   * out as one package of single-set batchable jobs: the GPU verifies them as one RLC batch
   * and, if that fails, re-verifies each set on its own (worker.ts:74-96).  A set whose
   * signature does not decode is reported false.
   */
  async verifySignatureSetsSameMessage(sets, message, opts = {}) {
    const jobs = sets.map((s) => ({
      opts: {batchable: true, priority: opts.priority},
      sets: [{pubkeys: [pubkeyBytes(s.publicKey)], message, signature: s.signature}],
    }));
    const verdicts = await Promise.all(
      jobs.map((workReq) => this._queueBlsWork(workReq).catch(() => false))
    );
    return verdicts;
  }

  async close() {
    if (this.bufferedJobs) {
      clearTimeout(this.bufferedJobs.timeout);
      for (const job of this.bufferedJobs.jobs) job.reject(new QueueError({code: QueueErrorCode.QUEUE_ABORTED}));
      this.bufferedJobs = null;
    }
    for (const job of this.jobs) {
      job.reject(new QueueError({code: QueueErrorCode.QUEUE_ABORTED}));
    }
    this.jobs.splice(0, this.jobs.length);
    this.closed = true;
    // let packages already on the GPU finish, then release the device context
    await Promise.all(Array.from(this.inflight).map((p) => p.catch(() => undefined)));
    if (this.ctx) {
      this.addon.close(this.ctx);
      this.ctx = null;
    }
  }

  _queueBlsWork(workReq) {
    if (this.closed) {
      return Promise.reject(new QueueError({code: QueueErrorCode.QUEUE_ABORTED}));
    }
    return new Promise((resolve, reject) => {
      const job = {resolve, reject, addedTimeMs: Date.now(), workReq};
      if (workReq.opts.batchable) {
        if (!this.bufferedJobs) {
          this.bufferedJobs = {
            jobs: [],
            sigCount: 0,
            firstPush: Date.now(),
            timeout: setTimeout(this._runBufferedJobs, MAX_BUFFER_WAIT_MS),
          };
        }
        if (workReq.opts.priority) this.bufferedJobs.jobs.unshift(job);
        else this.bufferedJobs.jobs.push(job);
        this.bufferedJobs.sigCount += job.workReq.sets.length;
        if (this.bufferedJobs.sigCount > MAX_BUFFERED_SIGS) {
          clearTimeout(this.bufferedJobs.timeout);
          this._runBufferedJobs();
        }
      } else {
        if (workReq.opts.priority) this.jobs.unshift(job);
        else this.jobs.push(job);
        setTimeout(this._runJob, 0);
      }
    });
  }

  async _runJob() {
    if (this.closed) return;
    if (this.workersBusy >= this.poolSize) return;
    const jobs = this._prepareWork();
    if (jobs.length === 0) return;

    const m = this.metrics && this.metrics.blsThreadPool;
    let startedSigSets = 0;
    for (const job of jobs) {
      if (m) m.jobWaitTime.observe((Date.now() - job.addedTimeMs) / 1000);
      startedSigSets += job.workReq.sets.length;
    }
    if (m) {
      m.totalJobsGroupsStarted.inc(1);
      m.totalJobsStarted.inc(jobs.length);
      m.totalSigSetsStarted.inc(startedSigSets);
    }

    this.workersBusy++;
    const run = (async () => {
      try {
        const pkg = jobs.map((job) => ({
          sets: job.workReq.sets,
          flags: (job.workReq.opts.batchable ? JOB_BATCHABLE : 0) | (job.workReq.opts.priority ? JOB_PRIORITY : 0),
        }));
        const jobStartNs = process.hrtime.bigint();
        const ticket = this.addon.submitJobs(this.ctx, pkg, this.seed);
        if (ticket === null) throw Error("BlsGpuVerifier: every pipeline slot is busy");
        const workResult = await this.addon.waitJobs(this.ctx, ticket);
        const jobEndNs = process.hrtime.bigint();
        let successCount = 0;
        let errorCount = 0;
        for (let i = 0; i < jobs.length; i++) {
          const job = jobs[i];
          const r = workResult.results[i];
          const n = job.workReq.sets.length;
          if (!r) {
            job.reject(Error(`No jobResult for index ${i}`));
            errorCount += n;
          } else if (r.status === LSG_ERROR) {
            job.reject(Error(errorMessage(r.errCode)));
            errorCount += n;
          } else {
            job.resolve(r.status === LSG_VALID);
            successCount += n;
          }
        }
        if (m) {
          // index.ts:362-381, with the GPU package in the worker's place
          const workerJobTimeSec = (workResult.endNs - workResult.startNs) / 1e9;
          const latencyToWorkerSec = (workResult.startNs - Number(jobStartNs)) / 1e9;
          const latencyFromWorkerSec = (Number(jobEndNs) - workResult.endNs) / 1e9;
          m.timePerSigSet.observe(workerJobTimeSec / startedSigSets);
          m.jobsWorkerTime.inc({workerId: workResult.workerId || 0}, workerJobTimeSec);
          m.latencyToWorker.observe(latencyToWorkerSec);
          m.latencyFromWorker.observe(latencyFromWorkerSec);
          m.successJobsSignatureSetsCount.inc(successCount);
          m.errorJobsSignatureSetsCount.inc(errorCount);
          m.batchRetries.inc(workResult.batchRetries);
          m.batchSigsSuccess.inc(workResult.batchSigsSuccess);
        }
      } catch (e) {
        if (!this.closed && this.logger) this.logger.error("BlsGpuVerifier error", {}, e);
        for (const job of jobs) job.reject(e);
      }
    })();
    this.inflight.add(run);
    await run;
    this.inflight.delete(run);
    this.workersBusy--;
    setTimeout(this._runJob, 0);
  }

  _prepareWork() {
    const jobs = [];
    let totalSigs = 0;
    while (totalSigs < this.maxSigsPerPackage) {
      const job = this.jobs.shift();
      if (!job) break;
      jobs.push(job);
      totalSigs += job.workReq.sets.length;
    }
    return jobs;
  }

  _runBufferedJobs() {
    if (this.bufferedJobs) {
      this.jobs.push(...this.bufferedJobs.jobs);
      this.bufferedJobs = null;
      setTimeout(this._runJob, 0);
    }
  }
}

/**
 * BlsSingleThreadVerifier (chain/bls/singleThread.ts:14-35) on the GPU: each call is one
 * verifySignatureSetsMaybeBatch (lsg_verify_sets) made synchronously from the calling thread,
 * with no queue and no retry; opts are ignored, errors propagate as throws.  The duration is
 * observed after the call as the reference does (it observes the total and the per-set time;
 * its startNs - endNs has the sign inverted, here the duration is positive).
 */
class BlsGpuSingleThreadVerifier {
  /**
   * @param {{device?: number, devices?: number[], seed?: number}} options
   * @param {{metrics?: object|null, addon?: object}} modules
   */
  constructor(options = {}, modules = {}) {
    this.metrics = modules.metrics || null;
    this.seed = options.seed || 0;
    this.addon = modules.addon || loadAddon();
    this.ctx = this.addon.open(Array.isArray(options.devices) ? options.devices : options.device || 0);
  }

  async verifySignatureSets(sets) {
    if (this.metrics && this.metrics.bls) this.metrics.bls.aggregatedPubkeys.inc(getAggregatedPubkeysCount(sets));
    const setsAggregated = sets.map(serializeSet);
    // Count time after aggregating
    const startNs = process.hrtime.bigint();
    const r = this.addon.verifySets(this.ctx, setsAggregated, this.seed);
    if (r.status === LSG_ERROR) throw Error(errorMessage(r.errCode));
    // Don't use a try/catch, only count run without exceptions
    const endNs = process.hrtime.bigint();
    const totalSec = Number(endNs - startNs) / 1e9;
    const m = this.metrics && this.metrics.blsThreadPool;
    if (m) {
      m.mainThreadDurationInThreadPool.observe(totalSec);
      m.mainThreadDurationInThreadPool.observe(totalSec / sets.length);
    }
    return r.status === LSG_VALID;
  }

  async close() {
    if (this.ctx) {
      this.addon.close(this.ctx);
      this.ctx = null;
    }
  }

  canAcceptWork() {
    // Since sigs are verified blocking the main thread, there's no mechanism to throttle
    return true;
  }
}

/** chain.ts:195-198: opts.blsVerifyAllMainThread selects the single-thread verifier. */
function createBlsVerifier(opts = {}, modules = {}) {
  return opts.blsVerifyAllMainThread ? new BlsGpuSingleThreadVerifier(opts, modules) : new BlsGpuVerifier(opts, modules);
}

module.exports = {
  BlsGpuVerifier,
  BlsGpuSingleThreadVerifier,
  createBlsVerifier,
  QueueError,
  QueueErrorCode,
  SignatureSetType,
  chunkifyMaximizeChunkSize,
  errorMessage,
  MAX_SIGNATURE_SETS_PER_JOB,
  MAX_BUFFERED_SIGS,
  MAX_BUFFER_WAIT_MS,
  MAX_JOBS_CAN_ACCEPT_WORK,
};
