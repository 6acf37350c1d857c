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
 *   canAcceptWork         index.ts:143-149  back-pressure, on sets for a GPU: queued +
 *                         buffered + in-flight sets < maxPendingSigs
 *   close                 index.ts:193-217  pending jobs reject with QueueError
 *                         QUEUE_ERROR_QUEUE_ABORTED
 *   _queueBlsWork         index.ts:255-302  batchable jobs buffered until > 32 sigs or
 *                         100 ms; others queued and run on the next macrotask
 *   _runJob/_prepareWork  index.ts:307-420  packages sized for the GPU (class comment);
 *                         per-job resolve/reject; metrics
 *   _runBufferedJobs      index.ts:425-431
 *   chunkifyMaximizeChunkSize  multithread/utils.ts:4-19
 * What replaces the worker threads and @chainsafe/blst: the N-API addon
 * (lodestar_amd/napi/lsg_napi.c) over the C ABI (include/lodestar_bls.h).  A package is
 * packed into one byte arena (packJobs) and handed to addon.verifyPacked, whose native
 * package thread submits and waits (neither the JS thread nor libuv's pool blocks); the
 * promise settles with per-job verdict arrays.  The GPU applies the worker's batch + per-job
 * retry rules (worker.ts:30-106) itself, so one package costs one round trip.  Aggregate sets
 * send all their pubkeys; the GPU sums them (utils.ts:11).
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
 * multithread/index.ts:135-140,319-381): queueLength, workersBusy (collected at scrape time),
 * jobWaitTime, totalJobsGroupsStarted, totalJobsStarted,
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

/**
 * verifySignatureSetsMaybeBatch(sets) (maybeBatch.ts:16-39) as ONE non-batchable job sent
 * straight to the addon, outside the queue and ahead of it: verifyPacked's priority flag runs it
 * on the addon's priority thread (never behind the package threads' queue) and on the
 * library's high-priority streams.  The reference runs this path synchronously on the main
 * thread (multithread/index.ts:155-168, ~0.9 ms of blst); here the caller's promise settles
 * with the verdict and the JS thread keeps running meanwhile.  No retry: one job is one
 * maybeBatch call; an error rejects with its BLST code (e.g. BLST_INVALID_SIZE).
 */
async function verifyDirect(addon, ctx, sets, seed) {
  const block = new VerdictBlock(false, false);
  block.add(sets, true);
  block.seal();
  const pkg = packBlocks([block], sets.length, undefined);
  if (pkg.jobBlock.length === 1) {
    const r = await addon.verifyPacked(ctx, pkg.arena, pkg.setDesc, pkg.jobDesc, seed, true);
    block.settle(0, r.status[0], r.errCode[0]);
  }
  return block.verdict(0);
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
  return require("../../lodestar_amd/napi/lsg_napi.node");
}

/** Reference set shape check done at call time, as serializeSet throws there (index.ts:177). */
function checkSet(set) {
  if (set.pubkeyIndices === undefined && set.type !== SignatureSetType.single && set.type !== SignatureSetType.aggregate) {
    throw Error("Unknown signature set type");
  }
}

/** FIFO with O(1) shift (Array.prototype.shift is O(n) on long queues). */
class Fifo {
  constructor() {
    this.items = [];
    this.head = 0;
  }
  get length() {
    return this.items.length - this.head;
  }
  push(x) {
    this.items.push(x);
  }
  shift() {
    if (this.head >= this.items.length) return undefined;
    const x = this.items[this.head];
    this.items[this.head++] = undefined;
    if (this.head > 1024 && this.head * 2 > this.items.length) {
      this.items = this.items.slice(this.head);
      this.head = 0;
    }
    return x;
  }
  drain() {
    const out = this.items.slice(this.head);
    this.items = [];
    this.head = 0;
    return out;
  }
}

/**
 * Jobs travel in blocks.  A block is the group of jobs queued together -- one buffered batch
 * of batchable jobs (index.ts:255-302 flushes it to the queue as a whole), or one
 * non-batchable job -- kept as parallel arrays (no object per job), and a job's promise is
 * `block.promise.then(PICK[idx])` with PICK[idx] a shared function reading verdict idx: one
 * promise per call, no executor, no per-call closure.  In node 12 `new Promise(executor)`
 * costs ~0.75 us against ~0.2 us for a `then` on a shared promise, which decides whether the
 * JS thread can feed the GPU at all (it has to issue >1M calls/s).  The block resolves when
 * its last job is answered.
 */
const JOB_PENDING = -1;
const JOB_FAILED = 3; // settled with a JS Error (queue aborted, serialisation)
const MAX_JOBS_PER_BLOCK = 4096;

class VerdictBlock {
  /** batchable: the block's jobs are batchable (a buffered block) or not (one job) */
  constructor(batchable, withTimes) {
    this.sets = []; // per job (queue order): its sets
    this.batchable = batchable;
    this.nFront = 0; // jobs put in front (priority): queue positions 0 .. nFront-1
    this.added = withTimes ? [] : null; // per job: Date.now() at queueing (jobWaitTime metric)
    this.order = null; // queue position -> verdict index, once a priority job went in front
    this.status = null; // per verdict index, allocated when the block is sealed
    this.codes = null;
    this.errors = null;
    this.nSigs = 0;
    this.remaining = 0;
    this.sealed = false;
    this.promise = new Promise((resolve) => {
      this._resolve = resolve;
    });
  }
  /** appends a job; priority jobs of a buffer go to its head (index.ts:296 unshift).
   * Returns the job's verdict index (the order of arrival). */
  add(sets, front) {
    const idx = this.sets.length;
    if (front) {
      if (!this.order) {
        this.order = [];
        for (let k = 0; k < idx; k++) this.order.push(k);
      }
      this.order.unshift(idx);
      this.sets.unshift(sets);
      this.nFront++;
      if (this.added) this.added.unshift(Date.now());
    } else {
      if (this.order) this.order.push(idx);
      this.sets.push(sets);
      if (this.added) this.added.push(Date.now());
    }
    this.nSigs += sets.length;
    return idx;
  }
  /** verdict index of the job at queue position k */
  at(k) {
    return this.order ? this.order[k] : k;
  }
  /** no more jobs: verdict storage for all of them */
  seal() {
    if (this.sealed) return;
    this.sealed = true;
    const n = this.sets.length;
    this.status = new Int8Array(n).fill(JOB_PENDING);
    this.codes = new Int32Array(n);
    this.remaining = n;
    if (n === 0) this._resolve(this);
  }
  settle(idx, status, code, error) {
    if (this.status[idx] !== JOB_PENDING) return;
    this.status[idx] = status;
    this.codes[idx] = code;
    if (status === JOB_FAILED) {
      if (!this.errors) this.errors = [];
      this.errors[idx] = error;
    }
    if (--this.remaining === 0) this._resolve(this);
  }
  failAll(error) {
    this.seal();
    for (let k = 0; k < this.status.length; k++) this.settle(k, JOB_FAILED, 0, error);
  }
  verdict(idx) {
    const st = this.status[idx];
    if (st === LSG_ERROR) throw Error(errorMessage(this.codes[idx]));
    if (st === JOB_FAILED) throw this.errors[idx];
    return st === LSG_VALID;
  }
}

const PICK = [];
for (let i = 0; i < MAX_JOBS_PER_BLOCK; i++) PICK.push((b) => b.verdict(i));

const SET_DESC_WORDS = 7; // pkOff, pkLen, nPks, msgOff, msgLen, sigOff, sigLen (lsg_napi.c verifyPacked)

/**
 * A package of blocks in the addon's packed form: one byte arena with every key, message and
 * signature, 7 descriptor words per set and 2 per job -- the role of the structured clone of
 * BlsWorkReq[] in multithread/index.ts:335 (and of getAggregatedPubkey + toBytes,
 * index.ts:177, except that aggregate keys are summed on the GPU).  A job whose sets cannot
 * be serialized fails on its own and is left out.  `into` (optional) is a previous package's
 * buffers, reused when large enough (fresh multi-MB typed arrays per package cost GC time).
 */
function packBlocks(blocks, nSigs, into, minSigs = 0) {
  let cap = Math.max(nSigs, minSigs) * 224 + 256;
  let arena = into && into.arenaBuf.length >= cap ? into.arenaBuf : new Uint8Array(cap);
  cap = arena.length;
  let off = 0;
  const put = (bytes) => {
    const n = bytes.length;
    if (off + n > cap) {
      while (off + n > cap) cap *= 2;
      const grown = new Uint8Array(cap);
      grown.set(arena.subarray(0, off));
      arena = grown;
    }
    const o = off;
    arena.set(bytes, o);
    off += n;
    return o;
  };
  const setDescBuf =
    into && into.setDescBuf.length >= SET_DESC_WORDS * nSigs ? into.setDescBuf : new Uint32Array(SET_DESC_WORDS * Math.max(nSigs, minSigs));
  let nJobs = 0;
  for (const b of blocks) nJobs += b.sets.length;
  const jobDescBuf = into && into.jobDescBuf.length >= 2 * nJobs ? into.jobDescBuf : new Uint32Array(2 * Math.max(nJobs, minSigs));
  const jobBlock = [];
  const jobIdx = [];
  const sd = setDescBuf;
  let k = 0;
  let j = 0;
  for (const block of blocks) {
    for (let q = 0; q < block.sets.length; q++) {
      const sets = block.sets[q];
      const off0 = off;
      const k0 = k;
      try {
        for (let si = 0; si < sets.length; si++) {
          const set = sets[si];
          const d = SET_DESC_WORDS * k;
          const pk1 = set.pubkeyIndices === undefined && set.type === SignatureSetType.single ? set.pubkey : null;
          const root = set.signingRoot;
          const sig = set.signature;
          if (pk1 instanceof Uint8Array && off + pk1.length + root.length + sig.length <= cap) {
            // the common shape (one raw key): three copies, no helper calls
            arena.set(pk1, off);
            sd[d] = off;
            sd[d + 1] = pk1.length;
            sd[d + 2] = 1;
            off += pk1.length;
            arena.set(root, off);
            sd[d + 3] = off;
            sd[d + 4] = root.length;
            off += root.length;
            arena.set(sig, off);
            sd[d + 5] = off;
            sd[d + 6] = sig.length;
            off += sig.length;
            k++;
            continue;
          }
          if (set.pubkeyIndices !== undefined) {
            const ix = set.pubkeyIndices instanceof Uint32Array ? set.pubkeyIndices : Uint32Array.from(set.pubkeyIndices);
            sd[d] = put(new Uint8Array(ix.buffer, ix.byteOffset, 4 * ix.length));
            sd[d + 1] = 4; // LSG_PK_INDEX
            sd[d + 2] = ix.length;
          } else if (set.type === SignatureSetType.single) {
            const pk = pubkeyBytes(set.pubkey);
            sd[d] = put(pk);
            sd[d + 1] = pk.length;
            sd[d + 2] = 1;
          } else if (set.type === SignatureSetType.aggregate) {
            const pks = set.pubkeys;
            const len = pks.length ? pubkeyBytes(pks[0]).length : 96;
            sd[d] = off;
            for (const pk of pks) {
              const b = pubkeyBytes(pk);
              if (b.length !== len) throw Error("every pubkey of an aggregate set must have the same encoding");
              put(b);
            }
            sd[d + 1] = len;
            sd[d + 2] = pks.length;
          } else {
            throw Error("Unknown signature set type");
          }
          sd[d + 3] = put(root);
          sd[d + 4] = root.length;
          sd[d + 5] = put(sig);
          sd[d + 6] = sig.length;
          k++;
        }
      } catch (e) {
        off = off0;
        k = k0;
        block.settle(block.at(q), JOB_FAILED, 0, e);
        continue;
      }
      jobDescBuf[2 * j] = sets.length;
      jobDescBuf[2 * j + 1] = (block.batchable ? JOB_BATCHABLE : 0) | (q < block.nFront ? JOB_PRIORITY : 0);
      jobBlock.push(block);
      jobIdx.push(block.at(q));
      j++;
    }
  }
  return {
    jobBlock,
    jobIdx,
    arena: arena.subarray(0, off),
    setDesc: sd.subarray(0, SET_DESC_WORDS * k),
    jobDesc: jobDescBuf.subarray(0, 2 * j),
    arenaBuf: arena,
    setDescBuf,
    jobDescBuf,
    nSigs: k,
  };
}

/** GPU package policy defaults (see the class comment) */
const DEFAULT_MAX_SIGS_PER_PACKAGE = 32768;
const DEFAULT_EAGER_PACKAGES = 2;

class BlsGpuVerifier {
  /**
   * @param {{blsVerifyAllMultiThread?: boolean, device?: number, devices?: number[], seed?: number,
   *          maxSigsPerPackage?: number, eagerPackages?: number, minSigsWhenBusy?: number,
   *          maxPendingSigs?: number, bufferWaitMs?: number, reserveSets?: number,
   *          reservePubkeys?: number}} options
   * @param {{logger?: object, metrics?: object|null, addon?: object}} modules  addon is
   *        injectable (tests drive the queue logic with a mock of the addon's surface)
   *
   * Package policy (replaces the CPU pool's "<= 128 sigs per idle worker", index.ts:400-418,
   * whose 16 busy workers would hold the GPU to ~128-set packages and ~40k sets/s):
   *   - up to `eagerPackages` (2) packages go out as soon as jobs are queued, whatever their
   *     size: an idle GPU answers a lone job at once;
   *   - beyond that a package goes out only when the queue holds `minSigsWhenBusy` sigs
   *     (maxSigsPerPackage / 4), or when an in-flight package completes: while the GPU is
   *     busy the queue grows, so under load packages approach `maxSigsPerPackage` (32,768,
   *     one launch filling all 256 CUs) and light load keeps the latency of small packages;
   *   - at most one package per pipeline slot / package thread (addon.slots) is in flight.
   * Back-pressure (canAcceptWork, index.ts:143-149) is on SETS: queued + buffered + in flight
   * < `maxPendingSigs` (3 x maxSigsPerPackage: enough to keep the GPU pipelined, and every
   * pending call is live JS state the young-generation collector copies).  Per-job verdicts do not depend on any of it:
   * the GPU applies worker.ts's batch + retry rules to whatever package it gets.
   * The reference's policy is {maxSigsPerPackage: 128, eagerPackages: slots}.
   */
  constructor(options = {}, modules = {}) {
    this.logger = modules.logger || null;
    this.metrics = modules.metrics || null;
    this.blsVerifyAllMultiThread = options.blsVerifyAllMultiThread === true;
    this.seed = options.seed || 0; // 0: randomizers from the OS CSPRNG (production)
    this.addon = modules.addon || loadAddon();
    // throws loudly without a gfx950 device
    this.ctx = this.addon.open(Array.isArray(options.devices) ? options.devices : options.device || 0);
    this.poolSize = this.addon.slots(this.ctx);
    this.maxSigsPerPackage = options.maxSigsPerPackage || DEFAULT_MAX_SIGS_PER_PACKAGE;
    this.eagerPackages = options.eagerPackages === undefined ? DEFAULT_EAGER_PACKAGES : options.eagerPackages;
    this.minSigsWhenBusy = options.minSigsWhenBusy || Math.max(1, Math.floor(this.maxSigsPerPackage / 4));
    this.maxPendingSigs = options.maxPendingSigs || 3 * this.maxSigsPerPackage;
    this.bufferWaitMs = options.bufferWaitMs === undefined ? MAX_BUFFER_WAIT_MS : options.bufferWaitMs;
    if (options.reserveSets && this.addon.reserve) {
      // preallocate every pipeline slot for packages of up to reserveSets sets (lsg_reserve)
      const pks = options.reservePubkeys || options.reserveSets;
      this.addon.reserve(this.ctx, options.reserveSets, pks, 32 * options.reserveSets, this.poolSize);
    }
    this.jobs = new Fifo(); // queued blocks (index.ts `jobs`, a block at a time)
    this.priorityJobs = []; // blocks of non-batchable priority jobs: a stack, drained first
    this.queuedJobs = 0;
    this.queuedSigs = 0;
    this.bufferedJobs = null;
    this.closed = false;
    this.workersBusy = 0; // packages in flight (the reference's busy workers)
    this.sigsInFlight = 0;
    this.inflight = new Set();
    this.spare = []; // packed buffers of completed packages, reused
    this.stats = {packages: 0, packageSigs: 0}; // packages submitted and their sets (bench, tests)
    this.scheduled = false;
    this.kick = false; // a package completed: the next dispatch goes out whatever its size
    this._runJob = this._runJob.bind(this);
    this._runBufferedJobs = this._runBufferedJobs.bind(this);
    this._onBufferTimer = this._onBufferTimer.bind(this);
    this.bufferTimer = null;
    const m = this.metrics && this.metrics.blsThreadPool;
    if (m && m.queueLength && m.workersBusy && typeof m.queueLength.addCollect === "function") {
      // index.ts:135-140: sampled at scrape time
      m.queueLength.addCollect(() => {
        m.queueLength.set(this.queuedJobs);
        m.workersBusy.set(this.workersBusy);
      });
    }
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

  /** Sets not yet answered: queued, buffered and on the GPU. */
  pendingSigs() {
    return this.queuedSigs + (this.bufferedJobs ? this.bufferedJobs.sigCount : 0) + this.sigsInFlight;
  }

  canAcceptWork() {
    return this.pendingSigs() < this.maxPendingSigs;
  }

  verifySignatureSets(sets, opts = {}) {
    try {
      if (this.metrics && this.metrics.bls) this.metrics.bls.aggregatedPubkeys.inc(getAggregatedPubkeysCount(sets));

      if (opts.verifyOnMainThread && !this.blsVerifyAllMultiThread) {
        // verifySignatureSetsMaybeBatch without the queue: no retry, errors reject
        const m = this.metrics && this.metrics.blsThreadPool;
        const timer = m ? m.mainThreadDurationInThreadPool.startTimer() : null;
        const p = verifyDirect(this.addon, this.ctx, sets, this.seed);
        if (timer) p.then(timer, timer);
        return p;
      }

      for (let i = 0; i < sets.length; i++) checkSet(sets[i]);
      // one chunk (the common case: a gossip call carries one set): the AND over one job's
      // boolean verdict is that verdict, so the job's own promise is the answer
      if (sets.length <= MAX_SIGNATURE_SETS_PER_JOB) return this._queueBlsWork(opts, sets);
      return Promise.all(
        chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map((setsWorker) => this._queueBlsWork(opts, setsWorker))
      ).then((results) => {
        // .every on an empty array returns true
        if (results.length === 0) {
          throw Error("Empty results array");
        }
        return results.every((isValid) => isValid === true);
      });
    } catch (e) {
      return Promise.reject(e);
    }
  }

  /**
   * Per-set verdicts for sets that share one message (north-star extension).  The sets go
   * out as one package of single-set batchable jobs: the GPU verifies them as one RLC batch
   * and, if that fails, re-verifies each set on its own (worker.ts:74-96).  A set whose
   * signature does not decode is reported false.
   */
  verifySignatureSetsSameMessage(sets, message, opts = {}) {
    const o = {batchable: true, priority: opts.priority};
    return Promise.all(
      sets.map((s) =>
        this._queueBlsWork(o, [{type: SignatureSetType.single, pubkey: s.publicKey, signingRoot: message, signature: s.signature}]).catch(
          () => false
        )
      )
    );
  }

  async close() {
    const aborted = new QueueError({code: QueueErrorCode.QUEUE_ABORTED});
    if (this.bufferTimer) {
      clearTimeout(this.bufferTimer);
      this.bufferTimer = null;
    }
    if (this.bufferedJobs) {
      this.bufferedJobs.block.failAll(aborted);
      this.bufferedJobs = null;
    }
    for (const b of this.priorityJobs) b.failAll(aborted);
    for (const b of this.jobs.drain()) b.failAll(aborted);
    this.priorityJobs = [];
    this.queuedJobs = 0;
    this.queuedSigs = 0;
    this.closed = true;
    // let packages already on the GPU finish, then release the device context
    await Promise.all(Array.from(this.inflight));
    if (this.ctx) {
      this.addon.close(this.ctx);
      this.ctx = null;
    }
  }

  _queueBlsWork(opts, sets) {
    if (this.closed) {
      return Promise.reject(new QueueError({code: QueueErrorCode.QUEUE_ABORTED}));
    }
    const priority = opts.priority === true;
    if (opts.batchable === true) {
      let buf = this.bufferedJobs;
      if (!buf) {
        buf = this.bufferedJobs = {sigCount: 0, firstPush: Date.now(), block: new VerdictBlock(true, this.metrics !== null)};
        this._armBufferTimer();
      }
      const idx = buf.block.add(sets, priority);
      const p = buf.block.promise.then(PICK[idx]);
      buf.sigCount += sets.length;
      if (buf.sigCount > MAX_BUFFERED_SIGS || buf.block.sets.length >= MAX_JOBS_PER_BLOCK) this._runBufferedJobs();
      return p;
    }
    const block = new VerdictBlock(false, this.metrics !== null);
    block.add(sets, priority);
    block.seal();
    if (priority) this.priorityJobs.push(block);
    else this.jobs.push(block);
    this.queuedJobs++;
    this.queuedSigs += sets.length;
    this._schedule();
    return block.promise.then(PICK[0]);
  }

  /** One timer for the buffer's 100 ms limit (index.ts:291-293 arms one per buffer; a buffer
   * that fills first would cost a setTimeout + clearTimeout pair per ~33 sigs): on firing it
   * flushes the buffer if it is old enough, else re-arms for the rest of its wait. */
  _armBufferTimer() {
    if (!this.bufferTimer) this.bufferTimer = setTimeout(this._onBufferTimer, this.bufferWaitMs);
  }

  _onBufferTimer() {
    this.bufferTimer = null;
    const buf = this.bufferedJobs;
    if (!buf) return;
    const age = Date.now() - buf.firstPush;
    if (age >= this.bufferWaitMs) this._runBufferedJobs();
    else this.bufferTimer = setTimeout(this._onBufferTimer, this.bufferWaitMs - age);
  }

  _schedule() {
    // setImmediate, not the reference's setTimeout(0) (a >= 1 ms timer in node)
    if (!this.scheduled) {
      this.scheduled = true;
      setImmediate(this._runJob);
    }
  }

  _runJob() {
    this.scheduled = false;
    if (this.closed) return;
    while (this.workersBusy < this.poolSize && this.queuedJobs > 0) {
      // while the GPU is busy let the queue grow into a large package, unless a package has
      // just completed (class comment)
      if (this.workersBusy >= this.eagerPackages && this.queuedSigs < this.minSigsWhenBusy && !this.kick) break;
      this.kick = false;
      const blocks = this._prepareWork();
      if (blocks.length === 0) break;
      this._runPackage(blocks);
    }
  }

  _runPackage(blocks) {
    const m = this.metrics && this.metrics.blsThreadPool;
    let startedSigSets = 0;
    let startedJobs = 0;
    const now = m ? Date.now() : 0;
    for (const b of blocks) {
      startedSigSets += b.nSigs;
      startedJobs += b.sets.length;
      if (m) for (const t of b.added) m.jobWaitTime.observe((now - t) / 1000);
    }
    if (m) {
      m.totalJobsGroupsStarted.inc(1);
      m.totalJobsStarted.inc(startedJobs);
      m.totalSigSetsStarted.inc(startedSigSets);
    }
    this.workersBusy++;
    this.sigsInFlight += startedSigSets;
    this.stats.packages++;
    this.stats.packageSigs += startedSigSets;
    const run = (async () => {
      let pkg = null;
      try {
        // buffers sized for a full package, so that every one can be reused
        pkg = packBlocks(blocks, startedSigSets, this.spare.pop(), this.maxSigsPerPackage);
        const n = pkg.jobBlock.length;
        if (n === 0) return;
        const jobStartNs = process.hrtime.bigint();
        const workResult = await this.addon.verifyPacked(this.ctx, pkg.arena, pkg.setDesc, pkg.jobDesc, this.seed);
        const jobEndNs = process.hrtime.bigint();
        const status = workResult.status;
        const codes = workResult.errCode;
        let errorCount = 0;
        for (let i = 0; i < n; i++) {
          if (status[i] === LSG_ERROR) errorCount += pkg.jobBlock[i].sets.length;
          pkg.jobBlock[i].settle(pkg.jobIdx[i], status[i], codes[i]);
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
          m.successJobsSignatureSetsCount.inc(pkg.nSigs - errorCount);
          m.errorJobsSignatureSetsCount.inc(errorCount);
          m.batchRetries.inc(workResult.batchRetries);
          m.batchSigsSuccess.inc(workResult.batchSigsSuccess);
        }
        if (this.spare.length < this.poolSize) this.spare.push(pkg);
      } catch (e) {
        if (!this.closed && this.logger) this.logger.error("BlsGpuVerifier error", {}, e);
        for (const b of blocks) b.failAll(e);
      }
    })();
    this.inflight.add(run);
    run.then(() => {
      this.inflight.delete(run);
      this.workersBusy--;
      this.sigsInFlight -= startedSigSets;
      this.kick = true;
      this._schedule();
    });
  }

  /** blocks for one package: priority blocks first, then FIFO, up to maxSigsPerPackage sigs
   * (a block is never split; index.ts:400-418 takes whole jobs the same way) */
  _prepareWork() {
    const blocks = [];
    let totalSigs = 0;
    let totalJobs = 0;
    while (totalSigs < this.maxSigsPerPackage) {
      const b = this.priorityJobs.length ? this.priorityJobs.pop() : this.jobs.shift();
      if (!b) break;
      blocks.push(b);
      totalSigs += b.nSigs;
      totalJobs += b.sets.length;
    }
    this.queuedSigs -= totalSigs;
    this.queuedJobs -= totalJobs;
    return blocks;
  }

  _runBufferedJobs() {
    const buf = this.bufferedJobs;
    if (buf) {
      // the buffer goes to the tail of the queue as a whole (index.ts:425-431)
      this.bufferedJobs = null;
      buf.block.seal();
      this.jobs.push(buf.block);
      this.queuedJobs += buf.block.sets.length;
      this.queuedSigs += buf.block.nSigs;
      this._schedule();
    }
  }
}

/**
 * BlsSingleThreadVerifier (chain/bls/singleThread.ts:14-35) on the GPU: each call is one
 * verifySignatureSetsMaybeBatch (verifyDirect: one priority job, no queue) with no retry; opts
 * are ignored, errors reject.  The reference blocks the event loop for the call; here the
 * promise settles when the GPU answers.  The duration is observed after the call as the
 * reference does (it observes the total and the per-set time; its startNs - endNs has the
 * sign inverted, here the duration is positive).
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
    // Count time after aggregating (serialisation happens inside verifyDirect)
    const startNs = process.hrtime.bigint();
    const valid = await verifyDirect(this.addon, this.ctx, sets, this.seed);
    // Don't use a try/catch, only count run without exceptions
    const endNs = process.hrtime.bigint();
    const totalSec = Number(endNs - startNs) / 1e9;
    const m = this.metrics && this.metrics.blsThreadPool;
    if (m) {
      m.mainThreadDurationInThreadPool.observe(totalSec);
      m.mainThreadDurationInThreadPool.observe(totalSec / sets.length);
    }
    return valid;
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
  packBlocks,
  DEFAULT_MAX_SIGS_PER_PACKAGE,
  MAX_SIGNATURE_SETS_PER_JOB,
  MAX_BUFFERED_SIGS,
  MAX_BUFFER_WAIT_MS,
  MAX_JOBS_CAN_ACCEPT_WORK,
};
