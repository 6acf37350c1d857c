"use strict";
/**
 * Host-logic tests of BlsGpuVerifier (lodestar_amd/js/blsGpuVerifier.js) on the CPU, with a
 * mock of the N-API addon's surface.  They restate the reference's own tests of the pool:
 *   test/unit/chain/bls/utils.test.ts:7-25          chunkifyMaximizeChunkSize cases
 *   test/e2e/chain/bls/multithread.test.ts:25-103   8 x 3 valid sets (sync / async / batchable),
 *                                                   a BLST_INVALID_SIZE job does not poison others
 * plus the queue rules of multithread/index.ts (buffering, <=128 sigs per package, AND over
 * chunks, empty -> throw, back-pressure, close -> QUEUE_ERROR_QUEUE_ABORTED).
 * The mock's verdict rule is a toy (signature[0] == message[0]); the real verdicts are
 * tested on the GPU (tests/js/test_verifier_gpu.js, tests/test_gpu_parity.py).
 * Run: node tests/js/test_verifier_host.js   (driven by tests/test_js_host.py)
 */
const assert = require("assert");
const path = require("path");
const V = require(path.join(__dirname, "..", "..", "lodestar_amd", "js", "blsGpuVerifier.js"));

/** Decodes verifyPacked's arena / descriptors back into jobs (lsg_napi.c layout). */
function unpack(arena, setDesc, jobDesc) {
  const jobs = [];
  let k = 0;
  for (let j = 0; j < jobDesc.length / 2; j++) {
    const sets = [];
    for (let q = 0; q < jobDesc[2 * j]; q++, k++) {
      const d = setDesc.subarray(7 * k, 7 * k + 7);
      const pubkeys = [];
      for (let p = 0; p < d[2]; p++) pubkeys.push(arena.slice(d[0] + p * d[1], d[0] + (p + 1) * d[1]));
      sets.push({pubkeys, pkLen: d[1], message: arena.slice(d[3], d[3] + d[4]), signature: arena.slice(d[5], d[5] + d[6])});
    }
    jobs.push({sets, flags: jobDesc[2 * j + 1]});
  }
  return jobs;
}

function mockAddon(slots = 2, {holdWaits = false} = {}) {
  const m = {
    packages: [],
    priorityPackages: [],
    pendingPriority: 0,
    syncCalls: 0,
    opened: 0,
    closed: 0,
    pending: [],
    openedWith: [],
    reserved: null,
    open(dev) {
      m.opened++;
      m.openedWith.push(dev);
      return {ctx: true};
    },
    reserve(ctx, sets, pks, bytes, slotsN) {
      m.reserved = [sets, pks, bytes, slotsN];
    },
    close() {
      m.closed++;
    },
    slots() {
      return slots;
    },
    setVerdict(set) {
      if (set.signature.length !== 96) return {status: 2, errCode: 10};
      for (const pk of set.pubkeys) if (pk.length !== 96) return {status: 2, errCode: 1};
      return {status: set.signature[0] === set.message[0] ? 1 : 0, errCode: 0};
    },
    jobVerdict(sets) {
      if (sets.length === 0) return {status: 2, errCode: 100};
      let ok = true;
      for (const s of sets) {
        const r = m.setVerdict(s);
        if (r.status === 2) return r;
        ok = ok && r.status === 1;
      }
      return {status: ok ? 1 : 0, errCode: 0};
    },
    verifyPacked(ctx, arena, setDesc, jobDesc, seed, priority) {
      // the engine runs at most `slots` packages at once (one package thread each), plus
      // priority packages on its priority thread
      const jobs = unpack(arena, setDesc, jobDesc);
      if (priority) {
        m.priorityPackages.push(jobs);
      } else {
        if (m.pending.length - m.pendingPriority >= slots) throw Error("mock: more packages in flight than package threads");
        m.packages.push(jobs);
      }
      const t = {ticket: m.packages.length, jobs, priority: !!priority};
      m.pending.push(t);
      if (priority) m.pendingPriority++;
      const vs = jobs.map((j) => m.jobVerdict(j.sets));
      // GPU package start/end on process.hrtime's clock (lsg_stats is CLOCK_MONOTONIC)
      const startNs = Number(process.hrtime.bigint());
      const done = {
        status: Uint8Array.from(vs.map((v) => v.status)),
        errCode: Int32Array.from(vs.map((v) => v.errCode)),
        batchRetries: 0,
        batchSigsSuccess: 0,
        startNs,
        endNs: startNs + 1e6,
        workerId: t.ticket % 3,
      };
      const finish = () => {
        m.pending.splice(m.pending.indexOf(t), 1);
        if (t.priority) m.pendingPriority--;
        return done;
      };
      if (!holdWaits) return new Promise((r) => setTimeout(() => r(finish()), 1));
      return new Promise((r) => {
        t.release = () => r(finish());
      });
    },
    verifySets(ctx, sets) {
      m.syncCalls++;
      return m.jobVerdict(sets);
    },
  };
  return m;
}

function set(i, valid = true) {
  const message = new Uint8Array(32).fill(i + 1);
  const signature = new Uint8Array(96).fill(valid ? i + 1 : i + 2);
  return {type: V.SignatureSetType.single, pubkey: new Uint8Array(96).fill(7), signingRoot: message, signature};
}

const sleep = (ms) => new Promise((r) => setTimeout(r, ms));
const tests = [];
function test(name, fn) {
  tests.push({name, fn});
}

test("chunkifyMaximizeChunkSize reference cases (utils.test.ts:7-25)", () => {
  const expected = [
    [[0]],
    [[0, 1]],
    [[0, 1, 2]],
    [[0, 1, 2, 3]],
    [[0, 1, 2, 3, 4]],
    [[0, 1, 2], [3, 4, 5]],
    [[0, 1, 2, 3], [4, 5, 6]],
    [[0, 1, 2, 3], [4, 5, 6, 7]],
  ];
  expected.forEach((exp, i) => {
    const arr = Array.from({length: i + 1}, (_, k) => k);
    assert.deepStrictEqual(V.chunkifyMaximizeChunkSize(arr, 3), exp);
  });
});

test("8 x 3 valid sets submitted synchronously -> one package (multithread.test.ts:72-75)", async () => {
  const a = mockAddon();
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  const sets = [0, 1, 2].map((i) => set(i));
  const res = await Promise.all(Array.from({length: 8}, () => pool.verifySignatureSets(sets)));
  assert.deepStrictEqual(res, Array(8).fill(true));
  // the first runJob takes up to 128 sigs: all 8 jobs (24 sets) in one package
  assert.strictEqual(a.packages.length, 1);
  assert.strictEqual(a.packages[0].length, 8);
  assert.strictEqual(a.packages[0][0].flags, 0);
  await pool.close();
});

test("8 x 3 valid sets submitted with sleeps -> separate packages (multithread.test.ts:77-80)", async () => {
  const a = mockAddon();
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  const sets = [0, 1, 2].map((i) => set(i));
  const ps = [];
  for (let i = 0; i < 8; i++) {
    ps.push(pool.verifySignatureSets(sets));
    await sleep(5);
  }
  assert.deepStrictEqual(await Promise.all(ps), Array(8).fill(true));
  assert.ok(a.packages.length >= 4, `packages ${a.packages.length}`);
  await pool.close();
});

test("batchable jobs are buffered: > 32 sigs flush immediately, else after 100 ms", async () => {
  const a = mockAddon();
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  const sets = [0, 1, 2].map((i) => set(i));
  // 11 x 3 = 33 sigs > MAX_BUFFERED_SIGS: flushed at the 11th call without waiting 100 ms
  const t0 = Date.now();
  const ps = Array.from({length: 11}, () => pool.verifySignatureSets(sets, {batchable: true}));
  assert.deepStrictEqual(await Promise.all(ps), Array(11).fill(true));
  assert.ok(Date.now() - t0 < 90, "flush by count must not wait for the timer");
  assert.strictEqual(a.packages.length, 1);
  assert.ok(a.packages[0].every((j) => j.flags === 1));
  // 2 x 3 sigs: held until the 100 ms timer
  const t1 = Date.now();
  const ps2 = [pool.verifySignatureSets(sets, {batchable: true}), pool.verifySignatureSets(sets, {batchable: true})];
  await sleep(30);
  assert.strictEqual(a.packages.length, 1, "still buffered");
  assert.deepStrictEqual(await Promise.all(ps2), [true, true]);
  assert.ok(Date.now() - t1 >= 95, "timer flush");
  assert.strictEqual(a.packages.length, 2);
  await pool.close();
});

test("invalid-size signature rejects with BLST_INVALID_SIZE without poisoning co-batched jobs (multithread.test.ts:88-103)", async () => {
  const a = mockAddon();
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  const sets = [0, 1, 2].map((i) => set(i));
  const bad = Object.assign({}, sets[0], {signature: new Uint8Array(32)});
  const pBad = pool.verifySignatureSets([bad], {batchable: true});
  const ps = Array.from({length: 8}, () => pool.verifySignatureSets(sets, {batchable: true}));
  await assert.rejects(pBad, /BLST_INVALID_SIZE/);
  assert.deepStrictEqual(await Promise.all(ps), Array(8).fill(true));
  await pool.close();
});

test("> 128 sets are chunked (<= 128 per job) and the verdict is the AND over chunks", async () => {
  const a = mockAddon();
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  const many = Array.from({length: 300}, (_, i) => set(i % 200));
  assert.strictEqual(await pool.verifySignatureSets(many), true);
  const jobs = [].concat(...a.packages);
  assert.deepStrictEqual(jobs.map((j) => j.sets.length), [150, 150]);
  many[299] = set(5, false);
  assert.strictEqual(await pool.verifySignatureSets(many), false);
  await pool.close();
});

test("reference policy: a package holds at most 128 sigs of queued jobs (prepareWork, index.ts:400-418)", async () => {
  const a = mockAddon(1);
  const pool = new V.BlsGpuVerifier({maxSigsPerPackage: 128, eagerPackages: 1}, {addon: a});
  const sets100 = Array.from({length: 100}, (_, i) => set(i));
  const ps = [pool.verifySignatureSets(sets100), pool.verifySignatureSets(sets100), pool.verifySignatureSets(sets100)];
  assert.deepStrictEqual(await Promise.all(ps), [true, true, true]);
  // 100 < 128 -> takes a second job (200 sigs), then the third goes alone
  assert.deepStrictEqual(a.packages.map((p) => p.length), [2, 1]);
  await pool.close();
});

test("GPU sizing: one package takes every queued job (default 32768 sigs) without changing verdicts", async () => {
  const a = mockAddon(1);
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  const sets100 = Array.from({length: 100}, (_, i) => set(i));
  const bad = Array.from({length: 100}, (_, i) => (i === 7 ? Object.assign({}, set(i), {signingRoot: new Uint8Array(32).fill(9)}) : set(i)));
  const ps = [pool.verifySignatureSets(sets100), pool.verifySignatureSets(bad), pool.verifySignatureSets(sets100)];
  assert.deepStrictEqual(await Promise.all(ps), [true, false, true]);
  // all three jobs (300 sigs) in one package, where the reference's 128 cap makes two
  assert.deepStrictEqual(a.packages.map((p) => p.length), [3]);
  await pool.close();
});

test("empty set list: job error 'Empty signature set' (maybeBatch.ts:29-31)", async () => {
  const a = mockAddon();
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  await assert.rejects(pool.verifySignatureSets([]), /Empty signature set/);
  await pool.close();
});

test("aggregate sets send every pubkey (summed on the GPU, utils.ts:11)", async () => {
  const a = mockAddon();
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  const s = set(3);
  const agg = {type: V.SignatureSetType.aggregate, pubkeys: [s.pubkey, s.pubkey, s.pubkey], signingRoot: s.signingRoot, signature: s.signature};
  assert.strictEqual(await pool.verifySignatureSets([agg]), true);
  assert.strictEqual(a.packages[0][0].sets[0].pubkeys.length, 3);
  await pool.close();
});

test("verifyOnMainThread: one priority job outside the queue, no retry, errors reject (index.ts:155-168)", async () => {
  const a = mockAddon();
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  assert.strictEqual(await pool.verifySignatureSets([set(1), set(2)], {verifyOnMainThread: true}), true);
  assert.strictEqual(a.syncCalls, 0);
  assert.strictEqual(a.packages.length, 0);
  assert.strictEqual(a.priorityPackages.length, 1);
  // one non-batchable priority job holding both sets: maybeBatch over them (no retry)
  assert.strictEqual(a.priorityPackages[0].length, 1);
  assert.strictEqual(a.priorityPackages[0][0].sets.length, 2);
  assert.strictEqual(a.priorityPackages[0][0].flags, 2 /* LSG_JOB_PRIORITY, not batchable */);
  assert.strictEqual(await pool.verifySignatureSets([set(3, false)], {verifyOnMainThread: true}), false);
  const bad = Object.assign({}, set(1), {signature: new Uint8Array(10)});
  await assert.rejects(pool.verifySignatureSets([bad], {verifyOnMainThread: true}), /BLST_INVALID_SIZE/);
  await assert.rejects(pool.verifySignatureSets([], {verifyOnMainThread: true}), /Empty signature set/);
  assert.strictEqual(a.syncCalls, 0);
  // blsVerifyAllMultiThread forces the queue path
  const pool2 = new V.BlsGpuVerifier({blsVerifyAllMultiThread: true}, {addon: a});
  assert.strictEqual(await pool2.verifySignatureSets([set(1)], {verifyOnMainThread: true}), true);
  assert.strictEqual(a.packages.length, 1);
  await pool.close();
  await pool2.close();
});

test("verifyOnMainThread does not block the event loop: setImmediate fires while it is pending (VERDICT r3 4)", async () => {
  const a = mockAddon(2, {holdWaits: true});
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  let settled = false;
  const p = pool.verifySignatureSets([set(1)], {verifyOnMainThread: true}).then((v) => {
    settled = true;
    return v;
  });
  let immediate = false;
  await new Promise((r) => setImmediate(() => {
    immediate = true;
    r();
  }));
  assert.strictEqual(immediate, true);
  assert.strictEqual(settled, false); // the GPU has not answered: the JS thread kept running
  assert.strictEqual(a.pending.length, 1);
  // it overtakes a full pool: both package threads busy with held packages
  const q1 = pool.verifySignatureSets([set(2)]);
  const q2 = pool.verifySignatureSets([set(3)]);
  await sleep(5);
  a.pending[0].release();
  assert.strictEqual(await p, true);
  while (a.pending.length) {
    a.pending[0].release();
    await sleep(2);
  }
  assert.deepStrictEqual(await Promise.all([q1, q2]), [true, true]);
  await pool.close();
});

test("canAcceptWork: back-pressure on sets pending (queued + buffered + in flight) (index.ts:143-149)", async () => {
  const a = mockAddon(2, {holdWaits: true});
  const pool = new V.BlsGpuVerifier({maxPendingSigs: 6}, {addon: a});
  assert.strictEqual(pool.canAcceptWork(), true);
  const p1 = pool.verifySignatureSets([set(1), set(2)]);
  const p2 = pool.verifySignatureSets([set(3), set(4)]);
  await sleep(2);
  assert.strictEqual(a.packages.length, 1, "both jobs queued in one tick go as one package");
  assert.strictEqual(pool.pendingSigs(), 4);
  assert.strictEqual(pool.canAcceptWork(), true);
  const p3 = pool.verifySignatureSets([set(5)], {batchable: true}); // buffered: counts too
  const p4 = pool.verifySignatureSets([set(6)], {batchable: true});
  assert.strictEqual(pool.pendingSigs(), 6);
  assert.strictEqual(pool.canAcceptWork(), false);
  a.pending[0].release();
  await sleep(5);
  assert.strictEqual(pool.pendingSigs(), 2);
  assert.strictEqual(pool.canAcceptWork(), true);
  assert.deepStrictEqual(await Promise.all([p1, p2]), [true, true]);
  await sleep(120); // buffer timer: the two batchable jobs go out as one package
  for (const t of a.pending.slice()) t.release();
  assert.deepStrictEqual(await Promise.all([p3, p4]), [true, true]);
  assert.strictEqual(pool.pendingSigs(), 0);
  await pool.close();
});

test("GPU package policy: eager packages while the GPU is idle, then the queue grows into large packages", async () => {
  const a = mockAddon(16, {holdWaits: true});
  const pool = new V.BlsGpuVerifier({maxSigsPerPackage: 1000, eagerPackages: 2, minSigsWhenBusy: 250}, {addon: a});
  const ps = [];
  ps.push(pool.verifySignatureSets([set(1)]));
  await sleep(2);
  ps.push(pool.verifySignatureSets([set(2)]));
  await sleep(2);
  assert.deepStrictEqual(a.packages.map((p) => p.length), [1, 1], "two eager one-job packages");
  for (let i = 0; i < 100; i++) ps.push(pool.verifySignatureSets([set(i % 7)]));
  await sleep(2);
  assert.strictEqual(a.packages.length, 2, "100 queued sigs < minSigsWhenBusy: held while 2 packages run");
  for (let i = 0; i < 200; i++) ps.push(pool.verifySignatureSets([set(i % 7)]));
  await sleep(2);
  assert.deepStrictEqual(a.packages.map((p) => p.length), [1, 1, 300], "300 >= 250 queued sigs: one package");
  for (let i = 0; i < 10; i++) ps.push(pool.verifySignatureSets([set(i % 7)]));
  await sleep(2);
  assert.strictEqual(a.packages.length, 3);
  a.pending[0].release(); // a package completes: the queue goes out at once
  await sleep(3);
  assert.deepStrictEqual(a.packages.map((p) => p.length), [1, 1, 300, 10]);
  for (let i = 0; i < 2500; i++) ps.push(pool.verifySignatureSets([set(i % 7)]));
  await sleep(3);
  // 2500 queued: packages of at most maxSigsPerPackage sigs
  assert.deepStrictEqual(a.packages.slice(4).map((p) => p.length), [1000, 1000, 500]);
  while (a.pending.length) {
    for (const t of a.pending.slice()) t.release();
    await sleep(2);
  }
  const res = await Promise.all(ps);
  assert.strictEqual(res.length, 2812);
  assert.ok(res.every((r) => r === true));
  await pool.close();
});

test("at most one package per package thread (addon.slots) is in flight", async () => {
  const a = mockAddon(2, {holdWaits: true});
  const pool = new V.BlsGpuVerifier({eagerPackages: 8}, {addon: a});
  const ps = [];
  for (let i = 0; i < 3; i++) {
    ps.push(pool.verifySignatureSets([set(i)]));
    await sleep(2);
  }
  assert.strictEqual(a.pending.length, 2);
  assert.strictEqual(a.packages.length, 2);
  a.pending[0].release();
  await sleep(3);
  assert.strictEqual(a.packages.length, 3, "freed slot picks up the queued job");
  for (const t of a.pending.slice()) t.release();
  assert.deepStrictEqual(await Promise.all(ps), [true, true, true]);
  await pool.close();
});

test("close rejects queued and buffered jobs with QUEUE_ERROR_QUEUE_ABORTED (index.ts:193-202)", async () => {
  const a = mockAddon(1, {holdWaits: true});
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  const running = pool.verifySignatureSets([set(1)]);
  await sleep(2);
  const queued = pool.verifySignatureSets([set(2)]);
  const buffered = pool.verifySignatureSets([set(3)], {batchable: true});
  await sleep(2);
  const closing = pool.close();
  await assert.rejects(queued, (e) => e.code === "QUEUE_ERROR_QUEUE_ABORTED");
  await assert.rejects(buffered, (e) => e.code === "QUEUE_ERROR_QUEUE_ABORTED");
  a.pending[0].release(); // the package already on the device completes normally
  assert.strictEqual(await running, true);
  await closing;
  assert.strictEqual(a.closed, 1);
  await assert.rejects(pool.verifySignatureSets([set(4)]), (e) => e.code === "QUEUE_ERROR_QUEUE_ABORTED");
});

test("priority jobs go to the head of the queue (north-star extension)", async () => {
  const a = mockAddon(1, {holdWaits: true});
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  const p0 = pool.verifySignatureSets(Array.from({length: 128}, (_, i) => set(i)));
  await sleep(2);
  const pa = pool.verifySignatureSets(Array.from({length: 128}, (_, i) => set(i)));
  const pb = pool.verifySignatureSets([set(9)], {priority: true});
  await sleep(2);
  a.pending[0].release();
  await sleep(5);
  assert.strictEqual(a.packages[1][0].sets.length, 1, "priority job runs first");
  assert.strictEqual(a.packages[1][0].flags & 2, 2);
  for (const t of a.pending.slice()) t.release();
  assert.deepStrictEqual(await Promise.all([p0, pa, pb]), [true, true, true]);
  await pool.close();
});

test("verifySignatureSetsSameMessage returns per-set verdicts (north-star extension)", async () => {
  const a = mockAddon();
  const pool = new V.BlsGpuVerifier({}, {addon: a});
  const msg = new Uint8Array(32).fill(4);
  const good = {publicKey: new Uint8Array(96), signature: new Uint8Array(96).fill(4)};
  const badSig = {publicKey: new Uint8Array(96), signature: new Uint8Array(96).fill(5)};
  const badLen = {publicKey: new Uint8Array(96), signature: new Uint8Array(20)};
  assert.deepStrictEqual(await pool.verifySignatureSetsSameMessage([good, badSig, good, badLen], msg), [true, false, true, false]);
  await pool.close();
});

/** A stand-in for the reference's metrics registry (gauges / histograms with the same method
 * names as prom-client's, metrics/metrics/lodestar.ts:350-430), recording every observation. */
function mockMetrics() {
  const rec = {};
  const gauge = (name) => ({
    inc(a, b) {
      (rec[name] = rec[name] || []).push(b === undefined ? a : [a, b]);
    },
  });
  const hist = (name) => ({
    observe(v) {
      (rec[name] = rec[name] || []).push(v);
    },
    startTimer() {
      const t0 = process.hrtime.bigint();
      return () => (rec[name] = rec[name] || []).push(Number(process.hrtime.bigint() - t0) / 1e9);
    },
  });
  const blsThreadPool = {};
  for (const g of ["jobsWorkerTime", "successJobsSignatureSetsCount", "errorJobsSignatureSetsCount", "totalJobsGroupsStarted",
                   "totalJobsStarted", "totalSigSetsStarted", "batchRetries", "batchSigsSuccess"])
    blsThreadPool[g] = gauge(g);
  for (const h of ["jobWaitTime", "latencyToWorker", "latencyFromWorker", "mainThreadDurationInThreadPool", "timePerSigSet"])
    blsThreadPool[h] = hist(h);
  return {rec, metrics: {bls: {aggregatedPubkeys: gauge("aggregatedPubkeys")}, blsThreadPool}};
}

test("metrics: the reference's names and observation points (index.ts:319-381, lodestar.ts:350-430)", async () => {
  const a = mockAddon();
  const {rec, metrics} = mockMetrics();
  const pool = new V.BlsGpuVerifier({}, {addon: a, metrics});
  const sets = [0, 1, 2].map((i) => set(i));
  await Promise.all([pool.verifySignatureSets(sets), pool.verifySignatureSets([set(4, false)])]);
  for (const k of ["jobWaitTime", "totalJobsGroupsStarted", "totalJobsStarted", "totalSigSetsStarted", "timePerSigSet",
                   "jobsWorkerTime", "latencyToWorker", "latencyFromWorker", "successJobsSignatureSetsCount",
                   "errorJobsSignatureSetsCount", "batchRetries", "batchSigsSuccess"])
    assert.ok(rec[k] && rec[k].length > 0, k);
  const [labels, sec] = rec.jobsWorkerTime[0];
  assert.ok("workerId" in labels && Math.abs(sec - 1e-3) < 1e-9, JSON.stringify(rec.jobsWorkerTime));
  assert.ok(rec.latencyToWorker.every((x) => x >= 0 && x < 1), rec.latencyToWorker);
  assert.ok(rec.latencyFromWorker.every((x) => x < 1), rec.latencyFromWorker);
  assert.ok(!rec.mainThreadDurationInThreadPool);
  assert.strictEqual(await pool.verifySignatureSets(sets, {verifyOnMainThread: true}), true);
  assert.strictEqual(rec.mainThreadDurationInThreadPool.length, 1);
  await pool.close();
});

test("BlsGpuSingleThreadVerifier: one maybeBatch per call, no retry, throws (singleThread.ts:14-35)", async () => {
  const a = mockAddon();
  const {rec, metrics} = mockMetrics();
  const v = V.createBlsVerifier({blsVerifyAllMainThread: true}, {addon: a, metrics});
  assert.ok(v instanceof V.BlsGpuSingleThreadVerifier);
  assert.strictEqual(v.canAcceptWork(), true);
  const sets = [0, 1, 2].map((i) => set(i));
  assert.strictEqual(await v.verifySignatureSets(sets), true);
  assert.strictEqual(await v.verifySignatureSets([set(0), set(1, false)], {batchable: true}), false);
  const bad = set(2);
  bad.signature = new Uint8Array(32);
  await assert.rejects(v.verifySignatureSets([bad]), /BLST_INVALID_SIZE/);
  assert.strictEqual(a.syncCalls, 0);
  assert.strictEqual(a.priorityPackages.length, 3, "one priority job per call");
  assert.strictEqual(a.packages.length, 0, "no queue, no worker packages");
  assert.strictEqual(rec.mainThreadDurationInThreadPool.length, 4, "total and per-set time of the two successful calls");
  assert.ok(rec.mainThreadDurationInThreadPool.every((x) => x >= 0));
  await v.close();
  assert.strictEqual(a.closed, 1);
  assert.ok(V.createBlsVerifier({}, {addon: mockAddon()}) instanceof V.BlsGpuVerifier);
});

test("devices / reserveSets open one context over the node's GPUs and preallocate (chain.ts:195-198)", async () => {
  const a = mockAddon();
  const pool = new V.BlsGpuVerifier({devices: [0, 1, 2, 3], reserveSets: 32768, maxSigsPerPackage: 32768}, {addon: a});
  assert.deepStrictEqual(a.openedWith, [[0, 1, 2, 3]]);
  assert.deepStrictEqual(a.reserved, [32768, 32768, 32 * 32768, 2]);
  await pool.close();
});

(async () => {
  let failed = 0;
  for (const t of tests) {
    try {
      await t.fn();
      console.log("ok  ", t.name);
    } catch (e) {
      failed++;
      console.log("FAIL", t.name, "\n", e && e.stack);
    }
  }
  console.log(`${tests.length - failed}/${tests.length} passed`);
  process.exit(failed ? 1 : 0);
})();
