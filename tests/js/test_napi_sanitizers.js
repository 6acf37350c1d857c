"use strict";
/**
 * Traffic for the sanitizer build of the N-API addon (tests/test_napi_sanitizers.py): the real
 * lsg_napi.c, compiled with -fsanitize=address,undefined and linked against the host stub of
 * the C ABI (tests/native/lsg_stub.c), driven through BlsGpuVerifier the way a beacon node
 * drives it (multithread/index.ts:151-431): thousands of concurrent batchable calls, non-batchable
 * and aggregate jobs, keys by table index, invalid sizes, verifyOnMainThread calls overtaking a
 * full pool, the single-thread verifier, the utility exports, and close() with packages in
 * flight -- with forced garbage collections so that a buffer the addon reads after its JS owner
 * died shows up as a use-after-free.  The stub's verdict rule: a set is valid iff
 * signature[0] == message[0].
 * Run: node --expose-gc tests/js/test_napi_sanitizers.js <addon.node>
 */
const assert = require("assert");
const path = require("path");
const V = require(path.join(__dirname, "..", "..", "lodestar_amd", "js", "blsGpuVerifier.js"));

const addon = require(path.resolve(process.argv[2]));
const gc = typeof global.gc === "function" ? global.gc : () => {};

let seed = 12345;
function rnd(n) {
  seed = (seed * 1103515245 + 12345) & 0x7fffffff;
  return seed % n;
}
function set(i, valid, {sigLen = 96, aggregate = 0, indices = 0} = {}) {
  const message = new Uint8Array(32).fill(i & 255);
  const signature = new Uint8Array(sigLen).fill(valid ? i & 255 : (i + 1) & 255);
  if (indices) return {pubkeyIndices: Uint32Array.from({length: indices}, (_, k) => k + i), signingRoot: message, signature};
  if (aggregate) {
    const pubkeys = Array.from({length: aggregate}, (_, k) => new Uint8Array(96).fill(k + 1));
    return {type: V.SignatureSetType.aggregate, pubkeys, signingRoot: message, signature};
  }
  return {type: V.SignatureSetType.single, pubkey: new Uint8Array(96).fill(7), signingRoot: message, signature};
}

(async () => {
  const pool = new V.BlsGpuVerifier({maxSigsPerPackage: 512, reserveSets: 512}, {addon});
  assert.ok(pool.poolSize >= 1);
  // 1. a firehose of batchable single-set calls, 5 % invalid
  for (let round = 0; round < 4; round++) {
    const calls = [];
    const expect = [];
    for (let i = 0; i < 3000; i++) {
      const ok = rnd(20) !== 0;
      calls.push(pool.verifySignatureSets([set(i, ok)], {batchable: true}));
      expect.push(ok);
    }
    gc();
    assert.deepStrictEqual(await Promise.all(calls), expect);
  }
  // 2. mixed jobs: non-batchable multi-set, aggregates, table indices, > 128 sets (chunked)
  const mixed = [];
  const mexp = [];
  for (let i = 0; i < 400; i++) {
    const n = 1 + rnd(4);
    const sets = [];
    let ok = true;
    for (let k = 0; k < n; k++) {
      const v = rnd(10) !== 0;
      ok = ok && v;
      const kind = rnd(3);
      sets.push(set(i * 7 + k, v, kind === 0 ? {} : kind === 1 ? {aggregate: 1 + rnd(20)} : {indices: 1 + rnd(40)}));
    }
    mixed.push(pool.verifySignatureSets(sets, {batchable: rnd(2) === 0}));
    mexp.push(ok);
  }
  const big = Array.from({length: 300}, (_, k) => set(k, true));
  mixed.push(pool.verifySignatureSets(big));
  mexp.push(true);
  gc();
  assert.deepStrictEqual(await Promise.all(mixed), mexp);
  // 3. errors: a wrong-size signature rejects without poisoning co-batched jobs; empty jobs
  const good = Array.from({length: 20}, (_, k) => pool.verifySignatureSets([set(k, true)], {batchable: true}));
  const bad = pool.verifySignatureSets([set(1, true, {sigLen: 32})], {batchable: true});
  await assert.rejects(bad, /BLST_INVALID_SIZE/);
  assert.ok((await Promise.all(good)).every((x) => x === true));
  await assert.rejects(pool.verifySignatureSets([]), /Empty/);
  // 4. verifyOnMainThread calls while the pool is saturated
  const load = Array.from({length: 4000}, (_, k) => pool.verifySignatureSets([set(k, true)], {batchable: true}));
  const main = [];
  for (let k = 0; k < 50; k++) main.push(pool.verifySignatureSets([set(k, k % 5 !== 0), set(k + 1, true)], {verifyOnMainThread: true}));
  await assert.rejects(pool.verifySignatureSets([set(3, true, {sigLen: 10})], {verifyOnMainThread: true}), /BLST_INVALID_SIZE/);
  gc();
  assert.deepStrictEqual(await Promise.all(main), main.map((_, k) => k % 5 !== 0));
  assert.ok((await Promise.all(load)).every((x) => x === true));
  // 5. same-message extension
  const sm = await pool.verifySignatureSetsSameMessage(
    [0, 1, 2, 3].map((k) => ({publicKey: new Uint8Array(96).fill(1), signature: new Uint8Array(96).fill(k === 2 ? 9 : 5)})),
    new Uint8Array(32).fill(5)
  );
  assert.deepStrictEqual(sm, [true, true, false, true]);
  // 6. the utility exports
  const ctx = pool.ctx;
  assert.strictEqual(typeof addon.deviceName(ctx), "string");
  assert.strictEqual(addon.deviceCount(ctx), 1);
  assert.strictEqual(addon.aggregatePubkeys(ctx, [new Uint8Array(96).fill(1), new Uint8Array(96).fill(2)]).bytes.length, 96);
  assert.deepStrictEqual(pool.loadPubkeys(0, [new Uint8Array(96).fill(1), new Uint8Array(48).fill(2)].slice(0, 1)), [0]);
  assert.strictEqual(addon.hashToG2(ctx, new Uint8Array(32), new Uint8Array(43)).length, 192);
  const ag = pool.aggregateSignatures([[new Uint8Array(96).fill(1), new Uint8Array(96).fill(2)], []]);
  assert.strictEqual(ag.length, 2);
  assert.ok(ag[0].signature && ag[1].signature === null);
  assert.strictEqual(addon.attestationSigningRoots(ctx, new Uint8Array(256), new Uint8Array(32)).length, 64);
  assert.strictEqual(addon.sign(ctx, new Uint8Array(64), new Uint8Array(64)).length, 192);
  assert.strictEqual(addon.skToPk(ctx, new Uint8Array(96)).length, 288);
  assert.throws(() => addon.verifyPacked(ctx, new Uint8Array(4), new Uint32Array(3), new Uint32Array(2)), /verifyPacked/);
  // a descriptor naming bytes outside the arena is an argument error, never a wild read
  await assert.rejects(addon.verifyPacked(ctx, new Uint8Array(8), Uint32Array.from([0, 96, 1, 0, 32, 0, 96]), Uint32Array.from([1, 0]), 0),
                       /status/);
  // 7. close with packages in flight: they settle first, later calls reject
  const tail = Array.from({length: 500}, (_, k) => pool.verifySignatureSets([set(k, true)], {batchable: true}));
  const closing = pool.close();
  await assert.rejects(pool.verifySignatureSets([set(1, true)]), /QUEUE_ERROR_QUEUE_ABORTED/);
  await closing;
  for (const r of await Promise.allSettled(tail)) assert.ok(r.status === "fulfilled" ? r.value === true : /ABORTED/.test(String(r.reason)));
  gc();
  // 8. the single-thread verifier (priority jobs), open/close cycles
  for (let k = 0; k < 3; k++) {
    const st = V.createBlsVerifier({blsVerifyAllMainThread: true}, {addon});
    assert.strictEqual(await st.verifySignatureSets([set(1, true), set(2, true)]), true);
    assert.strictEqual(await st.verifySignatureSets([set(1, false)]), false);
    await assert.rejects(st.verifySignatureSets([set(4, true, {sigLen: 95})]), /BLST_INVALID_SIZE/);
    await st.close();
  }
  gc();
  console.log("napi sanitizer traffic ok");
})().catch((e) => {
  console.error(e);
  process.exit(1);
});
