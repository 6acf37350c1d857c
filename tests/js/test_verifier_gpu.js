"use strict";
/**
 * BlsGpuVerifier through the real N-API addon on an MI355X (driven by
 * tests/test_gpu_parity.py::test_node_host_on_gpu, which writes the input file with
 * oracle-made sets and expected results).  Restates test/e2e/chain/bls/multithread.test.ts:
 * 25-103 against the GPU: 8 x 3 valid sets (sync, async, batchable) -> true; a 32-byte zero
 * signature rejects with BLST_INVALID_SIZE and does not poison co-batched jobs.
 * Run: node tests/js/test_verifier_gpu.js <cases.json>
 */
const assert = require("assert");
const fs = require("fs");
const path = require("path");
const V = require(path.join(__dirname, "..", "..", "lodestar_amd", "js", "blsGpuVerifier.js"));

const hex = (s) => Uint8Array.from(Buffer.from(s, "hex"));
const cases = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
const toSet = (c) =>
  c.pks.length === 1
    ? {type: V.SignatureSetType.single, pubkey: hex(c.pks[0]), signingRoot: hex(c.msg), signature: hex(c.sig)}
    : {type: V.SignatureSetType.aggregate, pubkeys: c.pks.map(hex), signingRoot: hex(c.msg), signature: hex(c.sig)};
const sleep = (ms) => new Promise((r) => setTimeout(r, ms));

(async () => {
  const pool = new V.BlsGpuVerifier({seed: 7});
  const sets = cases.valid.map(toSet);
  // multithread.test.ts:72-86
  assert.deepStrictEqual(await Promise.all(Array.from({length: 8}, () => pool.verifySignatureSets(sets))), Array(8).fill(true));
  const ps = [];
  for (let i = 0; i < 8; i++) {
    ps.push(pool.verifySignatureSets(sets, {batchable: true}));
    await sleep(5);
  }
  assert.deepStrictEqual(await Promise.all(ps), Array(8).fill(true));
  // multithread.test.ts:88-103
  const invalidSet = Object.assign({}, sets[0], {signature: new Uint8Array(32)});
  const pBad = pool.verifySignatureSets([invalidSet], {batchable: true});
  const pGood = Array.from({length: 8}, () => pool.verifySignatureSets(sets, {batchable: true}));
  await assert.rejects(pBad, /BLST_INVALID_SIZE/);
  assert.deepStrictEqual(await Promise.all(pGood), Array(8).fill(true));
  // wrong message -> false; aggregate set -> true; main-thread path
  assert.strictEqual(await pool.verifySignatureSets([sets[0], toSet(cases.wrong_message)]), false);
  assert.strictEqual(await pool.verifySignatureSets([toSet(cases.aggregate)]), true);
  assert.strictEqual(await pool.verifySignatureSets(sets, {verifyOnMainThread: true}), true);
  // per-set verdicts for one message
  const sm = cases.same_message;
  const got = await pool.verifySignatureSetsSameMessage(
    sm.sets.map((s) => ({publicKey: hex(s.pk), signature: hex(s.sig)})), hex(sm.msg));
  assert.deepStrictEqual(got, sm.expected);
  // parity exports
  const agg = pool.addon.aggregatePubkeys(pool.ctx, cases.aggregate.pks.map(hex));
  assert.strictEqual(agg.errCode, 0);
  assert.strictEqual(Buffer.from(agg.bytes).toString("hex"), cases.aggregate_pk);
  const h = pool.addon.hashToG2(pool.ctx, hex(cases.h2c.msg), Buffer.from(cases.h2c.dst, "latin1"));
  assert.strictEqual(Buffer.from(h).toString("hex"), cases.h2c.out);
  // signers by index into the device pubkey table (SURVEY 8f(1))
  const aggPks = cases.aggregate.pks.map(hex);
  assert.deepStrictEqual(pool.loadPubkeys(100, aggPks), Array(aggPks.length).fill(0));
  const ix = Uint32Array.from(aggPks.map((_, k) => 100 + k));
  const byIndex = {type: V.SignatureSetType.aggregate, pubkeyIndices: ix, signingRoot: hex(cases.aggregate.msg),
                   signature: hex(cases.aggregate.sig)};
  assert.strictEqual(await pool.verifySignatureSets([byIndex, sets[0]], {batchable: true}), true);
  assert.strictEqual(await pool.verifySignatureSets([Object.assign({}, byIndex, {pubkeyIndices: ix.slice(1)})]), false);
  // op-pool signature aggregation (SURVEY 8f(4)) against the oracle's golden fixture
  const gold = JSON.parse(fs.readFileSync(path.join(__dirname, "..", "golden", "aggregate_signatures.json")));
  const g96 = gold.cases.filter((c) => c.sigs[0].length === 192);
  const aggs = pool.aggregateSignatures(g96.map((c) => c.sigs.map(hex)).concat([[]]));
  g96.forEach((c, k) => {
    assert.strictEqual(aggs[k].err, c.err);
    if (c.err === 0) assert.strictEqual(Buffer.from(aggs[k].signature).toString("hex"), c.out);
  });
  assert.strictEqual(aggs[g96.length].err, 101);
  // signing roots (SURVEY 8f(3)) against the oracle's values in the cases file
  const sr = cases.signing_roots;
  const roots = pool.addon.attestationSigningRoots(pool.ctx, hex(sr.data), hex(sr.domain));
  assert.strictEqual(Buffer.from(roots).toString("hex"), sr.roots);
  // the package engine at volume: 4096 single-set batchable gossip calls (one 32-byte secret
  // key per set), 1% with a wrong message; gated on canAcceptWork like the gossip processor
  const n = 4096;
  const sks = Buffer.alloc(32 * n);
  const msgs = Buffer.alloc(32 * n);
  for (let i = 0; i < n; i++) {
    sks.writeUInt32BE(i + 1, 32 * i + 28);
    msgs.writeUInt32BE(0x5eed0000 + i, 32 * i);
  }
  const pks = pool.addon.skToPk(pool.ctx, sks);
  const sigs = pool.addon.sign(pool.ctx, sks, msgs);
  const wrong = new Set(Array.from({length: 41}, (_, k) => (k * 97 + 13) % n));
  const vol = [];
  for (let i = 0; i < n; i++) {
    const m = wrong.has(i) ? msgs.subarray(32 * ((i + 1) % n), 32 * ((i + 1) % n) + 32) : msgs.subarray(32 * i, 32 * i + 32);
    vol.push({type: V.SignatureSetType.single, pubkey: pks.subarray(96 * i, 96 * i + 96), signingRoot: m,
              signature: sigs.subarray(96 * i, 96 * i + 96)});
  }
  const pv = [];
  for (let i = 0; i < n; i++) {
    while (!pool.canAcceptWork()) await sleep(1);
    pv.push(pool.verifySignatureSets([vol[i]], {batchable: true}));
  }
  const verdicts = await Promise.all(pv);
  verdicts.forEach((v, i) => assert.strictEqual(v, !wrong.has(i), `set ${i}`));
  assert.ok(pool.stats.packages >= 1 && pool.stats.packageSigs >= n);
  await pool.close();
  console.log("node host on GPU: all checks passed; packages", pool.stats.packages, "sets", pool.stats.packageSigs);
})().catch((e) => {
  console.log("FAIL", e && e.stack);
  process.exit(1);
});
