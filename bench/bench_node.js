"use strict";
/**
 * Node bench of the drop-in path (BASELINE.json metric, SURVEY.md 8d config D shape): the
 * firehose of single-set gossip attestations driven through BlsGpuVerifier.verifySignatureSets
 * ([set], {batchable: true}) -- the call validateGossipAttestation makes
 * (chain/validation/attestation.ts -> chain.bls.verifySignatureSets) -- with intake gated on
 * canAcceptWork() as the gossip processor gates it (network/processor/index.ts:357-369
 * checkAcceptWork -> chain.blsThreadPoolCanAcceptWork).
 *
 * Inputs: interop keys sk_{i mod 1024} (state-transition/src/util/interop.ts:19-22), messages
 * sha256("lodestar-mi355x" || "node" || i), signatures made on the GPU (addon.sign) before
 * timing; `--packages` distinct 32,768-set slots cycled.  One step = one slot of sets; W
 * untimed steps, then K timed steps: every call's verdict is checked (all valid), the window
 * runs from the first timed call to the last timed verdict.  Prints one JSON line.
 *
 * Run: node bench/bench_node.js [--steps K] [--warmup W] [--sets-per-step N] [--packages P]
 *                               [--max-sigs-per-package M] [--device D]
 */
const crypto = require("crypto");
const path = require("path");
// LSG_VERIFIER_JS: another build of the verifier (A/B runs on one box)
const V = require(process.env.LSG_VERIFIER_JS || path.join(__dirname, "..", "lodestar_amd", "js", "blsGpuVerifier.js"));

function arg(name, def) {
  const i = process.argv.indexOf("--" + name);
  return i > 0 ? Number(process.argv[i + 1]) : def;
}
const steps = arg("steps", 30);
const warmup = arg("warmup", 5);
const perStep = arg("sets-per-step", 32768);
const nPackages = arg("packages", 2);
const maxSigs = arg("max-sigs-per-package", V.DEFAULT_MAX_SIGS_PER_PACKAGE);
const device = arg("device", 0);
const maxPending = arg("max-pending-sigs", 0); // 0: the verifier's default (4 x maxSigsPerPackage)
const N_KEYS = 1024;
const R = BigInt("0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001");

function interopSk(i) {
  // int_le(sha256(int_to_bytes_le(i, 32))) mod r, big-endian 32 bytes (interop.ts:19-22)
  const le = Buffer.alloc(32);
  le.writeUInt32LE(i, 0);
  const h = crypto.createHash("sha256").update(le).digest();
  let x = 0n;
  for (let k = 31; k >= 0; k--) x = (x << 8n) | BigInt(h[k]);
  x %= R;
  const out = Buffer.alloc(32);
  for (let k = 31; k >= 0; k--) {
    out[k] = Number(x & 255n);
    x >>= 8n;
  }
  return out;
}

function msg(i) {
  const b = Buffer.alloc(8);
  b.writeUInt32LE(i >>> 0, 0);
  b.writeUInt32LE(Math.floor(i / 4294967296), 4);
  return crypto.createHash("sha256").update(Buffer.concat([Buffer.from("lodestar-mi355xnode"), b])).digest();
}

async function main() {
  const pool = new V.BlsGpuVerifier({device, maxSigsPerPackage: maxSigs, reserveSets: maxSigs,
                                     maxPendingSigs: maxPending || undefined});
  const addon = pool.addon;
  const t0g = process.hrtime.bigint();
  const sks = Buffer.concat(Array.from({length: N_KEYS}, (_, i) => interopSk(i)));
  const pks = addon.skToPk(pool.ctx, sks);
  const total = perStep * nPackages;
  const msgs = Buffer.concat(Array.from({length: total}, (_, i) => msg(i)));
  const skRep = Buffer.alloc(32 * total);
  for (let i = 0; i < total; i++) sks.copy(skRep, 32 * i, 32 * (i % N_KEYS), 32 * (i % N_KEYS) + 32);
  const sigs = addon.sign(pool.ctx, skRep, msgs);
  const sets = new Array(total);
  for (let i = 0; i < total; i++) {
    const k = i % N_KEYS;
    sets[i] = {
      type: V.SignatureSetType.single,
      pubkey: pks.subarray(96 * k, 96 * k + 96),
      signingRoot: new Uint8Array(msgs.buffer, msgs.byteOffset + 32 * i, 32),
      signature: sigs.subarray(96 * i, 96 * i + 96),
    };
  }
  const genS = Number(process.hrtime.bigint() - t0g) / 1e9;

  // one run of n calls, intake gated on canAcceptWork; returns {seconds, lat (sampled ms)}
  function run(n, offset) {
    return new Promise((resolve, reject) => {
      const lat = [];
      let issued = 0;
      let done = 0;
      let bad = 0;
      const t0 = process.hrtime.bigint();
      const finish = () => {
        if (bad) reject(Error(`${bad} valid sets were not verified`));
        else resolve({seconds: Number(process.hrtime.bigint() - t0) / 1e9, lat});
      };
      // one shared continuation for the unsampled calls; every 16th call carries its own to
      // time its latency
      const onVerdict = (ok) => {
        if (ok !== true) bad++;
        if (++done === n) finish();
      };
      const pump = () => {
        while (issued < n && pool.canAcceptWork()) {
          const i = issued++;
          const s = sets[(offset + i) % total];
          const p = pool.verifySignatureSets([s], {batchable: true});
          if ((i & 15) === 0) {
            const ts = process.hrtime.bigint();
            p.then((ok) => {
              lat.push(Number(process.hrtime.bigint() - ts) / 1e6);
              onVerdict(ok);
            }, reject);
          } else {
            p.then(onVerdict, reject);
          }
        }
        if (issued < n) setImmediate(pump);
      };
      pump();
    });
  }

  // optional CPU profile of the timed run (env LSG_NODE_CPUPROF=<file>), started through the
  // inspector after the GPU context exists: node's --cpu-prof samples with SIGPROF from
  // process start, and the runtime's device initialisation does not survive it
  let prof = null;
  if (process.env.LSG_NODE_CPUPROF) {
    const inspector = require("inspector");
    prof = new inspector.Session();
    prof.connect();
    await new Promise((r) => prof.post("Profiler.enable", () => prof.post("Profiler.start", r)));
  }
  const statsBefore = {...pool.stats};
  await run(perStep * warmup, 0);
  const pk0 = pool.stats.packages;
  const ps0 = pool.stats.packageSigs;
  const timed = await run(perStep * steps, perStep * warmup);
  if (prof) {
    await new Promise((r) =>
      prof.post("Profiler.stop", (err, res) => {
        if (!err) require("fs").writeFileSync(process.env.LSG_NODE_CPUPROF, JSON.stringify(res.profile));
        r();
      })
    );
  }
  const packages = pool.stats.packages - pk0;
  const packageSigs = pool.stats.packageSigs - ps0;
  // unloaded: one call at a time (a lone batchable job waits for the 100 ms buffer timer in
  // the reference's queue; a non-batchable one goes at once)
  const lone = [];
  for (let i = 0; i < 5; i++) {
    const t = process.hrtime.bigint();
    const ok = await pool.verifySignatureSets([sets[i]]);
    if (ok !== true) throw Error("lone set not verified");
    lone.push(Number(process.hrtime.bigint() - t) / 1e6);
  }
  await pool.close();
  const lat = timed.lat.sort((a, b) => a - b);
  const q = (p) => lat[Math.min(lat.length - 1, Math.floor(p * lat.length))];
  lone.sort((a, b) => a - b);
  void statsBefore;
  console.log(
    JSON.stringify({
      sets: perStep * steps,
      seconds: timed.seconds,
      sets_per_s: (perStep * steps) / timed.seconds,
      ms_per_step: (1e3 * timed.seconds) / steps,
      p50_call_latency_ms: q(0.5),
      p99_call_latency_ms: q(0.99),
      p50_lone_call_latency_ms: lone[2],
      packages,
      mean_package_sets: packageSigs / Math.max(packages, 1),
      max_sigs_per_package: maxSigs,
      pool_size: pool.poolSize,
      max_pending_sigs: pool.maxPendingSigs,
      node_flags: process.execArgv.join(" "),
      input_generation_s: genS,
      node: process.version,
    })
  );
}

main().catch((e) => {
  console.error(e && e.stack ? e.stack : e);
  process.exit(1);
});
