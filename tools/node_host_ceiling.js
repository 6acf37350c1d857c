"use strict";
/**
 * JS-thread ceiling of the Node drop-in (VERDICT r5 item 1), on the CPU: bench/bench_node.js's
 * call loop -- verifySignatureSets([set], {batchable: true}) per set, intake gated on
 * canAcceptWork -- over BlsGpuVerifier with a mock addon whose packages complete after
 * `--gpu-rate` sets/s of simulated device time (0: at once, on the next macrotask).  With an
 * instant device the rate is what the JS thread alone can feed; the profile
 * (`--cpuprof <file>`, summarised by tools/node_prof_summary.py) says where its time goes.
 *
 * Run: node tools/node_host_ceiling.js [--sets N] [--gpu-rate R] [--slots S] [--max-pending-sigs P]
 *                                      [--cpuprof F]   (VERIFIER=<file> loads another verifier)
 */
const path = require("path");
const V = require(process.env.VERIFIER || path.join(__dirname, "..", "lodestar_amd", "js", "blsGpuVerifier.js"));

function arg(name, def) {
  const i = process.argv.indexOf("--" + name);
  return i > 0 ? process.argv[i + 1] : def;
}
const nSets = Number(arg("sets", 32768 * 40));
const gpuRate = Number(arg("gpu-rate", 0));
const slots = Number(arg("slots", 15));
const cpuprof = arg("cpuprof", null);
const maxPending = Number(arg("max-pending-sigs", 0));
const distinct = 65536;

function fastAddon() {
  let busyUntil = 0;
  return {
    open: () => ({}),
    slots: () => slots,
    reserve() {},
    close() {},
    verifyPacked(ctx, arena, setDesc, jobDesc) {
      const nJobs = jobDesc.length / 2;
      const status = new Uint8Array(nJobs).fill(1);
      const errCode = new Int32Array(nJobs);
      const res = {status, errCode, batchRetries: 0, batchSigsSuccess: setDesc.length / 7, startNs: 0, endNs: 0, workerId: 0};
      if (!gpuRate) return new Promise((r) => setImmediate(() => r(res)));
      const now = Date.now();
      busyUntil = Math.max(busyUntil, now) + (1e3 * setDesc.length) / 7 / gpuRate;
      return new Promise((r) => setTimeout(() => r(res), Math.max(0, busyUntil - now)));
    },
  };
}

async function main() {
  const pool = new V.BlsGpuVerifier({maxPendingSigs: maxPending || undefined}, {addon: fastAddon()});
  const pk = new Uint8Array(96 * 1024);
  const roots = new Uint8Array(32 * distinct);
  const sigs = new Uint8Array(96 * distinct);
  for (let i = 0; i < roots.length; i++) roots[i] = i * 7;
  const sets = new Array(distinct);
  for (let i = 0; i < distinct; i++) {
    const k = i % 1024;
    sets[i] = {
      type: V.SignatureSetType.single,
      pubkey: pk.subarray(96 * k, 96 * k + 96),
      signingRoot: roots.subarray(32 * i, 32 * i + 32),
      signature: sigs.subarray(96 * i, 96 * i + 96),
    };
  }
  function run(n) {
    return new Promise((resolve, reject) => {
      let issued = 0;
      let done = 0;
      const t0 = process.hrtime.bigint();
      const onVerdict = (ok) => {
        if (ok !== true) reject(Error("bad verdict"));
        if (++done === n) resolve(Number(process.hrtime.bigint() - t0) / 1e9);
      };
      const pump = () => {
        while (issued < n && pool.canAcceptWork()) {
          const s = sets[issued++ % distinct];
          pool.verifySignatureSets([s], {batchable: true}).then(onVerdict, reject);
        }
        if (issued < n) setImmediate(pump);
      };
      pump();
    });
  }
  await run(32768 * 4);
  let prof = null;
  if (cpuprof) {
    prof = new (require("inspector").Session)();
    prof.connect();
    await new Promise((r) => prof.post("Profiler.enable", () => prof.post("Profiler.start", r)));
  }
  const s = await run(nSets);
  if (prof) {
    await new Promise((r) =>
      prof.post("Profiler.stop", (err, res) => {
        if (!err) require("fs").writeFileSync(cpuprof, JSON.stringify(res.profile));
        r();
      })
    );
  }
  await pool.close();
  console.log(JSON.stringify({sets: nSets, seconds: s, sets_per_s: nSets / s, us_per_call: (1e6 * s) / nSets, gpu_rate: gpuRate, node_flags: process.execArgv.join(" ")}));
}
main().catch((e) => {
  console.error(e);
  process.exit(1);
});
