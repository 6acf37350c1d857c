#!/usr/bin/env python3
"""Benchmark: BLS signature sets verified/sec on MI355X (BASELINE.json metric), through the
drop-in jobs path (lsg_submit_jobs / lsg_wait_jobs: the C ABI BlsGpuVerifier calls).

One step = one work package per GPU (BlsWorkReq[]: the jobs one worker would get,
packages/beacon-node/src/chain/bls/multithread/worker.ts:30-106), run the way the Node host
runs it: the C side copies every input byte from host memory into pinned staging, draws
fresh RLC randomizers from the OS CSPRNG (getrandom), plans the bucket MSM, launches every
stage, and the wait applies the reference's verdict rules; the bench then checks every job's
verdict.  Nothing is pre-staged on the device and no per-package work happens outside the
timed region except building the host-side job arrays (PreparedJobs, once per distinct
package) -- what the Node host does when it serialises sets.

Workloads:
  jobs         config D shape (default, the headline): 32,768 single-pubkey gossip sets per
               package = one mainnet slot of unaggregated attestations per GPU (weak scaling:
               at 8 GPUs the node takes 8 slots' worth per step); one batchable job per set
  block        config C: 64 blocks per package, each one non-batchable job of 128 aggregate
               sets of 440-460 signers named by index into the device pubkey table
  sync         config B: 256 sync-committee contributions per package, each one batchable
               job of one 512-signer aggregate set
  gossip       config A: one job of 128 single sets per package (latency-bound)
  adversarial  config E: the jobs workload with 1% of the sets corrupted over the five kinds
               (wrong message, flipped x bit, truncated, non-subgroup point, infinity); every
               verdict is checked against its expected value
  committees   config D mainnet-shaped: the jobs package with the messages a slot's attesters
               actually sign -- 64 distinct AttestationData (one per committee of 512, before
               EIP-7549 moved the committee index out of it), arrivals interleaved over the
               committees; every set has its own key (no duplicate sets)
Keys: interop keys sk_{v mod 1024} (state-transition/src/util/interop.ts:19-22); messages
sha256(b"lodestar-mi355x" || workload || i); signatures made on the GPU before timing.

N > 1 (torch.distributed.run, one process per GPU): every rank resolves its package with the
node check of SURVEY.md 8e -- its partial (lsg_jobs_partial) is all-gathered over RCCL, the
product of the N partials gets one final exponentiation (lsg_final_*), and the ticket is
resolved with that verdict (lsg_wait_jobs_node).
Launch: python bench.py [--gpus N --steps K --warmup W --workload jobs]
"""
import argparse
import collections
import hashlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
# Hardware queues: the library sets GPU_MAX_HW_QUEUES itself (LSG_HW_QUEUES, default 16) before
# its first HIP call (lsg_init_devices, as in a Node process).  One GPU: nothing is set here,
# so the run measures the library's own setting.  Several ranks, and the one-rank rehearsal of
# the node protocol: torch initialises HIP before the library, so the same value is set here
# first (without it the rehearsal ran at the box's 4 queues against the plain run's 16).
if int(os.environ.get("WORLD_SIZE", "1")) > 1 or os.environ.get("LSG_BENCH_REHEARSE") == "1":
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("LSG_HW_QUEUES", "16")
sys.path.insert(0, ROOT)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
METRIC = "BLS signature sets verified/sec (whole node) at 1/2/4/8 MI355X; p50 batch latency"
N_KEYS = 1024
N_VALIDATORS = 1 << 20  # block workload: the pubkey table's rows (~1M validators, mainnet 2023)


def interop_sk(i):
    return int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R_ORDER


def msg(tag, i):
    return hashlib.sha256(b"lodestar-mi355x" + tag + i.to_bytes(8, "little")).digest()


class Workload:
    """Builds the distinct packages of one workload: .packages = list of (jobs, expected)
    with expected = per-job (status, code) or None (all valid)."""

    def __init__(self, ctx, name, rank, sets_per_step, n_packages, blocks=64, validators=N_VALIDATORS):
        from lodestar_amd._native import PkIndices
        self.name = name
        sks = [interop_sk(i) for i in range(N_KEYS)]
        pks = ctx.sk_to_pk(sks)
        self.packages = []
        tag = name.encode()
        self.msgs_per_set = 1.0
        if name in ("jobs", "adversarial", "gossip", "single", "committees"):
            n = 128 if name == "gossip" else (1 if name == "single" else sets_per_step)
            for p in range(n_packages):
                base = (rank * n_packages + p) * n
                if name == "committees":  # set i: key i mod 1024, committee (i + i // 1024) mod 64
                    msgs = [msg(tag, (rank * n_packages + p) * 64 + (i + i // N_KEYS) % 64) for i in range(n)]
                    self.msgs_per_set = min(64, n) / n
                else:
                    msgs = [msg(tag, base + i) for i in range(n)]
                sigs = ctx.sign([sks[(base + i) % N_KEYS] for i in range(n)], msgs)
                sets = [([pks[(base + i) % N_KEYS]], msgs[i], sigs[i]) for i in range(n)]
                if name == "gossip":
                    self.packages.append(([(sets, 1)], None))
                elif name == "single":  # verifyOnMainThread / BlsSingleThreadVerifier: one set, one verify
                    self.packages.append(([(sets, 0)], None))
                elif name in ("jobs", "committees"):
                    self.packages.append(([([s], 1) for s in sets], None))
                else:
                    self.packages.append(self._corrupt(ctx, sets, seed=base))
            self.sets_per_package = n
            self.pks_per_set = 1.0
        elif name == "block":
            # a mainnet-sized index2pubkey: N_VALIDATORS rows, validator v holding key v mod
            # 1024, each attestation's signers a random committee subset of them --
            # the table gathers are scattered over ~112 MB of HBM as on mainnet
            import random as _random
            table = [pks[v % N_KEYS] for v in range(validators)]
            errs = ctx.pubkey_table_set(0, table)
            del table
            if any(errs):
                raise SystemExit("pubkey table load failed")
            per_block = 128
            for p in range(n_packages):
                jobs, npk = [], 0
                for b in range(blocks):
                    idx, agg, msgs = [], [], []
                    for i in range(per_block):
                        g = ((rank * n_packages + p) * blocks + b) * per_block + i
                        size = 440 + (g * 7) % 21
                        ix = _random.Random(g).sample(range(validators), size)
                        idx.append(PkIndices(ix))
                        agg.append(sum(sks[k % N_KEYS] for k in ix) % R_ORDER)
                        msgs.append(msg(tag, g))
                        npk += size
                    sigs = ctx.sign(agg, msgs)
                    jobs.append(([(idx[i], msgs[i], sigs[i]) for i in range(per_block)], 0))  # non-batchable
                self.packages.append((jobs, None))
            self.sets_per_package = blocks * per_block
            self.pks_per_set = npk / (blocks * per_block)
        elif name == "sync":
            errs = ctx.pubkey_table_set(0, pks)
            if any(errs):
                raise SystemExit("pubkey table load failed")
            contributions, size = 256, 512
            for p in range(n_packages):
                ixs, aggs, ms = [], [], []
                for c in range(contributions):
                    g = (rank * n_packages + p) * contributions + c
                    start = (g * 131) % N_KEYS
                    ix = [(start + j) % N_KEYS for j in range(size)]
                    ixs.append(ix)
                    aggs.append(sum(sks[k] for k in ix) % R_ORDER)
                    ms.append(msg(tag, g))
                sigs = ctx.sign(aggs, ms)  # one signing launch per package
                self.packages.append(([([(PkIndices(ixs[c]), ms[c], sigs[c])], 1) for c in range(contributions)], None))
            self.sets_per_package = contributions
            self.pks_per_set = float(size)
        else:
            raise SystemExit(f"unknown workload {name}")

    @staticmethod
    def _non_subgroup_sig():
        """A 96-byte compressed point on E2 outside G2, from the committed decode fixtures
        (tests/golden/sig_decode.json: data, not the oracle)."""
        gold = json.load(open(os.path.join(ROOT, "tests", "golden", "sig_decode.json")))
        for c in gold["cases"]:
            if c["err"] == 3 and len(c["sig"]) == 192:
                return bytes.fromhex(c["sig"])
        raise SystemExit("no non-subgroup fixture")

    def _corrupt(self, ctx, sets, seed):
        """1% corrupted, split evenly over the five kinds of SURVEY.md 8d config E with their
        expected outcomes: wrong message -> false; truncated -> BLST_INVALID_SIZE; non-subgroup
        point -> BLST_POINT_NOT_IN_GROUP; infinity -> false; flipped x bit -> the decode error
        Signature.fromBytes gives (lsg_sig_decode; GPU decode parity is pinned by the golden
        decode vectors in tests/test_gpu_parity.py).  Parity of these outcomes with the oracle is
        tested in tests/test_gpu_configs.py (config E)."""
        import random
        rng = random.Random(seed)
        n = len(sets)
        idx = sorted(rng.sample(range(n), max(5, n // 100)))
        out = list(sets)
        exp = [(1, 0)] * n
        nsg = self._non_subgroup_sig()
        flips = []
        for k, i in enumerate(idx):
            pks, m, sig = out[i]
            kind = k % 5
            if kind == 0:
                out[i], exp[i] = (pks, hashlib.sha256(m).digest(), sig), (0, 0)
            elif kind == 1:
                b = bytearray(sig)
                b[40] ^= 1 << (k % 8)
                out[i] = (pks, m, bytes(b))
                flips.append(i)
            elif kind == 2:
                out[i], exp[i] = (pks, m, sig[:32]), (2, 10)
            elif kind == 3:
                out[i], exp[i] = (pks, m, nsg), (2, 3)
            else:
                out[i], exp[i] = (pks, m, bytes([0xC0]) + bytes(95)), (0, 0)
        if flips:
            dec = ctx.sig_decode([out[i][2] for i in flips])
            for i, (_pt, e) in zip(flips, dec):
                exp[i] = (2, e) if e else None
            if any(exp[i] is None for i in flips):  # a flip that still decodes to a G2 point
                raise SystemExit("flipped signature decoded to a subgroup point; change the seed")
        return [([s], 1) for s in out], exp


def host_cores():
    """Host threads this job may use: the box's CPU share (OMP_NUM_THREADS is set to it on the
    GPU box; os.cpu_count() there shows the whole machine), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_baseline_oracle(sets, budget_s=12.0):
    """Reference-semantics CPU path: oracle/c (the C restatement of the oracle, checked against
    it and the golden vectors by tests/test_oracle_c.py) verifying the same workload the way
    the reference's worker pool does -- RLC batches of 16 sets (worker.ts:17,54), one thread
    per host core (poolSize.ts:7) -- on a bounded sample of ~budget_s seconds.  A stand-in for
    the @chainsafe/blst pool, which cannot run here; it runs at ~1.6 ms per set
    and thread against the ~0.9 ms blst note of metrics/metrics/lodestar.ts:427."""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "c", "libbls_cpu.so"))
    lib.cpu_verify_chunks.restype = ctypes.c_int
    lib.cpu_verify_chunks.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]
    cores = host_cores()
    chunk = 16

    def run(k):  # the first k sets of the workload (wrapping), 16-set batches on `cores` threads
        sub = [sets[i % len(sets)] for i in range(k)]
        pk = b"".join(p[0] for p, _, _ in sub)
        m = b"".join(x for _, x, _ in sub)
        sig = b"".join(s for _, _, s in sub)
        nch = -(-k // chunk)
        verdicts = (ctypes.c_int * nch)()
        t0 = time.perf_counter()
        ok = lib.cpu_verify_chunks(pk, m, sig, k, chunk, cores, 0x5EED, verdicts)
        dt = time.perf_counter() - t0
        if ok != nch:
            raise SystemExit(f"cpu baseline: {nch - ok} of {nch} batches failed on valid sets")
        return dt

    k = chunk * cores
    dt = run(k)  # calibration round: one batch per thread
    k = max(k, int(k * budget_s / max(dt, 1e-3)) // (chunk * cores) * chunk * cores)
    dt = run(k)
    return {"value": k / dt, "unit": "sets/s", "cores": cores, "kind": "port",
            "sample": f"{k} single sets of this workload in 16-set RLC batches on {cores} threads "
                      f"(oracle/c, C restatement of the oracle, gcc -O3) in {dt:.1f}s; "
                      f"{1e3 * dt * cores / k:.2f} ms per set and thread"}


def pmc_traffic(kernel, sets_per_launch):
    """HBM bytes per launch of `kernel` from the committed PMC passes (tools/pmc_traffic.py ->
    profiles/rNN_pmc_traffic.json: 2 x FETCH_SIZE + WRITE_SIZE), when they were measured at
    this launch size; None otherwise (PMC counters cannot be read inside the timed run)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    k = d["kernels"].get(kernel)
    if k is None or d.get("sets_per_launch") != sets_per_launch:
        return None
    return k["hbm_bytes_per_dispatch"]


def pmc_alone(kernel, sets_per_launch):
    """The kernel alone on the GPU, from the committed isolation profile (tools/gpu_pmc.sh ->
    tools/pmc_summary.py -> profiles/rNN_pmc_isolation.json: rocprofv3 --pmc serialises the
    dispatches): its average duration and fraction of the mad peak.  The live `achieved`
    above shares the SIMDs with the other packages in flight."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_isolation.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    k = d["kernels"].get(kernel)
    if k is None or d.get("sets_per_launch") != sets_per_launch or "serial_us" not in k:
        return None
    return {"kernel_us": k["serial_us"], "frac": k.get("frac_of_peak_serial"),
            "wave_cycles_per_valu": k.get("wave_cycles_per_valu"), "source": os.path.relpath(files[-1], ROOT)}


def run_node_workload(args):
    """The drop-in path itself: node bench/bench_node.js drives BlsGpuVerifier.verifySignatureSets
    ([set], {batchable: true}) at the config D shape (one 32,768-set slot per step), intake gated
    on canAcceptWork() as the gossip processor gates it; the JS host packs the arena, the addon's
    package threads submit and wait, the verdicts settle every call's promise.  One GPU: the
    verifier of a multi-GPU node opens one context over all of them (lsg_init_devices), which
    `--devices` in the jobs workload measures."""
    import subprocess
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        raise SystemExit("--workload node runs one Node process per node (use --gpus 1)")
    # at least 150 timed steps (~2.5 s): over a 30-step window (~0.6 s) the JIT, the heap
    # growth and single collections moved the rate by +-25 % between runs
    args.steps = max(args.steps or 0, 150)
    # 40 untimed steps: the first Node process on a fresh box ran its first ~10-20 packages
    # 20-30 % slower (1.35-1.53M against 1.86-1.97M for a second run in the same call)
    args.warmup = max(args.warmup, 40)
    cmd = ["node"] + args.node_flags.split() + [os.path.join(ROOT, "bench", "bench_node.js"), "--steps", str(args.steps), "--warmup",
           str(args.warmup), "--sets-per-step", str(args.sets_per_step), "--max-sigs-per-package",
           str(args.node_max_sigs), "--device", str(local), "--max-pending-sigs", str(args.node_max_pending)]
    w0 = time.monotonic_ns()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    w1 = time.monotonic_ns()
    if r.returncode != 0:
        raise SystemExit("bench_node.js failed:\n" + r.stdout[-2000:] + r.stderr[-4000:])
    nb = json.loads(r.stdout.strip().splitlines()[-1])
    cpu = None
    if not args.no_cpu_baseline:
        from lodestar_amd._native import Context
        ctx = Context(local)
        wl = Workload(ctx, "jobs", 0, 4096, 1)
        ctx.close()
        cpu = cpu_baseline_oracle([s for job, _ in wl.packages[0][0] for s in job])
    line = {
        "metric": METRIC, "value": round(nb["sets_per_s"], 1), "unit": "sets/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(nb["ms_per_step"], 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (interop keys, GPU-signed; fresh OS-CSPRNG randomizers per package)",
        "config": {"workload": "drop-in Node host (SURVEY 8d config D shape): BlsGpuVerifier.verifySignatureSets"
                               "([set], {batchable: true}) per single-pubkey gossip set, intake gated on canAcceptWork, "
                               "through the N-API addon's package threads",
                   "sets_per_step_per_gpu": args.sets_per_step, "global_batch": args.sets_per_step,
                   "max_sigs_per_package": nb["max_sigs_per_package"], "parallelism": "shard1", "node": nb["node"],
                   "node_flags": args.node_flags},
        "p50_batch_latency_ms": round(nb["p50_call_latency_ms"], 3),
        "p99_call_latency_ms": round(nb["p99_call_latency_ms"], 3),
        "p50_unloaded_latency_ms": round(nb["p50_lone_call_latency_ms"], 3),
        "packages": nb["packages"], "mean_package_sets": round(nb["mean_package_sets"], 1),
        "timed_window_monotonic_ns": [w0, w1], "roofline": None,
        "roofline_note": "kernel-level roofline: the jobs workload (same kernels, ctypes host)",
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


def _build_record():
    """provenance of the library this run loaded: its manifest (lodestar_amd/build.py) and whether
    the sources in this tree still hash to what it was built from"""
    from lodestar_amd import build as b
    from lodestar_amd import _native
    lib = _native.LIB_PATH
    man = b.read_manifest(lib)
    if man is None:
        return {"lib": os.path.basename(lib), "manifest": None}
    srcs = b.SOURCES + (b.AB_SOURCES if lib == b.AB_OUT else [])
    with open(lib, "rb") as fh:
        so16 = hashlib.sha256(fh.read()).hexdigest()[:16]
    return {"lib": man["lib"], "src_sha256_16": man["src_sha256"][:16], "so_sha256_16": man["so_sha256_16"],
            "so_matches_manifest": so16 == man["so_sha256_16"],
            "tree_matches_manifest": b.source_hash(srcs) == man["src_sha256"], "compiler": man["compiler"],
            "built_utc": man["built_utc"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed packages per GPU (default 30; 10 x depth for the deep small-package workloads, "
                         "so that the timed region is the steady state, not one burst of the pipeline)")
    ap.add_argument("--warmup", type=int, default=5, help="untimed packages per GPU (at least --depth are run)")
    ap.add_argument("--workload", choices=["jobs", "block", "sync", "gossip", "adversarial", "node", "single", "committees"],
                    default="jobs")
    ap.add_argument("--sets-per-step", type=int, default=32768, help="sets per package (jobs / adversarial)")
    ap.add_argument("--depth", type=int, default=None, help="packages in flight per GPU")
    ap.add_argument("--blocks", type=int, default=128, help="block workload: blocks (128-set jobs) per package")
    ap.add_argument("--validators", type=int, default=N_VALIDATORS,
                    help="block workload: pubkey table rows (validator v holds key v mod 1024)")
    ap.add_argument("--packages", type=int, default=None, help="distinct packages cycled through")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--waits", choices=["thread", "inline"], default="thread",
                    help="one GPU: wait each ticket on its own thread (as the Node host) or inline")
    ap.add_argument("--node-max-sigs", type=int, default=32768, help="node workload: maxSigsPerPackage")
    ap.add_argument("--node-max-pending", type=int, default=0, help="node workload: maxPendingSigs (0: default)")
    ap.add_argument("--node-flags", default="--max-old-space-size=4096 --max-semi-space-size=64",
                    help="node workload: node/V8 flags -- the reference's production heap setting (Dockerfile:45 "
                         "NODE_OPTIONS=--max-old-space-size=4096) plus a 64 MB young generation for the verifier's "
                         "per-call promises (INTEGRATION.md)")
    ap.add_argument("--coalesce", type=int, default=None,
                    help="lsg_set_coalesce max sets per package (default: 4096 for gossip / sync, else 0 = off)")
    ap.add_argument("--coalesce-inflight", type=int, default=4, help="launches on the device before packages are held")
    ap.add_argument("--devices", type=int, default=0,
                    help="one process over N GPUs (lsg_init_devices, in-library RCCL exchange: the context "
                         "BlsGpuVerifier({devices}) opens); packages of sets-per-step x N sets")
    ap.add_argument("--devices-same", action="store_true",
                    help="with --devices N: the context's N devices are all this process's GPU (duplicate ids, "
                         "device copies instead of RCCL) -- rehearses the multi-device host path on one GPU")
    args = ap.parse_args()
    if args.workload == "node":
        return run_node_workload(args)
    if args.depth is None:
        args.depth = {"jobs": 6, "adversarial": 5, "block": 4, "sync": 32, "gossip": 64, "single": 1,
                      "committees": 6}[args.workload]
    if args.steps is None:
        args.steps = 10 * args.depth if args.workload in ("gossip", "sync") else 30
    if args.coalesce is None:
        args.coalesce = 4096 if args.workload in ("gossip", "sync") else 0
    if args.packages is None:  # distinct packages cycled (the aggregate workloads are costly to build)
        args.packages = 2 if args.workload == "block" else args.depth + 1

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # LSG_BENCH_REHEARSE=1: a multi-rank rehearsal on a one-GPU box -- every rank on device 0,
    # the partials exchanged over gloo through host memory (RCCL refuses two ranks on one GPU).
    # The rank protocol, data split, barriers and max-over-ranks timing are the real ones.
    rehearse = os.environ.get("LSG_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    dist = None
    if world > 1 or rehearse:  # (a one-rank rehearsal runs the node protocol too)
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            # the per-package all-gather of 576-byte partials must not queue behind the
            # package kernels in flight: RCCL on a high-priority stream
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), pg_options=opts)

    from lodestar_amd._native import Context, PreparedJobs
    # multi-rank: node verdicts awaited this many exchanges late (run()); the threaded loop lets
    # NODE_LAG more packages than --depth wait for their node verdicts
    NODE_LAG = int(os.environ.get("LSG_BENCH_NODE_LAG", "2"))
    # packages whose per-kernel HIP-event times are read back in the timed region (the
    # reading costs host time: a sample, not every package of a 640-step small-package run)
    KT_SAMPLE = 30
    t_start = time.perf_counter()

    def progress(what):  # (stderr: a long input generation or reservation is not a hang)
        print(f"[bench {time.perf_counter() - t_start:7.1f} s] {what}", file=sys.stderr, flush=True)

    n_dev = max(args.devices, 1)
    if args.devices:
        if world > 1:
            raise SystemExit("--devices runs one process over several GPUs (no torch.distributed launch)")
        ctx = Context(devices=[local] * args.devices if args.devices_same else list(range(args.devices)))
    else:
        ctx = Context(local)
    progress("context open; generating inputs")
    wl = Workload(ctx, args.workload, rank, args.sets_per_step * n_dev, args.packages, blocks=args.blocks,
                  validators=args.validators)
    progress("inputs generated")
    prepared = [PreparedJobs(jobs) for jobs, _ in wl.packages]
    n_sets = wl.sets_per_package
    max_pks = int(n_sets * wl.pks_per_set) + 1
    # coalesced launches hold up to `depth` packages: slots sized for that
    co = args.depth if args.coalesce and n_sets <= args.coalesce else 1
    # (multi-rank: NODE_LAG more packages wait for their node verdicts with their GPU work done)
    ctx.reserve(n_sets * co, max_pks * co, 32 * n_sets * co, n_slots=args.depth + 1 + (NODE_LAG if world > 1 or rehearse else 0))
    if args.coalesce:
        ctx.set_coalesce(args.coalesce, args.coalesce_inflight)
    progress("slots reserved")

    import numpy as np

    def verdict_ok(k, res, n_jobs):
        st = np.frombuffer(res, dtype=np.int32, count=2 * n_jobs).reshape(-1, 2)
        exp = wl.packages[k][1]
        if exp is None:
            return bool((st[:, 0] == 1).all())
        e = np.array([[s, c if s == 2 else 0] for s, c in exp], dtype=np.int32)
        got = st.copy()
        got[got[:, 0] != 2, 1] = 0
        return bool((got == e).all())

    xstream = []  # the exchange's own high-priority torch stream (created on first use)

    def gather_node(t):
        """all-gather the 576-byte partials of one package over RCCL, device-resident: the
        library copies its partial into the collective's send buffer and reads the gathered
        partials from its receive buffer (no host round trip); -> node verdict ticket.
        Torch's side of the exchange (the collective's stream waits, the gloo copies) runs on a
        high-priority stream of its own: on torch's default stream, which shares a hardware
        queue with some of the library's package streams, each of those steps queued behind
        another package's kernels (8 ms of host time per package in the round-5 rehearsal)."""
        import torch
        if not xstream:
            xstream.append(torch.cuda.Stream(device=f"cuda:{local}", priority=-1))
        with torch.cuda.stream(xstream[0]):
            send = torch.empty(576, dtype=torch.uint8, device=f"cuda:{local}")
            recv = torch.empty(world * 576, dtype=torch.uint8, device=f"cuda:{local}")
            c0 = time.perf_counter()
            ctx.jobs_partial_device(t, send.data_ptr())
            c1 = time.perf_counter()
            if rehearse:  # gloo: through host memory (the export above is complete; no device sync)
                parts = [torch.empty(576, dtype=torch.uint8) for _ in range(world)]
                dist.all_gather(parts, send.cpu())
                recv.copy_(torch.cat(parts))
            else:
                dist.all_gather_into_tensor(recv, send)
            xstream[0].synchronize()  # the gathered bytes are complete
        node_ms["partial"] += (c1 - c0) * 1e3
        node_ms["gather"] += (time.perf_counter() - c1) * 1e3
        node_ms["n"] += 1
        ft = ctx.final_submit_device(recv.data_ptr(), world)
        if ft is None:
            raise SystemExit("final-exponentiation entries exhausted")
        return ft

    stats_acc = collections.Counter()
    node_ms = collections.Counter()  # host time per node check: partial ready, all-gather, node FE + wait
    submit_wall = []  # wall time of each lsg_submit_jobs call (lock wait + staging + enqueue)

    def run(n_pkgs, depth, capture=False, seq0=0):
        """n_pkgs packages, `depth` in flight; returns per-package submit->verdict latencies and
        (capture) per-package HIP-event kernel times"""
        if dist is None and args.waits == "thread":
            return run_threaded(n_pkgs, depth, capture)
        if dist is not None:
            return run_node(n_pkgs, depth, capture)
        lat, times = [], []
        pend = collections.deque()
        done = 0
        seq = seq0

        def submit():
            nonlocal seq
            k = seq % len(prepared)
            t0 = time.perf_counter()
            t = ctx.submit_jobs(prepared[k])
            submit_wall.append(time.perf_counter() - t0)
            if t is None:
                raise SystemExit("pipeline slots exhausted: lower --depth")
            pend.append((t, k, time.perf_counter()))
            seq += 1

        def finish(t, k, t_sub, res, st):
            nonlocal done
            lat.append(time.perf_counter() - t_sub)
            if not verdict_ok(k, res, t[1]):
                raise SystemExit(f"rank {rank}: package {k} verdicts differ from the expected ones")
            stats_acc.update({"batch_retries": st["batch_retries"], "n_final_exps": st["n_final_exps"],
                              "submit_us": st["submit_us"], "packages": 1})
            if capture and len(times) < KT_SAMPLE:
                times.append(ctx.last_kernel_times())
            done += 1

        # node checks are pipelined: package k's partial is exchanged and its node
        # final exponentiation launched, then package k+1's, ...; a node verdict is awaited
        # NODE_LAG exchanges later, so the host never idles on one final exponentiation while
        # the GPU runs the packages behind it.  Every rank exchanges in submission order.
        fins = collections.deque()

        def resolve_node():
            t, k, t_sub, ft = fins.popleft()
            c2 = time.perf_counter()
            node_ok = ctx.final_wait(ft)
            c3 = time.perf_counter()
            res, st = ctx.wait_jobs_node(t, 1 if node_ok else 0, raw=True)
            node_ms["final"] += (c3 - c2) * 1e3
            node_ms["resolve"] += (time.perf_counter() - c3) * 1e3
            finish(t, k, t_sub, res, st)

        while len(pend) < min(depth, n_pkgs):
            submit()
        while pend or fins:
            if pend:
                t, k, t_sub = pend.popleft()
                if dist is not None:
                    fins.append((t, k, t_sub, gather_node(t)))
                    if len(fins) > NODE_LAG or not pend:
                        resolve_node()
                else:
                    res, st = ctx.wait_jobs(t, raw=True)
                    finish(t, k, t_sub, res, st)
            else:
                resolve_node()
            while seq - seq0 < n_pkgs and len(pend) < depth and len(pend) + len(fins) < depth + NODE_LAG:
                submit()
        return lat, times

    def run_node(n_pkgs, depth, capture):
        """Multi-rank: the main thread submits, an exchange thread takes the
        packages in submission order (every rank alike: the collectives' order) through partial
        -> RCCL all-gather -> node final exponentiation, and a resolver thread waits each node
        verdict and resolves the package -- host work overlaps the GPU as in the one-GPU
        threaded path.  depth packages execute; NODE_LAG more may wait for their verdicts."""
        import queue
        import threading
        import torch
        lat, times = [], []
        room = threading.Semaphore(depth + NODE_LAG)
        exq, rq = queue.Queue(), queue.Queue()
        failed = []

        def guard(fn):
            def body():
                try:
                    torch.cuda.set_device(local)
                    fn()
                except BaseException as e:  # surface in the main thread, never hang it
                    failed.append(e)
                    for _ in range(n_pkgs + depth + NODE_LAG):
                        room.release()
                        rq.put(None)
            return body

        def exchanger():
            for _ in range(n_pkgs):
                t, k, t_sub = exq.get()
                rq.put((t, k, t_sub, gather_node(t)))

        def resolver():
            for _ in range(n_pkgs):
                item = rq.get()
                if item is None:
                    return
                t, k, t_sub, ft = item
                c2 = time.perf_counter()
                node_ok = ctx.final_wait(ft)
                c3 = time.perf_counter()
                res, st = ctx.wait_jobs_node(t, 1 if node_ok else 0, raw=True)
                node_ms["final"] += (c3 - c2) * 1e3
                node_ms["resolve"] += (time.perf_counter() - c3) * 1e3
                lat.append(time.perf_counter() - t_sub)
                if not verdict_ok(k, res, t[1]):
                    raise SystemExit(f"rank {rank}: package {k} verdicts differ from the expected ones")
                stats_acc.update({"batch_retries": st["batch_retries"], "n_final_exps": st["n_final_exps"],
                                  "submit_us": st["submit_us"], "packages": 1})
                if capture and len(times) < KT_SAMPLE:
                    times.append(ctx.last_kernel_times())
                room.release()

        threads = [threading.Thread(target=guard(f), daemon=True) for f in (exchanger, resolver)]
        for th in threads:
            th.start()
        for seq in range(n_pkgs):
            room.acquire()
            if failed:
                break
            k = seq % len(prepared)
            t0 = time.perf_counter()
            t = ctx.submit_jobs(prepared[k])
            submit_wall.append(time.perf_counter() - t0)
            if t is None:
                raise SystemExit("pipeline slots exhausted: lower --depth")
            exq.put((t, k, time.perf_counter()))
        for th in threads:
            th.join()
        if failed:
            raise failed[0]
        return lat, times

    def run_threaded(n_pkgs, depth, capture):
        """One GPU, no collective: each ticket is waited on its own thread (as the Node host's
        libuv pool does), so a package in its fallback phases never holds back the submission
        of the next ones (the C side releases its lock while a fallback phase runs)."""
        from concurrent.futures import ThreadPoolExecutor
        lat, times = [], []

        def wait(t, k, t_sub):
            res, st = ctx.wait_jobs(t, raw=True)
            return time.perf_counter() - t_sub, k, t, res, st

        with ThreadPoolExecutor(max_workers=depth) as ex:
            inflight = collections.deque()
            seq = 0

            def submit():
                nonlocal seq
                k = seq % len(prepared)
                t0 = time.perf_counter()
                t = ctx.submit_jobs(prepared[k])
                submit_wall.append(time.perf_counter() - t0)
                if t is None:
                    raise SystemExit("pipeline slots exhausted: lower --depth")
                inflight.append(ex.submit(wait, t, k, time.perf_counter()))
                seq += 1

            while seq < min(depth, n_pkgs):
                submit()
            while inflight:
                dt, k, t, res, st = inflight.popleft().result()
                lat.append(dt)
                if not verdict_ok(k, res, t[1]):
                    raise SystemExit(f"rank {rank}: package {k} verdicts differ from the expected ones")
                stats_acc.update({"batch_retries": st["batch_retries"], "n_final_exps": st["n_final_exps"],
                                  "submit_us": st["submit_us"], "packages": 1})
                if capture and len(times) < KT_SAMPLE:
                    times.append(ctx.last_kernel_times())
                if seq < n_pkgs:
                    submit()
        return lat, times

    def barrier():
        if dist is not None:
            dist.barrier()

    run(max(args.warmup, args.depth), args.depth)
    progress("warmup done")
    allocs0 = ctx.allocation_count()
    stats_acc.clear()
    barrier()
    cpu0 = os.times()
    t0 = time.perf_counter()
    w0 = time.monotonic_ns()  # CLOCK_MONOTONIC: the clock of rocprofv3's API/kernel timestamps
    submit_wall.clear()
    lat, ktimes = run(args.steps, args.depth, capture=True)
    submit_wall_timed = sorted(submit_wall)
    barrier()
    elapsed = time.perf_counter() - t0
    w1 = time.monotonic_ns()
    cpu1 = os.times()
    host_cpu = (cpu1.user - cpu0.user + cpu1.system - cpu0.system) / max(elapsed, 1e-9)
    allocs = ctx.allocation_count() - allocs0
    if dist is not None:
        import torch
        te = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearse else f"cuda:{local}")
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        elapsed = float(te.item())
    # unloaded latency: one package at a time, each alone on the GPU
    lat1, _ = run(3, 1)

    # kernel-level roofline for the dominant kernel, from HIP events recorded on the streams
    # the kernels ran on, averaged over the timed packages
    opc = json.load(open(os.path.join(ROOT, "bench", "opcount.json")))
    probe_fp, _probe_mad = ctx.probe_fp_mul_rate()
    peak_mad = ctx.probe_mad_peak()  # measured v_mad_u64_u32 issue rate of this GPU (k_probe_mad)
    agg, calls = {}, {}
    for pkg_times in ktimes:
        for name, ms in pkg_times:
            agg[name] = agg.get(name, 0.0) + ms / len(ktimes)
            calls[name] = calls.get(name, 0) + 1 / len(ktimes)
    mk = os.environ.get("LSG_MILLER_K", "4")
    accum_key = f"miller_accum{mk}_per_set" if f"miller_accum{mk}_per_set" in opc["stage_fp_muls"] \
        else "miller_accum2_per_set"
    stage_of = {"k_miller_accum": [accum_key], "k_miller_lines": ["miller_lines"],
                "k_miller_fused": ["miller_fused_per_set"], "k_sig_subgroup": ["sig_subgroup"],
                "k_sig_decode": ["sig_decode"], "k_pk_scale": ["pk_scale"], "k_h2c_map": ["hash_map"]}
    per_set = {k: v for k, v in agg.items() if k in stage_of and k != "k_h2c_map"}
    dom = max(per_set, key=per_set.get) if per_set else "k_miller_fused"
    # one launch covers the package's sets
    muls = sum(opc["stage_fp_muls"][st] for st in stage_of[dom]) * (n_sets // n_dev)  # device 0's launch
    achieved = muls * opc["mads_per_fp_mul"] / (agg[dom] / max(calls[dom], 1) * 1e-3) / 1e12
    peak = peak_mad / 1e12
    roof = {"bound": "valu", "kernel": dom, "achieved": round(achieved, 3), "peak": round(peak, 3),
            "unit": "Tmad/s (v_mad_u64_u32)", "frac": round(achieved / peak, 4),
            "traffic": pmc_traffic(dom, n_sets // n_dev), "alone": pmc_alone(dom, n_sets // n_dev),
            "kernel_ms": round(agg[dom] / max(calls[dom], 1), 3), "work_per_launch_fp_muls": muls}
    total_sets = n_sets * world * args.steps  # (n_sets spans all devices of a --devices context)
    value = total_sets / elapsed
    # whole-path work per set: the per-set stages with the bucket-MSM signature sum (groups of
    # >= 256 sets) plus the package group's share of its per-group stages, plus one G1
    # addition per extra signer of an aggregate set
    # the RLC group a set is verified in: the package group (block bodies: the package's
    # non-batchable jobs as one merged group, lsg_host.hip nb_merge_on); a coalesced launch's
    # sub-package; a lone set
    group = n_sets if args.workload in ("jobs", "adversarial", "committees", "block") else \
        (n_sets if args.coalesce else 1)
    if group >= 256:  # bucket MSM, 8-bit windows (lsg_host.hip plan_phase, msm_window_bits)
        per_set_muls = opc["batched_single_set_msm_fp_muls"] + opc["per_batch_msm_fp_muls"] / group
    elif group >= 48:  # 4-bit windows
        per_set_muls = opc["batched_single_set_msm4_fp_muls"] + opc["per_batch_msm4_fp_muls"] / group
    elif group >= 4:  # 2-bit windows
        per_set_muls = opc["batched_single_set_msm2_fp_muls"] + opc["per_batch_msm2_fp_muls"] / group
    else:
        per_set_muls = opc["batched_single_set_fp_muls"] + opc["per_batch_fp_muls"] / group
    fused = os.environ.get("LSG_MILLER_FUSED", "1") != "0"
    sf = opc["stage_fp_muls"]
    per_set_muls += (sf["miller_fused_per_set"] if fused else sf["miller_lines"] + sf[accum_key]) \
        - sf["miller_multi2_per_set"]
    # extra signers: the shipped library's fused gather + mixed-addition fold (k_pk_agg_seg,
    # 12 M per key); the batch-affine tree only in the A/B build with LSG_AGG_TREE=1
    tree = (os.environ.get("LSG_AGG_TREE") == "1" and "_ab" in os.environ.get("LSG_LIB", "")
            and wl.pks_per_set * n_sets >= 32768)
    per_set_muls += (wl.pks_per_set - 1) * opc["aggregate_tree_extra_per_pubkey_fp_muls" if tree else
                                                "aggregate_extra_per_pubkey_fp_muls"]
    per_set_muls -= (1.0 - wl.msgs_per_set) * sf["hash_map"]  # hash_to_G2 once per distinct message
    if os.environ.get("LSG_MSG_AGG", "1") != "0":  # and one Miller pair per distinct message
        per_set_muls -= (1.0 - wl.msgs_per_set) * (sf["miller_fused_per_set"] if fused else sf["miller_multi2_per_set"])
    node_mads = value * per_set_muls * opc["mads_per_fp_mul"]
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            if args.workload in ("jobs", "adversarial", "gossip", "single", "committees"):
                sets = [s for job, _ in wl.packages[0][0] for s in job]
                if args.workload == "adversarial":
                    sets = [s for (job, _), e in zip(wl.packages[0][0], wl.packages[0][1]) if e == (1, 0) for s in job]
                cpu = cpu_baseline_oracle(sets)
            else:  # aggregate workloads: the CPU path gets the aggregated keys for free (favours the CPU)
                from lodestar_amd._native import PkIndices  # noqa: F401
                sub = [s for job, _ in wl.packages[0][0] for s in job][:256]
                cpu = cpu_baseline_oracle([([ctx.aggregate_pubkeys(p)[0]], m, sg) for p, m, sg in sub])
                cpu["sample"] += "; pubkey aggregation (main thread in the reference) excluded"
        desc = {
            "jobs": "firehose (SURVEY 8d config D): one mainnet slot of unaggregated attestations per GPU -- "
                    "single-pubkey gossip sets, one batchable job each, through lsg_submit_jobs/lsg_wait_jobs",
            "adversarial": "adversarial (SURVEY 8d config E): the firehose package with 1% corrupted sets, "
                           "batch failure + chunk/per-job retry, every verdict checked",
            "block": f"block-body (SURVEY 8d config C): {args.blocks} blocks per package, each a non-batchable job of 128 "
                     "aggregate sets of 440-460 random signers named by index into a device pubkey table of --validators rows",
            "sync": "sync-committee contributions (SURVEY 8d config B): 256 batchable jobs per package, each one "
                    "512-signer aggregate set (keys by index)",
            "gossip": "gossip-128 (SURVEY 8d config A): one batchable job of 128 single sets per package",
            "single": "one set per call (verifyOnMainThread / BlsSingleThreadVerifier, maybeBatch.ts:34-38 verify): "
                      "latency of a lone verification",
            "committees": "firehose, mainnet-shaped messages (SURVEY 8d config D): one slot of unaggregated "
                          "attestations per GPU signing 64 distinct AttestationData (committees of 512, interleaved), "
                          "one batchable job per set, hash_to_G2 once per distinct message",
        }[args.workload]
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "sets/s", "n_gpus": world * n_dev, "steps": args.steps,
            "warmup": max(args.warmup, args.depth), "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (interop keys, GPU-signed; fresh OS-CSPRNG randomizers per package)",
            "config": {"workload": desc, "sets_per_step_per_gpu": n_sets // n_dev, "global_batch": n_sets * world,
                       "jobs_per_package": len(wl.packages[0][0]), "pubkeys_per_set": round(wl.pks_per_set, 1),
                       "keys": N_KEYS, "validators": args.validators if args.workload == "block" else None,
                       "parallelism": (f"devices{args.devices}x{local} (one context, one GPU: duplicate ids)" if args.devices_same
                                       else f"devices{args.devices} (one context, RCCL exchange)") if args.devices else f"shard{world}"},
            "p50_batch_latency_ms": round(1e3 * statistics.median(lat), 3),
            "p50_unloaded_latency_ms": round(1e3 * statistics.median(lat1), 3),
            "pipeline_depth": args.depth, "distinct_packages": len(prepared),
            "coalesce": {"max_sets": args.coalesce, "inflight": args.coalesce_inflight} if args.coalesce else None,
            "allocations_in_timed_region": allocs, "timed_window_monotonic_ns": [w0, w1],
            "batch_retries": stats_acc["batch_retries"], "final_exps": stats_acc["n_final_exps"],
            # (coalesced launches: every ticket reports its launch's count, lodestar_bls.h lsg_set_coalesce;
            # the sum over tickets counts a launch once per sub-package)
            "final_exps_counting": "per launch, once per ticket" if args.coalesce else "per package",
            "host_submit_ms_per_package": round(stats_acc["submit_us"] / max(stats_acc["packages"], 1) / 1e3, 3),
            "submit_call_ms_p50_max": [round(1e3 * statistics.median(submit_wall_timed), 3),
                                       round(1e3 * submit_wall_timed[-1], 3)],
            "host_cpu_cores_busy": round(host_cpu, 2),  # this process's CPU time / timed wall time
            "node_check_host_ms_per_package": ({k: round(v / node_ms["n"], 3) for k, v in node_ms.items() if k != "n"}
                                               if node_ms["n"] else None),
            "roofline": roof,
            "whole_path_mad_frac": round(node_mads / (peak_mad * world * n_dev), 4),
            "kernel_ms": {k: round(v, 3) for k, v in agg.items()},
            "probe_lane_fp_mul_per_s": probe_fp,
            "cpu_baseline": cpu,
            "build": _build_record(),
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
