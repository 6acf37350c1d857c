#!/usr/bin/env python3
"""Benchmark: BLS signature sets verified/sec on MI355X (BASELINE.json metric).

Workload ("epoch firehose"): every GPU verifies a shard of 4096
single-pubkey gossip-attestation sets per step (weak scaling: at 8 GPUs the node covers the
~32k-set mainnet slot).  Keys are the interop keys sk_{v mod 1024}
(packages/state-transition/src/util/interop.ts:19-22), messages sha256(b"lodestar-mi355x" ||
b"firehose" || i), signatures sk*H(m) -- synthetic, generated on the GPU before timing.

One step = the sharded hot path of SURVEY.md 8(e) on inputs already resident in HBM:
  per GPU  lsg_batch_submit/wait: decode + subgroup-check signatures, decode pubkeys,
           hash_to_G2, 64-bit RLC scalars, per-set Miller loops, signature-sum Miller loop,
           Fp12 product
  node     all_gather of the 576-byte Fp12 partials (RCCL over xGMI when N > 1)
  rank 0.. lsg_final_submit/wait: product of partials + one final exponentiation -> verdict
Steps are pipelined as a firehose verifier runs them: two batches in flight (the library's two
pipeline slots) and the final exponentiation of batch k on its own stream while batch k+1
computes.  Every batch is verified (verdict checked) inside the timed region.
Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torch.distributed.run.
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
# 2 pipeline slots x 2 streams + the final-exponentiation stream (+ RCCL's): give each its
# own hardware queue instead of HIP's default 4 shared ones
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("LSG_HW_QUEUES", "16")
sys.path.insert(0, ROOT)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
METRIC = "BLS signature sets verified/sec (whole node) at 1/2/4/8 MI355X; p50 batch latency"


def interop_sk(i):
    return int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R_ORDER


def make_shard(ctx, rank, n):
    keys = 1024
    sks = [interop_sk(i) for i in range(keys)]
    pks = ctx.sk_to_pk(sks)
    base = rank * n
    msgs = [hashlib.sha256(b"lodestar-mi355x" + b"firehose" + (base + i).to_bytes(8, "little")).digest()
            for i in range(n)]
    sigs = ctx.sign([sks[(base + i) % keys] for i in range(n)], msgs)
    return [([pks[(base + i) % keys]], msgs[i], sigs[i]) for i in range(n)]


def make_block(ctx, rank, n):
    """SURVEY 8(d) config C, "full mainnet block body": n aggregate-attestation sets of 440-460
    signers each (~450), distinct messages.  Keys live in the device pubkey table (8f(1),
    lsg_pubkey_table_set over the 1024 interop keys) and sets name their signers by index,
    as the node's index2pubkey cache does; signatures are (sum sk) * H(m)."""
    from lodestar_amd._native import PkIndices
    keys = 1024
    sks = [interop_sk(i) for i in range(keys)]
    errs = ctx.pubkey_table_set(0, ctx.sk_to_pk(sks))
    if any(errs):
        raise SystemExit("pubkey table load failed")
    idx, agg_sk, msgs = [], [], []
    for i in range(n):
        g = rank * n + i
        size = 440 + (g * 7) % 21
        start = (g * 53) % keys
        ix = [(start + j) % keys for j in range(size)]
        idx.append(PkIndices(ix))
        agg_sk.append(sum(sks[k] for k in ix) % R_ORDER)
        msgs.append(hashlib.sha256(b"lodestar-mi355x" + b"block" + g.to_bytes(8, "little")).digest())
    sigs = ctx.sign(agg_sk, msgs)
    return [(idx[i], msgs[i], sigs[i]) for i in range(n)]


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
    per host core (poolSize.ts:7) -- on a bounded sample of ~budget_s seconds."""
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
        msg = b"".join(m for _, m, _ in sub)
        sig = b"".join(s for _, _, s in sub)
        nch = -(-k // chunk)
        verdicts = (ctypes.c_int * nch)()
        t0 = time.perf_counter()
        ok = lib.cpu_verify_chunks(pk, msg, sig, k, chunk, cores, 0x5EED, verdicts)
        dt = time.perf_counter() - t0
        if ok != nch:
            raise SystemExit(f"cpu baseline: {nch - ok} of {nch} batches failed on valid sets")
        return dt

    k = chunk * cores
    dt = run(k)  # calibration round: one batch per thread
    k = max(k, int(k * budget_s / max(dt, 1e-3)) // (chunk * cores) * chunk * cores)
    dt = run(k)
    return {"value": k / dt, "unit": "sets/s", "cores": cores, "kind": "port",
            "sample": f"{k} sets of this workload in 16-set RLC batches on {cores} threads "
                      f"(oracle/c, C restatement of the oracle, gcc -O3) in {dt:.1f}s"}


def pmc_traffic(kernel, sets_per_launch):
    """HBM bytes per launch of `kernel` from the committed PMC passes (tools/gpu_traffic.sh ->
    tools/pmc_traffic.py -> profiles/rNN_pmc_traffic.json: 2 x FETCH_SIZE + WRITE_SIZE), when
    they were measured at this launch size; None otherwise (PMC counters cannot be read from
    inside the timed run)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    k = d["kernels"].get(kernel)
    if k is None or d["sets_per_launch"] != sets_per_launch:
        return None
    return k["hbm_bytes_per_dispatch"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=384)
    ap.add_argument("--warmup", type=int, default=48)
    ap.add_argument("--workload", choices=["firehose", "block"], default="firehose",
                    help="firehose: config D shard (default, the headline line); block: config C")
    ap.add_argument("--sets-per-gpu", type=int, default=None, help="sets per step (4096 firehose, 128 block)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--depth", type=int, default=None,
                    help="submissions in flight (<= library pipeline slots; 3 firehose, 4 block)")
    ap.add_argument("--groups", type=int, default=None,
                    help="batches (steps) per submission, verified as separate RLC groups (12 firehose, 32 block)")
    args = ap.parse_args()
    block = args.workload == "block"
    if args.sets_per_gpu is None:
        args.sets_per_gpu = 128 if block else 4096
    # firehose default 12 x 3 (profiles/r01_bench_sweeps_inline.txt): 2.28M sets/s at p50 78 ms,
    # against 2.03-2.19M at p50 52 ms for 6 x 4 and 2.33M at p50 97 ms for 12 x 4
    if args.groups is None:
        args.groups = 32 if block else 12
    if args.depth is None:
        args.depth = 4 if block else 3

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from lodestar_amd._native import Context
    ctx = Context(local)
    n = args.sets_per_gpu
    M = max(1, args.groups)
    sets = make_block(ctx, rank, n * M) if block else make_shard(ctx, rank, n * M)
    # M steps' shards staged as one package; each ticket verifies them as M separate RLC
    # batches (groups of n sets, one Miller partial and one final exponentiation each)
    staged = ctx.stage(sets, seed=0x5EED + rank)

    def gather(parts):
        """all-gather the M partials of one ticket; -> per group, the partials of every rank"""
        if dist is None:
            return [[p] for p in parts]
        import torch
        t = torch.frombuffer(bytearray(b"".join(parts)), dtype=torch.uint8).cuda(local)
        out = torch.empty(world * 576 * M, dtype=torch.uint8, device=t.device)
        dist.all_gather_into_tensor(out, t)
        b = out.cpu().numpy().tobytes()
        return [[b[576 * (k * M + g):576 * (k * M + g) + 576] for k in range(world)] for g in range(M)]

    def barrier():
        if dist is not None:
            dist.barrier()

    def check(anyerr, ok):
        if anyerr or not ok:
            raise SystemExit(f"rank {rank}: verification failed (anyerr={anyerr}, verdict={ok})")

    def submit():
        t = ctx.batch_submit(staged, group_size=n if M > 1 else 0)
        if t is None:
            raise SystemExit("pipeline slots exhausted: lower --depth")
        return t

    def run(k_tickets, depth=2, capture=False):
        """k_tickets submissions of M batches each, `depth` in flight; returns per-ticket
        submit->last-verdict latencies and (if capture) the per-kernel HIP-event times of the
        last ticket and its final exponentiations."""
        lat, times = [], []
        pend_b, pend_f = collections.deque(), collections.deque()
        submitted = 0
        while submitted < k_tickets and len(pend_b) < depth:
            pend_b.append((submit(), time.perf_counter()))
            submitted += 1
        while pend_b:
            tb, t_sub = pend_b.popleft()
            parts, _errs, anyerr = ctx.batch_wait(tb)
            check(anyerr, True)
            if M == 1:
                parts = [parts]
            if capture:  # HIP-event kernel times of this ticket (recorded on the kernels' own streams)
                times.append(ctx.last_kernel_times())
            ft = ctx.final_submit_groups(gather(parts))  # the M batches' final checks in one ticket
            if ft is None:
                raise SystemExit("final-exponentiation entries exhausted")
            pend_f.append((ft, t_sub, anyerr))
            if submitted < k_tickets:
                pend_b.append((submit(), time.perf_counter()))
                submitted += 1
            while pend_f and (len(pend_f) > 1 or not pend_b):
                ft0, t0, ae = pend_f.popleft()
                check(ae, all(ctx.final_wait_groups(ft0)))
                lat.append(time.perf_counter() - t0)
        return lat, times

    tickets = -(-args.steps // M)
    steps = tickets * M
    run(max(1, -(-args.warmup // M)), depth=args.depth)
    barrier()
    t0 = time.perf_counter()
    lat, ktimes = run(tickets, depth=args.depth, capture=True)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        te = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        elapsed = float(te.item())
    # unloaded latency: one batch at a time
    lat1, _ = run(3, depth=1)

    # kernel-level roofline for the dominant kernel, from HIP events recorded on the streams
    # the kernels ran on during the last timed batch
    opc = json.load(open(os.path.join(ROOT, "bench", "opcount.json")))
    probe_fp, probe_mad = ctx.probe_fp_mul_rate()
    peak_mad = ctx.probe_mad_peak()  # measured v_mad_u64_u32 issue rate of this GPU (k_probe_mad)
    # per-ticket sum per kernel name (tree levels add up), averaged over the timed tickets
    agg = {}
    for ticket_times in ktimes:
        for name, ms in ticket_times:
            agg[name] = agg.get(name, 0.0) + ms / len(ktimes)
    # pairs per Miller item: the library's LSG_MILLER_K (default 4) sets k_miller_accum's work per set
    mk = os.environ.get("LSG_MILLER_K", "4")
    accum_key = f"miller_accum{mk}_per_set" if f"miller_accum{mk}_per_set" in opc["stage_fp_muls"] \
        else "miller_accum2_per_set"
    stage_of = {"k_miller_multi": "miller_multi2_per_set", "k_miller_accum": accum_key,
                "k_miller_lines": "miller_lines", "k_sig_scale": "sig_scale",
                "k_sig_subgroup": "sig_subgroup", "k_sig_decode": "sig_decode", "k_pk_scale": "pk_scale"}
    per_set = {k: v for k, v in agg.items() if k in stage_of}
    dom = max(per_set, key=per_set.get)
    muls = opc["stage_fp_muls"][stage_of[dom]] * n * M  # one launch covers the M groups' sets
    achieved = muls * opc["mads_per_fp_mul"] / (agg[dom] * 1e-3) / 1e12
    peak = peak_mad / 1e12
    roof = {"bound": "valu", "kernel": dom, "achieved": round(achieved, 3), "peak": round(peak, 3),
            "unit": "Tmad/s (v_mad_u64_u32)", "frac": round(achieved / peak, 4),
            "traffic": pmc_traffic(dom, n * M),
            "kernel_ms": round(agg[dom], 3), "work_per_launch_fp_muls": muls}
    total_sets = n * world * steps
    value = total_sets / elapsed
    # whole-path work per set: the per-set stages with the bucket-MSM signature sums (groups of
    # n >= 256 sets take the MSM path, smaller ones per-set [r_i] sig_i) plus each group's share
    # of its per-group stages, plus one G1 addition per extra signer of an aggregate set
    if n >= 256:
        per_set_muls = opc["batched_single_set_msm_fp_muls"] + opc["per_batch_msm_fp_muls"] / n
    else:
        per_set_muls = opc["batched_single_set_fp_muls"] + opc["per_batch_fp_muls"] / n
    # the whole-path counts price the Miller stage at K = 2; credit only the work K actually does
    per_set_muls += opc["stage_fp_muls"][accum_key] - opc["stage_fp_muls"]["miller_accum2_per_set"]
    pks_per_set = sum(len(p) for p, _, _ in sets) / len(sets)
    per_set_muls += (pks_per_set - 1) * opc["aggregate_extra_per_pubkey_fp_muls"]
    node_mads = value * per_set_muls * opc["mads_per_fp_mul"]
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            if block:  # the CPU path gets the aggregated keys for free (favours the CPU)
                cpu = cpu_baseline_oracle([([ctx.aggregate_pubkeys(p)[0]], m, sg) for p, m, sg in sets[:256]])
                cpu["sample"] += "; pubkey aggregation (main thread in the reference) excluded"
            else:
                cpu = cpu_baseline_oracle(sets)
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "sets/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": ({"workload": "block-body (SURVEY 8d config C): aggregate-attestation sets of 440-460 "
                                    "signers named by index into the device pubkey table, distinct messages, one "
                                    "RLC multi-pairing per block",
                        "sets_per_gpu": n, "global_batch": n * world, "keys": 1024,
                        "pubkeys_per_set": round(pks_per_set, 1), "parallelism": f"shard{world}"} if block else
                       {"workload": "firehose-32k shard (SURVEY 8d config D): single-pubkey gossip sets, RLC batch "
                                    "per GPU, RCCL all-gather of Fp12 partials, one final exponentiation",
                        "sets_per_gpu": n, "global_batch": n * world, "keys": 1024,
                        "parallelism": f"shard{world}"}),
            "p50_batch_latency_ms": round(1e3 * statistics.median(lat), 3),
            "p50_unloaded_latency_ms": round(1e3 * statistics.median(lat1), 3),
            "pipeline_depth": args.depth, "batches_per_submission": M,
            "roofline": roof,
            "whole_path_mad_frac": round(node_mads / (peak_mad * world), 4),
            "kernel_ms": {k: round(v, 3) for k, v in agg.items()},
            "probe_lane_fp_mul_per_s": probe_fp,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    staged.free()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
