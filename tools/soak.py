#!/usr/bin/env python3
"""Verdict soak on the GPU (north_star: "zero verdict mismatches over 10^7 valid plus
adversarially corrupted sets").

Streams packages of worker jobs through the asynchronous jobs path (lsg_submit_jobs /
lsg_wait_jobs: batch per package, per-job retry, worker.ts:30-106) and compares every job's
verdict with its expected value:
  - sets come from a pool of valid single sets (interop keys, GPU-signed) and, at --bad-rate
    (default 1%), from corrupted variants split evenly over the config E corruptions
    (wrong message, flipped x bit, truncated, non-subgroup point, infinity);
  - each corrupted variant's outcome (false, or the BLST code Signature.fromBytes throws) is
    computed once by the oracle (tests/blsdata.py, oracle/verifier.py);
  - a job's expected verdict is maybeBatch's (maybeBatch.ts:16-39): the first set in job
    order whose signature does not decode rejects the job with that code; otherwise false if
    any set is false, else true.
Job sizes mix gossip singles, small batches and 128-set chunks; 90% are batchable.  RLC
randomizers come from the OS CSPRNG (seed 0), fresh for every package.
Prints one progress line per ~10 s and a final JSON summary line.
"""
import argparse
import ctypes
import hashlib
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("LSG_HW_QUEUES", "16")
sys.path.insert(0, ROOT)

from lodestar_amd import _native as N  # noqa: E402

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def interop_sk(i):
    return int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R_ORDER


def expected_of(s):
    """(status, code) of a one-set maybeBatch call from the oracle: the corrupted variants only."""
    from oracle import verifier as ov
    from oracle.curves import BlstError
    pks, m, sig = s
    try:
        ov.signature_from_bytes(sig)
    except BlstError as e:
        return (N.LSG_ERROR, e.code)
    pk = ov.public_key_from_bytes(pks[0])
    ok = ov.verify_signature_sets_maybe_batch([{"publicKey": pk, "message": m, "signature": sig}])
    return (N.LSG_VALID if ok else N.LSG_INVALID, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=10_000_000)
    ap.add_argument("--pool", type=int, default=8192)
    ap.add_argument("--bad-rate", type=float, default=0.01)
    ap.add_argument("--package", type=int, default=4096, help="sets per package (lsg_submit_jobs call)")
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    rng = random.Random(args.seed)

    from tests import blsdata as bd
    ctx = N.Context(0)
    t0 = time.time()
    sks = [interop_sk(i) for i in range(1024)]
    pks = ctx.sk_to_pk(sks)
    msgs = [hashlib.sha256(b"lodestar-mi355x" + b"soak" + i.to_bytes(8, "little")).digest() for i in range(args.pool)]
    sigs = ctx.sign([sks[i % 1024] for i in range(args.pool)], msgs)
    valid = [([pks[i % 1024]], msgs[i], sigs[i]) for i in range(args.pool)]
    bad, bad_exp = [], []
    kinds = [bd.corrupt_wrong_message, lambda s: bd.corrupt_flip_x_bit(s, rng.randrange(8)), bd.corrupt_truncate,
             lambda s: bd.corrupt_not_in_group(s, rng.randrange(256)), bd.corrupt_infinity]
    for k in range(40):
        s = kinds[k % len(kinds)](valid[rng.randrange(args.pool)])
        bad.append(s)
        bad_exp.append(expected_of(s))
        print(f"corrupted variant {k}: expected {bad_exp[-1]} ({time.time() - t0:.1f}s)", flush=True)
    print(f"pool: {len(valid)} valid, {len(bad)} corrupted ({time.time() - t0:.1f}s)", flush=True)

    pool = valid + bad
    pool_exp = [(N.LSG_VALID, 0)] * len(valid) + bad_exp
    pool_buf = N.SetBuffer(pool)  # one ctypes struct per pool set; packages copy them

    def job_verdict(idx):
        for j in idx:
            if pool_exp[j][0] == N.LSG_ERROR:
                return pool_exp[j]
        for j in idx:
            if pool_exp[j][0] == N.LSG_INVALID:
                return (N.LSG_INVALID, 0)
        return (N.LSG_VALID, 0)

    def make_package():
        jobs, total = [], 0
        while total < args.package:
            u = rng.random()
            size = 1 if u < 0.5 else (rng.randrange(2, 17) if u < 0.75 else 128)
            idx = [len(valid) + rng.randrange(len(bad)) if rng.random() < args.bad_rate else rng.randrange(len(valid))
                   for _ in range(size)]
            jobs.append((idx, N.LSG_JOB_BATCHABLE if rng.random() < 0.9 else 0))
            total += size
        arr = (N.LsgSet * total)()
        jarr = (N.LsgJob * len(jobs))()
        o = 0
        for k, (idx, flags) in enumerate(jobs):
            for q, j in enumerate(idx):
                arr[o + q] = pool_buf.arr[j]
            jarr[k].sets = ctypes.cast(ctypes.byref(arr, o * ctypes.sizeof(N.LsgSet)), ctypes.POINTER(N.LsgSet))
            jarr[k].n_sets = len(idx)
            jarr[k].flags = flags
            o += len(idx)
        return jarr, arr, [job_verdict(idx) for idx, _ in jobs], total

    lib = ctx.lib
    done_sets = done_jobs = mismatches = retries = 0
    n_false = n_err = 0
    pend = []
    t_start = t_last = time.time()

    def drain_one():
        nonlocal done_sets, done_jobs, mismatches, retries, n_false, n_err
        t, nj, exp, total = pend.pop(0)
        res = (N.LsgJobResult * nj)()
        st = N.LsgStats()
        ctx._check(lib.lsg_wait_jobs(ctx.h, t, res, ctypes.byref(st)), "lsg_wait_jobs")
        for k in range(nj):
            got = (res[k].status, res[k].err_code if res[k].status == N.LSG_ERROR else 0)
            if got != exp[k]:
                mismatches += 1
                if mismatches <= 10:
                    print(f"MISMATCH job {done_jobs + k}: got {got} expected {exp[k]}", flush=True)
            n_false += got[0] == N.LSG_INVALID
            n_err += got[0] == N.LSG_ERROR
        retries += st.batch_retries
        done_sets += total
        done_jobs += nj

    submitted = 0
    while submitted < args.sets or pend:
        if submitted < args.sets and len(pend) < args.depth:
            jarr, arr, exp, total = make_package()
            t = ctypes.c_uint64()
            rc = lib.lsg_submit_jobs(ctx.h, jarr, len(exp), 0, ctypes.byref(t))
            if rc == N.LSG_ERR_BUSY:
                drain_one()
                continue
            ctx._check(rc, "lsg_submit_jobs")
            pend.append((t.value, len(exp), exp, total))
            submitted += total
            continue
        drain_one()
        if time.time() - t_last > 10:
            t_last = time.time()
            el = t_last - t_start
            print(f"{done_sets} sets / {done_jobs} jobs verified, {mismatches} mismatches, {n_false} false, "
                  f"{n_err} rejected, {retries} batch retries, {done_sets / el:.0f} sets/s", flush=True)
    el = time.time() - t_start
    print(json.dumps({"sets": done_sets, "jobs": done_jobs, "mismatches": mismatches, "jobs_false": n_false,
                      "jobs_rejected": n_err, "batch_retries": retries, "bad_rate": args.bad_rate,
                      "corrupted_variants": len(bad), "seconds": round(el, 1),
                      "sets_per_s": round(done_sets / el, 1), "path": "lsg_submit_jobs/lsg_wait_jobs (H7 semantics)",
                      "package_sets": args.package, "depth": args.depth}), flush=True)
    ctx.close()
    return 1 if mismatches else 0


if __name__ == "__main__":
    sys.exit(main())
