#!/usr/bin/env python3
"""Verdict soak on the GPU (north_star: "zero verdict mismatches over 10^7 valid plus
adversarially corrupted sets").  Test infrastructure (tests/).

Every set is distinct: each package draws fresh messages (a global counter; every
--committee-every-th package signs 64 committee messages shared by its sets, so hash_to_G2
runs once per message), signs them on the
GPU with the interop keys sk_{v mod 1024}, corrupts --bad-rate of them (default 1%) split
evenly over the config E kinds, cuts them into worker jobs of mixed sizes (gossip singles,
2-16-set batches, 128-set chunks; 90% batchable) and streams the packages through the
asynchronous jobs path (lsg_submit_jobs / lsg_wait_jobs: one RLC group per package, then the
chunk and per-job fallback of worker.ts:30-106), with fresh OS-CSPRNG randomizers.
Expected verdicts never come from the GPU:
  - valid sets: true by construction (and a sample per package is checked by the C oracle);
  - wrong message / infinity signature: false; truncated: BLST_INVALID_SIZE; non-subgroup
    point (the committed decode fixtures, tests/golden/sig_decode.json): BLST_POINT_NOT_IN_GROUP;
  - flipped x bit: the C oracle's decode outcome (tests/cpu_oracle.py);
  - a job: maybeBatch.ts:16-39 -- the first set whose signature does not decode rejects the job
    with its code, else false if any set is false, else true.
Prints a progress line every ~10 s and a final JSON summary line.
"""
import argparse
import hashlib
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lodestar_amd import _native as N  # noqa: E402
from tests import cpu_oracle as co  # noqa: E402

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def interop_sk(i):
    return int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R_ORDER


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=10_000_000)
    ap.add_argument("--bad-rate", type=float, default=0.01)
    ap.add_argument("--package", type=int, default=32768, help="sets per package (lsg_submit_jobs call)")
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--committee-every", type=int, default=2,
                    help="every K-th package signs committee messages: 64 distinct messages, set i of the "
                         "package in committee (i + i // 1024) mod 64 (hash_to_G2 once per message); 0: never")
    ap.add_argument("--devices", type=int, default=1,
                    help="> 1: one context over this many duplicate ids of GPU 0 (each device's share of a "
                         "package staged on a thread of its own, device-copy exchange)")
    ap.add_argument("--submitters", type=int, default=1,
                    help="host threads submitting and waiting packages at once (packages are staged with the "
                         "context lock released)")
    args = ap.parse_args()
    import threading
    import numpy as np

    ctx = N.Context(0) if args.devices <= 1 else N.Context(devices=[0] * args.devices)
    ctx.reserve(args.package + 256, n_slots=min(16, args.submitters * args.depth + 1))
    sks = [interop_sk(i) for i in range(1024)]
    pks = ctx.sk_to_pk(sks)
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "sig_decode.json")))
    non_subgroup = [bytes.fromhex(c["sig"]) for c in gold["cases"] if c["err"] == 3 and len(c["sig"]) == 192]
    counter = 0
    n_pkg = 0
    lock = threading.Lock()

    def make_package(rng):
        nonlocal counter
        nonlocal n_pkg
        n = args.package
        with lock:  # distinct messages across the submitting threads
            base = counter
            counter += n
            n_pkg += 1
            pkg_no = n_pkg
        if args.committee_every and pkg_no % args.committee_every == 0:
            # base + c: distinct from every other package's messages (bases step by n >= 64)
            msgs = [hashlib.sha256(b"lodestar-mi355x" + b"soak" + (base + (i + i // 1024) % 64).to_bytes(8, "little"))
                    .digest() for i in range(n)]
        else:
            msgs = [hashlib.sha256(b"lodestar-mi355x" + b"soak" + (base + i).to_bytes(8, "little")).digest()
                    for i in range(n)]
        keys = [(base + i) % 1024 for i in range(n)]
        sigs = ctx.sign([sks[k] for k in keys], msgs)
        sets = [([pks[keys[i]]], msgs[i], sigs[i]) for i in range(n)]
        exp = [(N.LSG_VALID, 0)] * n
        bad = sorted(rng.sample(range(n), int(n * args.bad_rate)))
        flips = []
        for q, i in enumerate(bad):
            pk, m, sg = sets[i]
            kind = q % 5
            if kind == 0:
                sets[i], exp[i] = (pk, hashlib.sha256(m).digest(), sg), (N.LSG_INVALID, 0)
            elif kind == 1:
                b = bytearray(sg)
                b[40 + rng.randrange(8)] ^= 1 << rng.randrange(8)
                sets[i] = (pk, m, bytes(b))
                flips.append(i)
            elif kind == 2:
                sets[i], exp[i] = (pk, m, sg[:32]), (N.LSG_ERROR, 10)
            elif kind == 3:
                sets[i], exp[i] = (pk, m, rng.choice(non_subgroup)), (N.LSG_ERROR, 3)
            else:
                sets[i], exp[i] = (pk, m, bytes([0xC0]) + bytes(95)), (N.LSG_INVALID, 0)
        check = flips + rng.sample(range(n), 16)  # the flipped sets + a sample of the valid ones
        per = co.verify_each([sets[i][0][0] for i in check], [sets[i][1] for i in check], [sets[i][2] for i in check])
        for i, v in zip(check, per):
            e = (N.LSG_ERROR, -v) if v < 0 else ((N.LSG_VALID if v else N.LSG_INVALID), 0)
            if i in flips:
                exp[i] = e
            elif e != exp[i]:
                raise SystemExit(f"oracle disagrees with the construction of set {base + i}: {e} vs {exp[i]}")
        jobs, jexp, pos = [], [], 0
        while pos < n:
            u = rng.random()
            size = min(n - pos, 1 if u < 0.5 else (rng.randrange(2, 17) if u < 0.75 else 128))
            idx = list(range(pos, pos + size))
            pos += size
            jobs.append(([sets[i] for i in idx], N.LSG_JOB_BATCHABLE if rng.random() < 0.9 else 0))
            v = (N.LSG_VALID, 0)
            err = next((exp[i] for i in idx if exp[i][0] == N.LSG_ERROR), None)
            if err:
                v = err
            elif any(exp[i][0] == N.LSG_INVALID for i in idx):
                v = (N.LSG_INVALID, 0)
            jexp.append(v)
        return N.PreparedJobs(jobs), np.array(jexp, dtype=np.int32), n

    done_sets = done_jobs = mismatches = retries = n_false = n_err = 0
    t_start = time.time()
    t_last = [t_start]
    failures = []

    def drain_one(pend):
        nonlocal done_sets, done_jobs, mismatches, retries, n_false, n_err
        t, exp, n, _pj = pend.pop(0)
        res, st = ctx.wait_jobs(t, raw=True)
        got = np.frombuffer(res, dtype=np.int32, count=2 * len(exp)).reshape(-1, 2).copy()
        got[got[:, 0] != N.LSG_ERROR, 1] = 0
        bad = np.nonzero((got != exp).any(axis=1))[0]
        with lock:
            for k in bad[:max(0, 10 - mismatches)]:
                print(f"MISMATCH job {done_jobs + int(k)}: got {tuple(got[k])} expected {tuple(exp[k])}", flush=True)
            mismatches += len(bad)
            n_false += int((got[:, 0] == N.LSG_INVALID).sum())
            n_err += int((got[:, 0] == N.LSG_ERROR).sum())
            retries += st["batch_retries"]
            done_sets += n
            done_jobs += len(exp)
            if time.time() - t_last[0] > 10:
                t_last[0] = time.time()
                print(f"{done_sets} sets / {done_jobs} jobs verified, {mismatches} mismatches, {n_false} false, "
                      f"{n_err} rejected, {retries} batch retries ({t_last[0] - t_start:.0f} s, generation included)",
                      flush=True)

    def submitter(k, quota):
        try:
            rng = random.Random(args.seed * 1000003 + k)
            pend = []
            submitted = 0
            while submitted < quota or pend:
                if submitted < quota and len(pend) < args.depth:
                    pj, exp, n = make_package(rng)
                    t = ctx.submit_jobs(pj)
                    while t is None:  # every slot busy (other threads' packages): wait one of ours
                        if pend:
                            drain_one(pend)
                        else:
                            time.sleep(0.001)
                        t = ctx.submit_jobs(pj)
                    pend.append((t, exp, n, pj))
                    submitted += n
                    continue
                drain_one(pend)
        except BaseException as e:  # noqa: BLE001 -- reported as a failure of the soak
            failures.append(repr(e))

    per = -(-args.sets // args.submitters)
    threads = [threading.Thread(target=submitter, args=(k, max(0, min(per, args.sets - k * per)))) for k in range(args.submitters)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    if failures:
        raise SystemExit(f"soak: a submitting thread failed: {failures[:3]}")
    el = time.time() - t_start
    print(json.dumps({"sets": done_sets, "distinct_sets": done_sets, "committee_every": args.committee_every,
                      "jobs": done_jobs, "mismatches": mismatches,
                      "jobs_false": n_false, "jobs_rejected": n_err, "batch_retries": retries,
                      "bad_rate": args.bad_rate, "seconds_incl_generation": round(el, 1),
                      "path": "lsg_submit_jobs/lsg_wait_jobs (one RLC group per package + worker.ts fallback)",
                      "package_sets": args.package, "depth": args.depth, "devices": args.devices,
                      "submitters": args.submitters}), flush=True)
    ctx.close()
    return 1 if mismatches else 0


if __name__ == "__main__":
    sys.exit(main())
