"""Node-sharded verification (lodestar_amd/sharded.py) on the CPU: world_size 2
over torch.distributed "gloo", with an oracle-backed backend standing in for the GPU.  The
multi-GPU bench runs the same gather -> one final exponentiation -> localise-on-failure
logic over RCCL; here every rank's partial comes from the oracle, so the test pins the
host-side protocol: job assignment, the one collective, the node verdict, failure
localisation and the per-job fallback verdicts (worker.ts:30-106 semantics)."""
import os
import random
import socket

import pytest

from lodestar_amd.sharded import ShardedVerifier, assign_jobs, rank_seed, VALID, INVALID, ERROR
from oracle import verifier as ov
from oracle.curves import BLST_NAMES, BlstError
from tests import blsdata as bd


class OracleBackend:
    """ShardedVerifier backend computed by the oracle (test infrastructure only): the same
    submit / partial / final_verify / resolve protocol as GpuBackend, and ``resolve`` follows
    the device's package rules (lsg_host.hip pkg_resolve): the rank's own package-group check
    (every batchable set that decodes, one RLC batch) decides -- the node verdict is advisory;
    a passing group answers every batchable job, a failing one is localised by the 16-job
    chunks (phase B) and then per job (phase C); a bad key rejects every job."""

    @staticmethod
    def _rands(seed, n):
        rng = random.Random(seed)
        return [rng.getrandbits(64) or 1 for _ in range(n)]

    def submit(self, jobs, seed=0):
        return (jobs, seed)

    @staticmethod
    def _batch_sets(jobs):
        return [(pks[0], m, s) for sets, flags in jobs if flags & 1 for pks, m, s in sets]

    def partial(self, handle):
        jobs, seed = handle
        flat = self._batch_sets(jobs)
        part, _errs = ov.batch_partial(flat, self._rands(seed, len(flat)))
        return part, bool(flat)

    def final_verify(self, partials):
        return ov.final_verify_partials(list(partials))

    @staticmethod
    def _set_error(s):
        pks, _m, sig = s
        try:
            ov.signature_from_bytes(sig, True)
            if ov.public_key_from_bytes(pks[0]) is None:
                return 6  # BLST_PK_IS_INFINITY
        except BlstError as e:
            return e.code
        return 0

    @staticmethod
    def _maybe_batch(sets, rng):
        return ov.verify_signature_sets_maybe_batch(
            [{"publicKey": ov.public_key_from_bytes(p[0]), "message": m, "signature": s} for p, m, s in sets],
            [rng.getrandbits(64) or 1 for _ in sets])

    def resolve(self, handle, node_valid):
        jobs, seed = handle
        rng = random.Random(seed + 1)
        res = [None] * len(jobs)
        stats = {"batch_retries": 0, "batch_sigs_success": 0}
        for j, (sets, _f) in enumerate(jobs):  # deserializeSet over the package (worker.ts:41-43)
            for pks, _m, _s in sets:
                try:
                    ov.public_key_from_bytes(pks[0])
                except BlstError as e:
                    stats.update(key_error=e.code, key_error_job=j)
                    return [(ERROR, e.code)] * len(jobs), stats

        def job_error(sets):
            if not sets:
                return 100
            codes = [self._set_error(s) for s in sets]
            return next((c for c in codes if c and c != 6), 0) or next((c for c in codes if c), 0)

        flat = self._batch_sets(jobs)
        own_ok = True
        if flat:  # the package group's own final exponentiation (computed in phase A)
            part, _ = ov.batch_partial(flat, self._rands(seed, len(flat)))
            own_ok = ov.final_verify_partials([part])
        retry = []
        for j, (sets, flags) in enumerate(jobs):
            if not flags & 1:
                e = job_error(sets)
                res[j] = (ERROR, e) if e else ((VALID if self._maybe_batch(sets, rng) else INVALID), 0)
        bjobs = [j for j, (_s, f) in enumerate(jobs) if f & 1]
        chunks = ov.chunkify_maximize_chunk_size(bjobs, 16) if bjobs else []
        errc = [any(self._set_error(s) for j in c for s in jobs[j][0]) for c in chunks]
        for c, chunk in enumerate(chunks):
            n = sum(len(jobs[j][0]) for j in chunk)
            if n == 0:
                stats["batch_retries"] += 1
                for j in chunk:
                    res[j] = (ERROR, 100)
            elif not errc[c]:
                if own_ok:
                    stats["batch_sigs_success"] += n
                    for j in chunk:
                        res[j] = (VALID, 0)
                elif self._maybe_batch([s for j in chunk for s in jobs[j][0]], rng):  # phase B
                    stats["batch_sigs_success"] += n
                    for j in chunk:
                        res[j] = (VALID, 0)
                else:
                    stats["batch_retries"] += 1
                    retry.extend(chunk)
            else:
                stats["batch_retries"] += 1
                for j in chunk:
                    e = job_error(jobs[j][0])
                    if e:
                        res[j] = (ERROR, e)
                    elif own_ok:
                        res[j] = (VALID, 0)
                    else:
                        retry.append(j)
        for j in retry:  # phase C
            e = job_error(jobs[j][0])
            res[j] = (ERROR, e) if e else ((VALID if self._maybe_batch(jobs[j][0], rng) else INVALID), 0)
        return res, stats

    def verify_jobs(self, jobs, seed=0):
        """worker.ts:30-106 itself (the reference the package rules must agree with)."""
        reqs = []
        for sets, flags in jobs:
            reqs.append({"opts": {"batchable": bool(flags & 1)},
                         "sets": [{"publicKey": pks[0], "message": m, "signature": s} for pks, m, s in sets]})
        rng = random.Random(seed)
        out = ov.verify_many_signature_sets(reqs, rand_fn=lambda: rng.getrandbits(64) or 1)
        res = []
        codes = {"BLST_ERROR: " + name: code for code, name in BLST_NAMES.items()}
        codes["Empty signature set"] = 100
        for kind, val in out["results"]:
            res.append((VALID if val else INVALID, 0) if kind == "success" else (ERROR, codes[val]))
        return res, {"batch_retries": out["batch_retries"], "batch_sigs_success": out["batch_sigs_success"]}


def corrupt_pubkey(s):
    """a 96-byte key off the curve: deserializeSet throws BLST_POINT_NOT_ON_CURVE"""
    pks, m, sig = s
    b = bytearray(pks[0])
    b[95] ^= 1
    return ([bytes(b)], m, sig)


CASES = {"valid": None, "wrong_msg": (3, 1, bd.corrupt_wrong_message), "truncated": (0, 0, bd.corrupt_truncate),
         "bad_key": (3, 0, corrupt_pubkey), "one_job": "one_job"}


def make_jobs(corrupt=None):
    if corrupt == "one_job":  # rank 1 gets an empty shard
        return [([bd.single_set(700 + k, tag="shard") for k in range(2)], 1)]
    jobs = []
    for j in range(4):
        sets = [bd.single_set(700 + 2 * j + k, tag="shard") for k in range(1 + (j % 2))]
        jobs.append((sets, 1))
    if corrupt is not None:
        j, k, fn = corrupt
        sets = list(jobs[j][0])
        sets[k] = fn(sets[k])
        jobs[j] = (sets, 1)
    return jobs


def expected(jobs):
    try:
        return [tuple(r) for r in OracleBackend().verify_jobs(jobs, seed=1)[0]]
    except BlstError as e:  # deserializeSet threw: the worker rejects every job of the package
        return [(ERROR, e.code)] * len(jobs)


def test_assign_jobs_balanced_and_whole():
    assert assign_jobs([1, 2, 1, 2], 2) == [0, 0, 1, 1]
    assert assign_jobs([5, 1, 1, 1], 2) == [0, 1, 1, 1]
    assert assign_jobs([1] * 8, 4) == [0, 0, 1, 1, 2, 2, 3, 3]
    assert assign_jobs([3, 0, 3], 8) == [0, 4, 4]
    assert assign_jobs([], 2) == [] and assign_jobs([2, 2], 1) == [0, 0]


def test_rank_seed_keeps_os_randomness():
    """seed 0 (production) must reach every rank unchanged, so that the RLC
    randomizers come from the OS CSPRNG on every rank, never from a public splitmix sequence."""
    assert [rank_seed(0, r) for r in range(8)] == [0] * 8
    assert [rank_seed(5, r) for r in range(3)] == [5, 6, 7]


def test_sharded_single_rank_matches_worker_semantics():
    sv = ShardedVerifier(OracleBackend())
    ok = sv.verify_jobs(make_jobs(), seed=3)
    assert ok.combined_ok and ok.results == [(VALID, 0)] * 4
    bad = make_jobs(corrupt=(1, 1, bd.corrupt_wrong_message))
    out = sv.verify_jobs(bad, seed=3)
    assert not out.combined_ok and out.retried_ranks == [0]
    assert out.results == expected(bad)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, case, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = ShardedVerifier(OracleBackend(), dist=dist).verify_jobs(make_jobs(CASES[case]), seed=11)
        q.put((rank, out.results, out.combined_ok, out.retried_ranks, out.rank_stats))
    finally:
        dist.destroy_process_group()


# the node check covers every set that decodes (an undecodable set contributes nothing and
# its job errors through the chunk rules), so only the wrong-message case fails it
@pytest.mark.parametrize("case,retried,combined", [("valid", [], True), ("wrong_msg", [1], False),
                                                   ("truncated", [0], True), ("bad_key", None, True),
                                                   ("one_job", [], True)])
def test_sharded_gloo_world2(case, retried, combined):
    """world_size 2 over gloo: every rank's verdicts equal worker.ts over the whole package,
    and every rank's counters equal worker.ts over its own share (chunks form per rank)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    jobs = make_jobs(CASES[case])
    exp = expected(jobs)
    owner = assign_jobs([len(s) for s, _ in jobs], 2)
    for rank, results, combined_ok, rr, rank_stats in got:
        assert results == exp, (rank, results, exp)
        if case == "bad_key":  # the bad key sits on rank 1; rank 0's jobs are rejected too
            assert all(r == (ERROR, 2) for r in results)
            continue
        assert combined_ok == combined
        assert rr == retried
        for r in range(2):
            share = [jobs[j] for j in range(len(jobs)) if owner[j] == r]
            _res, st = OracleBackend().verify_jobs(share, seed=5)
            assert rank_stats[r]["batch_retries"] == st["batch_retries"], (r, rank_stats[r], st)
            assert rank_stats[r]["batch_sigs_success"] == st["batch_sigs_success"], (r, rank_stats[r], st)


def test_resolve_ignores_a_wrong_node_pass():
    """a caller that claims the node check passed (node_valid 1) for a share whose
    own check fails gets the localised verdicts, never a wrongly accepted package."""
    be = OracleBackend()
    jobs = make_jobs(CASES["wrong_msg"])
    res, st = be.resolve(be.submit(jobs, seed=2), 1)
    assert res == expected(jobs) and res[3] == (INVALID, 0)
    assert st["batch_retries"] == be.verify_jobs(jobs, seed=2)[1]["batch_retries"]
