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
from tests import blsdata as bd


class OracleBackend:
    """ShardedVerifier backend computed by the oracle (test infrastructure only): the same
    submit / partial / final_verify / resolve protocol as GpuBackend."""

    @staticmethod
    def _rands(seed, n):
        rng = random.Random(seed)
        return [rng.getrandbits(64) or 1 for _ in range(n)]

    def submit(self, jobs, seed=0):
        return (jobs, seed)

    def partial(self, handle):
        from oracle.curves import g1_serialize
        jobs, seed = handle
        flat = [(g1_serialize(ov.aggregate_pubkeys([ov.public_key_from_bytes(p) for p in pks])), m, s)
                for sets, flags in jobs if flags & 1 for pks, m, s in sets]
        part, _errs = ov.batch_partial(flat, self._rands(seed, len(flat)))
        return part, bool(flat)

    def final_verify(self, partials):
        return ov.final_verify_partials(list(partials))

    def resolve(self, handle, node_valid):
        jobs, seed = handle
        return self.verify_jobs(jobs, seed)

    def verify_jobs(self, jobs, seed=0):
        reqs = []
        for sets, flags in jobs:
            reqs.append({"opts": {"batchable": bool(flags & 1)},
                         "sets": [{"publicKey": pks[0], "message": m, "signature": s} for pks, m, s in sets]})
        rng = random.Random(seed)
        out = ov.verify_many_signature_sets(reqs, rand_fn=lambda: rng.getrandbits(64) or 1)
        res = []
        for kind, val in out["results"]:
            res.append((VALID if val else INVALID, 0) if kind == "success" else (ERROR, val))
        return res, {"batch_retries": out["batch_retries"]}


def make_jobs(corrupt=None):
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
    return [tuple(r) for r in OracleBackend().verify_jobs(jobs, seed=1)[0]]


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
        corrupt = {"valid": None, "wrong_msg": (3, 1, bd.corrupt_wrong_message),
                   "truncated": (0, 0, bd.corrupt_truncate)}[case]
        out = ShardedVerifier(OracleBackend(), dist=dist).verify_jobs(make_jobs(corrupt), seed=11)
        q.put((rank, out.results, out.combined_ok, out.retried_ranks))
    finally:
        dist.destroy_process_group()


# the node check covers every set that decodes (an undecodable set contributes nothing and
# its job errors through the chunk rules), so only the wrong-message case fails it
@pytest.mark.parametrize("case,retried,combined", [("valid", [], True), ("wrong_msg", [1], False),
                                                   ("truncated", [0], True)])
def test_sharded_gloo_world2(case, retried, combined):
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
    corrupt = {"valid": None, "wrong_msg": (3, 1, bd.corrupt_wrong_message),
               "truncated": (0, 0, bd.corrupt_truncate)}[case]
    exp = expected(make_jobs(corrupt))
    for rank, results, combined_ok, rr in got:
        assert results == exp, (rank, results, exp)
        assert combined_ok == combined
        assert rr == retried
