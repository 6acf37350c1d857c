"""Node-sharded verification across the GPUs of one node.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on ROCm, "gloo" in
the CPU tests).  For one package of jobs (BlsWorkReq[], packages/beacon-node/src/chain/bls/
multithread/types.ts:14-17) every rank:

1. takes its shard: whole jobs, never split, assigned by cumulative set count so that the
   shards are balanced (``assign_jobs``);
2. reduces its shard to one un-exponentiated Fp12 Miller product (``backend.batch_partial``:
   decode + subgroup check, hash_to_G2, RLC scalars, Miller loops, the local
   ML(-G1, sum r_i sig_i) term);
3. all-gathers the 576-byte partials (one collective: the path's only exchange step);
4. multiplies them and runs ONE final exponentiation (``backend.final_verify``).

If that combined check fails, or some shard could not be batched, each rank
final-exponentiates its own partial to localise the failing shards; only those ranks run the
per-job path (``backend.verify_jobs``: worker.ts:30-106 batch + per-job retry), and the
per-job verdicts are all-gathered.  Passing shards report every job valid, exactly what the
per-job path would give for them (a valid RLC batch implies valid jobs up to the 2^-64
randomizer soundness bound the reference accepts too).

The backend is duck-typed: ``GpuBackend`` (this package, HIP through the C ABI) in
production, an oracle-backed one in the CPU tests.
"""
from dataclasses import dataclass

VALID, INVALID, ERROR = 1, 0, 2


def assign_jobs(job_sizes, world):
    """Rank of every job: contiguous, balanced by cumulative set count (a job is never split).
    Job j goes to floor(sets_before_j * world / total)."""
    total = sum(job_sizes)
    if total == 0 or world <= 1:
        return [0] * len(job_sizes)
    out, before = [], 0
    for n in job_sizes:
        out.append(min(world - 1, before * world // total))
        before += n
    return out


@dataclass
class ShardOutcome:
    results: list          # per job: (status, err_code)
    combined_ok: bool      # the one-final-exponentiation node check passed
    retried_ranks: list    # ranks that fell back to the per-job path


class ShardedVerifier:
    def __init__(self, backend, dist=None, group=None):
        self.backend = backend
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group) if dist is not None else 0
        self.world = dist.get_world_size(group) if dist is not None else 1

    def _all_gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def verify_jobs(self, jobs, seed=0):
        """jobs: list of (sets, flags), sets = [(pks, msg, sig)], identical on every rank.
        Returns a ShardOutcome with per-job (status, err_code) for ALL jobs."""
        owner = assign_jobs([len(s) for s, _ in jobs], self.world)
        mine = [j for j, r in enumerate(owner) if r == self.rank]
        my_sets = [st for j in mine for st in jobs[j][0]]
        # a job with an aggregate set, a multi-key set or an empty job goes to the per-job path
        batchable = all(len(jobs[j][0]) > 0 for j in mine) and all(len(pks) == 1 for pks, _, _ in my_sets)
        part, any_err = None, True
        if my_sets and batchable:
            part, _errs, any_err = self.backend.batch_partial(my_sets, seed=seed + self.rank)
        elif not my_sets:
            any_err = False  # nothing to contribute
        gathered = self._all_gather((part, bool(any_err)))
        parts = [p for p, _ in gathered if p is not None]
        node_ok = not any(e for _, e in gathered) and bool(parts) and self.backend.final_verify(parts)
        if node_ok:
            return ShardOutcome([(VALID, 0)] * len(jobs), True, [])
        # localise: a shard passes on its own iff it could be batched and its partial verifies
        own_ok = (not my_sets) or (part is not None and not any_err and self.backend.final_verify([part]))
        local = {}
        if not own_ok:
            res, _stats = self.backend.verify_jobs([jobs[j] for j in mine], seed=seed + 7919 * (self.rank + 1))
            local = {j: tuple(r) for j, r in zip(mine, res)}
        else:
            local = {j: (VALID, 0) for j in mine}
        merged = {}
        retried = []
        for r, d in enumerate(self._all_gather((own_ok, local))):
            ok_r, loc = d
            if not ok_r:
                retried.append(r)
            merged.update(loc)
        return ShardOutcome([merged[j] for j in range(len(jobs))], False, retried)


class GpuBackend:
    """ShardedVerifier backend on one GPU through the C ABI (lodestar_amd._native.Context)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def batch_partial(self, sets, seed=0):
        return self.ctx.batch_partial(sets, seed=seed)

    def final_verify(self, partials):
        return self.ctx.final_verify(list(partials))

    def verify_jobs(self, jobs, seed=0):
        return self.ctx.verify_jobs(jobs, seed=seed)
