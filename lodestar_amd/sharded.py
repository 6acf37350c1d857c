"""Node-sharded verification across the GPUs of one node, one process per GPU.

The in-process alternative is one context over every GPU (include/lodestar_bls.h
lsg_init_devices: RCCL communicators owned by the C side).  This module is the same protocol
for hosts that run one process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on
ROCm, "gloo" in the CPU tests).  For one package of jobs (BlsWorkReq[],
packages/beacon-node/src/chain/bls/multithread/types.ts:14-17) every rank:

1. takes its shard: whole jobs, never split, assigned by cumulative set count so that the
   shards are balanced (``assign_jobs``, the same rule as lsg_assign_jobs);
2. submits it (``backend.submit``): decode + subgroup check, pubkey aggregation, hash_to_G2,
   RLC scalars, Miller loops, the local ML(-G1, sum r_i sig_i) term -- every batchable set of
   the shard is one RLC group, including aggregate and multi-key sets;
3. all-gathers the 576-byte partial of that group (``backend.partial``; one collective, the
   path's only exchange step);
4. multiplies the partials and runs ONE final exponentiation (``backend.final_verify``);
5. resolves its jobs with that node verdict (``backend.resolve``): when the node check fails,
   the rank's own package check (already computed on its GPU) localises, and only a failing
   rank runs the reference's chunk / per-job fallback (worker.ts:51-96).  Per-job verdicts
   are all-gathered.  A key that does not deserialize on ANY rank rejects every job of the
   package with the code of the first bad key in caller order (worker.ts:41-43), as on one
   device.  The node verdict is advisory: a rank's own check of its share decides its jobs.

Randomizers: seed 0 means the OS CSPRNG on every rank (production); a nonzero seed (tests)
is offset per rank.

The backend is duck-typed: ``GpuBackend`` (this package, HIP through the C ABI) in production,
an oracle-backed one in the CPU tests.
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


def rank_seed(seed, rank):
    """0 stays 0 (every rank draws from the OS CSPRNG); test seeds differ per rank."""
    return seed + rank if seed else 0


@dataclass
class ShardOutcome:
    results: list          # per job: (status, err_code)
    combined_ok: bool      # the one-final-exponentiation node check passed
    retried_ranks: list    # ranks that ran the reference's batch-retry fallback
    rank_stats: list = None  # per rank: its BlsWorkResult counters for its own share


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
        h = self.backend.submit([jobs[j] for j in mine], seed=rank_seed(seed, self.rank))
        part, _has = self.backend.partial(h)
        parts = self._all_gather(part)
        node_ok = self.backend.final_verify(parts)
        res, stats = self.backend.resolve(h, 1 if node_ok else 0)
        local = {j: tuple(r) for j, r in zip(mine, res)}
        # a key that does not deserialize rejects the WHOLE package (worker.ts:41-43): the
        # first bad key in caller job order over all ranks decides the code
        kerr = stats.get("key_error", 0)
        key = (mine[stats.get("key_error_job", 0)], kerr) if kerr else None
        merged, retried, stats_all, key_errs = {}, [], [], []
        for r, (loc, st, ke) in enumerate(self._all_gather((local, stats, key))):
            if st.get("batch_retries", 0):
                retried.append(r)
            merged.update(loc)
            stats_all.append(st)
            if ke is not None:
                key_errs.append(ke)
        results = [merged[j] for j in range(len(jobs))]
        if key_errs:
            code = min(key_errs)[1]
            results = [(ERROR, code)] * len(jobs)
        return ShardOutcome(results, node_ok, retried, stats_all)


class GpuBackend:
    """ShardedVerifier backend on one GPU through the C ABI (lodestar_amd._native.Context):
    lsg_submit_jobs, lsg_jobs_partial, lsg_final_verify, lsg_wait_jobs_node."""

    def __init__(self, ctx):
        self.ctx = ctx

    def submit(self, jobs, seed=0):
        t = self.ctx.submit_jobs(jobs, seed=seed)
        if t is None:
            raise RuntimeError("every pipeline slot is busy")
        return t

    def partial(self, handle):
        return self.ctx.jobs_partial(handle)

    def final_verify(self, partials):
        return self.ctx.final_verify(list(partials))

    def resolve(self, handle, node_valid):
        return self.ctx.wait_jobs_node(handle, node_valid)
