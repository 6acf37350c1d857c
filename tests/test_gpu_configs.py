"""GPU parity at the BASELINE configs' sizes (BASELINE.json configs A-E) and the
drop-in jobs path's contract, through the C ABI against the C restatement of the oracle
(tests/cpu_oracle.py) and the Python oracle.  Every test here needs an MI355X.

Inputs: interop keys sk_{v mod 1024} (packages/state-transition/src/util/interop.ts:19-22,
keypairsMod reuse of state-transition/test/perf/util.ts:47-48), messages
sha256(b"lodestar-mi355x" || tag || i), signatures made on the GPU (lsg_sign, itself pinned by
the genesis KAT and golden vectors in test_gpu_parity.py).  Expected verdicts never come from
the GPU: the oracle verifies every set, and the tests first assert that constructed-valid
sets are valid to the oracle.
"""
import hashlib
import os

import pytest

from oracle.fields import R
from oracle.interop import interop_secret_key
from tests import blsdata as bd
from tests import cpu_oracle as co

pytestmark = pytest.mark.gpu
N_KEYS = 1024


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd._native import Context
    c = Context(0)  # raises NativeUnavailable loudly if the HIP library or the GPU is missing
    yield c
    c.close()


@pytest.fixture(scope="module")
def keys(ctx):
    sks = [interop_secret_key(i) for i in range(N_KEYS)]
    return sks, ctx.sk_to_pk(sks)


def msgs_for(tag, n, base=0):
    return [hashlib.sha256(b"lodestar-mi355x" + tag + (base + i).to_bytes(8, "little")).digest() for i in range(n)]


def single_sets(ctx, keys, tag, n):
    sks, pks = keys
    msgs = msgs_for(tag, n)
    sigs = ctx.sign([sks[i % N_KEYS] for i in range(n)], msgs)
    return [([pks[i % N_KEYS]], msgs[i], sigs[i]) for i in range(n)]


def corrupt(ctx, keys, sets, frac, seed):
    """Config E: a fraction of the sets corrupted, split evenly over the five kinds of
    SURVEY.md 8d (wrong message, flipped x bit, truncated, non-subgroup point, infinity)."""
    import random
    rng = random.Random(seed)
    out = list(sets)
    idx = sorted(rng.sample(range(len(sets)), max(5, int(len(sets) * frac))))
    for k, i in enumerate(idx):
        out[i] = bd.CORRUPTIONS[k % len(bd.CORRUPTIONS)](out[i])
    return out, idx


def oracle_each(sets):
    return co.verify_each([p[0] for p, _, _ in sets], [m for _, m, _ in sets], [s for _, _, s in sets])


def run_jobs(ctx, jobs, seed=0):
    got, stats = ctx.verify_jobs(jobs, seed=seed)
    return got, stats


def check_against_oracle(ctx, jobs, per_set, seed=0):
    jsets, pos = [], 0
    for sets, _ in jobs:
        jsets.append(list(range(pos, pos + len(sets))))
        pos += len(sets)
    exp, retries, success = co.expected_jobs(jsets, [bool(f & 1) for _, f in jobs], per_set)
    got, stats = run_jobs(ctx, jobs, seed=seed)
    bad = [(j, g, e) for j, (g, e) in enumerate(zip(got, exp)) if (g[0], g[1] if g[0] == 2 else 0) != e]
    assert not bad, bad[:10]
    assert stats["batch_retries"] == retries and stats["batch_sigs_success"] == success, (stats, retries, success)
    return got, stats


# ---- config A: gossip-128 -- 128 single sets (BlsSingleThreadVerifier path, singleThread.ts:14-35)
def test_config_a_gossip_128(ctx, keys):
    sets = single_sets(ctx, keys, b"cfgA", 128)
    per = oracle_each(sets)
    assert per == [1] * 128
    assert ctx.verify_sets(sets) == (1, 0)  # maybeBatch over one call (lsg_verify_sets)
    bad, idx = corrupt(ctx, keys, sets, 0.02, 1)
    per_bad = oracle_each(bad)
    exp_err = next((-v for v in per_bad if v < 0), None)
    assert ctx.verify_sets(bad)[0] == (2 if exp_err else 0)
    # the same 128 sets as 128 batchable single-set jobs (worker.ts chunks of 16)
    check_against_oracle(ctx, [([s], 1) for s in sets], per)
    check_against_oracle(ctx, [([s], 1) for s in bad], per_bad)


# ---- config B: sync-committee contribution -- one 512-key aggregate set, same message
def test_config_b_sync_contribution_512(ctx, keys):
    from oracle.verifier import sk_to_pk
    from oracle.curves import g1_serialize
    sks, pks = keys
    members = list(range(7, 7 + 512))
    m = msgs_for(b"cfgB", 1)[0]
    agg_sk = sum(sks[k % N_KEYS] for k in members) % R
    sig = ctx.sign([agg_sk], [m])[0]
    agg_pk = g1_serialize(sk_to_pk(agg_sk))  # the oracle's aggregate key: (sum sk) G1
    assert co.verify_each([agg_pk], [m], [sig]) == [1]
    assert ctx.aggregate_pubkeys([pks[k % N_KEYS] for k in members]) == (agg_pk, 0)
    s = ([pks[k % N_KEYS] for k in members], m, sig)
    assert ctx.verify_sets([s]) == (1, 0)
    assert ctx.verify_sets([(s[0][:-1], m, sig)]) == (0, 0)  # one signer missing
    # verifySignatureSetsSameMessage shape: 32 contributions of one message, one forged
    ms = [([pks[i]], m, x) for i, x in enumerate(ctx.sign(sks[:32], [m] * 32))]
    ms[9] = (ms[9][0], m, ms[10][2])
    per = oracle_each(ms)
    assert per.count(0) == 1 and per[9] == 0
    check_against_oracle(ctx, [([x], 1) for x in ms], per)


# ---- config C: block body -- 128 aggregate sets of ~450 keys by index, distinct messages
@pytest.fixture(scope="module")
def table_ctx(keys):
    from lodestar_amd._native import Context
    c = Context(0)
    assert c.pubkey_table_set(0, keys[1]) == [0] * N_KEYS
    yield c
    c.close()


def test_config_c_block_128x450(table_ctx, keys):
    from lodestar_amd._native import PkIndices
    from oracle.verifier import sk_to_pk
    from oracle.curves import g1_serialize
    sks, _ = keys
    c = table_ctx
    n = 128
    idx, agg_sk = [], []
    for g in range(n):
        size = 440 + (g * 7) % 21
        start = (g * 53) % N_KEYS
        ix = [(start + j) % N_KEYS for j in range(size)]
        idx.append(ix)
        agg_sk.append(sum(sks[k] for k in ix) % R)
    msgs = msgs_for(b"cfgC", n)
    sigs = c.sign(agg_sk, msgs)
    agg_pks = [g1_serialize(sk_to_pk(k)) for k in agg_sk]
    per = co.verify_each(agg_pks, msgs, sigs)
    assert per == [1] * n
    sets = [(PkIndices(idx[g]), msgs[g], sigs[g]) for g in range(n)]
    # verifyBlocksSignatures.ts:37: one non-batchable job per block (<= 128 sets)
    got, stats = c.verify_jobs([(sets, 0)])
    assert got == [(1, 0)]
    wrong = list(sets)
    wrong[77] = (wrong[77][0], msgs[76], wrong[77][2])
    assert co.verify_each([agg_pks[77]], [msgs[76]], [sigs[77]]) == [0]
    got, _ = c.verify_jobs([(wrong[:64], 0), (wrong[64:], 0)])
    assert got == [(1, 0), (0, 0)]
    # the aggregated keys themselves, bit-exact against the oracle's (sum sk) G1: all 128 sets
    # (57k keys) in one pass of the shipped library's fused gather + mixed-addition fold
    # (k_pk_agg_seg; the batch-affine tree is A/B-build only), and a few one set at a time
    assert c.aggregate_pubkeys_multi([PkIndices(ix) for ix in idx]) == [(agg_pks[g], 0) for g in range(n)]
    for g in (0, 77, 127):
        assert c.aggregate_pubkeys(PkIndices(idx[g])) == (agg_pks[g], 0)


# ---- config D: firehose shard -- a 4096-set package, one RLC group
def test_config_d_4096_package(ctx, keys):
    sets = single_sets(ctx, keys, b"cfgD", 4096)
    per = oracle_each(sets)
    assert per == [1] * 4096
    got, stats = run_jobs(ctx, [([s], 1) for s in sets])
    assert got == [(1, 0)] * 4096
    assert stats["batch_retries"] == 0 and stats["batch_sigs_success"] == 4096
    assert stats["n_final_exps"] == 1  # the package group answers all 4096 jobs
    part, errs, anyerr = ctx.batch_partial(sets)
    assert not anyerr and ctx.final_verify([part])
    bad = list(sets)
    bad[3001] = bd.corrupt_wrong_message(bad[3001])
    per_bad = oracle_each(bad)
    assert per_bad.count(0) == 1
    _, stats = check_against_oracle(ctx, [([s], 1) for s in bad], per_bad)
    assert stats["batch_retries"] == 1 and stats["batch_sigs_success"] == 4096 - 16
    part_b, _, _ = ctx.batch_partial(bad)
    assert not ctx.final_verify([part_b])


# ---- config E: adversarial -- a 4096-set package at 1% corruption through the retry path
def test_config_e_adversarial_4096(ctx, keys):
    sets = single_sets(ctx, keys, b"cfgE", 4096)
    bad, idx = corrupt(ctx, keys, sets, 0.01, 7)
    per = oracle_each(bad)
    assert all(per[i] == 1 for i in range(4096) if i not in set(idx))
    check_against_oracle(ctx, [([s], 1) for s in bad], per)
    # mixed shape: multi-set jobs, non-batchable jobs
    jobs, pos, jper = [], 0, []
    while pos < 1024:
        n = 1 + (pos % 3)
        jobs.append((bad[pos:pos + n], 0 if pos % 5 == 0 else 1))
        pos += n
    check_against_oracle(ctx, jobs, per[:pos])


def test_thrown_chunk_localises_its_live_jobs(ctx, keys):
    """A chunk whose batch throws (an undecodable signature) is checked as one group of its
    other jobs; a thrown job's remaining sets still take part, so a failing Miller-item group
    whose only live job shares it with a thrown job must not convict that job (found by the
    10^7 soak, pkg_resolve phase C1).  The package has more than 8192 distinct messages (so its
    group keeps per-set Miller items) and more than 2048 sets (four-set items, k_miller_fused):
    sets 0-3 = job [truncated, wrong message, valid] + job [valid] form one item.  Verdicts and
    batch counters against the oracle's worker.ts rules (multithread/worker.ts:51-96); the
    untouched sets are valid by construction (GPU-signed), the corrupted ones by the oracle."""
    n = 8400
    sets = single_sets(ctx, keys, b"thrown", n)
    s = list(sets)
    starts = (0, 64, 640, 5200)
    for base in starts:
        s[base] = bd.corrupt_truncate(s[base])
        s[base + 1] = bd.corrupt_wrong_message(s[base + 1])
    lone = (300, 301, 7800)
    for i in lone:
        s[i] = bd.corrupt_wrong_message(s[i])
    per = [1] * n
    touched = sorted(set(lone) | {b + k for b in starts for k in (0, 1)})
    for i, v in zip(touched, oracle_each([s[i] for i in touched])):
        per[i] = v
    jobs, pos = [], 0
    while pos < n:
        k = 3 if pos in starts else 1
        jobs.append((s[pos:pos + k], 1))
        pos += k
    check_against_oracle(ctx, jobs, per)


def test_phase_b0_runs_localise_like_chunks(ctx, keys):
    """Phase B0 (lsg_host.hip pkg_resolve): a failing package of 2048 single-set jobs (128
    chunks of 16) is first checked as 32 runs of four chunks; only the chunks of a failing run
    are checked on their own.  An invalid set in chunk 5, an undecodable one in chunk 9 (its run
    passes: the thrown set is the identity, as in the chunk's own group) and an invalid set at
    the end of chunk 63 (the last chunk of run 15): per-job verdicts and batch counters equal
    the oracle's worker.ts rules (multithread/worker.ts:51-96), with fewer final
    exponentiations than the 1 + 128 chunk checks alone would take."""
    n = 2048
    s = list(single_sets(ctx, keys, b"b0runs", n))
    touched = (5 * 16 + 3, 9 * 16 + 7, 63 * 16 + 15)
    s[touched[0]] = bd.corrupt_wrong_message(s[touched[0]])
    s[touched[1]] = bd.corrupt_truncate(s[touched[1]])
    s[touched[2]] = bd.corrupt_wrong_message(s[touched[2]])
    per = [1] * n
    for i, v in zip(touched, oracle_each([s[i] for i in touched])):
        per[i] = v
    assert per[touched[0]] == 0 and per[touched[1]] < 0 and per[touched[2]] == 0
    _, stats = check_against_oracle(ctx, [([x], 1) for x in s], per)
    assert stats["n_final_exps"] < 1 + 128, stats


def test_one_wave_programs_in_wide_fallback_phases(ctx, keys):
    """Fallback phases of more than 128 groups run the one-wave straight-line programs with
    typed steps (lsg_slp.hip slp_waves, tools/gen_slp.py TYPED_PROGRAMS).  One invalid set in
    every run of four chunks of a 4096-job package: every B0 run fails, so phase B checks all
    256 chunks, C1 256 item groups and C2 the 256 jobs of the failing items -- each a one-wave
    launch.  Verdicts and batch counters against the oracle's worker.ts rules."""
    n = 4096
    s = list(single_sets(ctx, keys, b"w1progs", n))
    bad = [64 * k + (k * 7) % 64 for k in range(n // 64)]
    for i in bad:
        s[i] = bd.corrupt_wrong_message(s[i])
    per = [1] * n
    for i, v in zip(bad, oracle_each([s[i] for i in bad])):
        per[i] = v
    assert all(per[i] == 0 for i in bad)
    _, stats = check_against_oracle(ctx, [([x], 1) for x in s], per)
    assert stats["n_final_exps"] > 1 + 64 + 128, stats  # B alone is 256 groups


def test_package_group_matches_chunk_mode(ab_ctx, keys, monkeypatch):
    """The one-group phase A (default) and the reference's chunk-16 phase A
    (LSG_PACKAGE_GROUP=0, A/B build) give identical per-job verdicts AND batch_retries /
    batch_sigs_success, on a valid and on an adversarial package."""
    ctx = ab_ctx
    sets = single_sets(ctx, keys, b"modes", 600)
    bad, _ = corrupt(ctx, keys, sets, 0.02, 3)
    for pkg in (sets, bad):
        jobs = [([s], 1) for s in pkg[:300]] + [(pkg[300 + 2 * k:302 + 2 * k], 1 if k % 4 else 0) for k in range(150)]
        out = {}
        for mode in ("1", "0"):
            monkeypatch.setenv("LSG_PACKAGE_GROUP", mode)
            got, stats = ctx.verify_jobs(jobs, seed=17)
            out[mode] = (got, stats["batch_retries"], stats["batch_sigs_success"])
        assert out["1"] == out["0"]


def test_reserve_then_no_allocations(ctx, keys, capfd, monkeypatch):
    """lsg_reserve sizes every buffer up front: steady-state submissions allocate nothing
    (no hipMalloc / hipHostMalloc / hipFree in the submit path).  Any
    allocation is traced (LSG_TRACE_ALLOC) into the failure message."""
    sets = single_sets(ctx, keys, b"resv", 2048)
    from lodestar_amd._native import PreparedJobs
    pj = PreparedJobs([([s], 1) for s in sets])
    ctx.reserve(4096, n_slots=0)
    monkeypatch.setenv("LSG_TRACE_ALLOC", "1")
    capfd.readouterr()
    before = ctx.allocation_count()
    for rep in range(2):
        tickets = [ctx.submit_jobs(pj) for _ in range(4)]
        for t in tickets:
            res, stats = ctx.wait_jobs(t)
            assert res == [(1, 0)] * 2048
    trace = [ln for ln in capfd.readouterr().err.splitlines() if "lsg alloc" in ln]
    assert ctx.allocation_count() == before, trace


def test_node_mode_partials(ctx, keys):
    """One-process-per-GPU protocol (lsg_jobs_partial / lsg_wait_jobs_node): the package
    partial verifies alone, a forged package's does not, and the node verdict drives the
    resolution exactly as the package's own check would."""
    sets = single_sets(ctx, keys, b"node", 300)
    bad = list(sets)
    bad[10] = bd.corrupt_wrong_message(bad[10])
    for pkg, ok in ((sets, True), (bad, False)):
        jobs = [([s], 1) for s in pkg]
        t = ctx.submit_jobs(jobs)
        part, has = ctx.jobs_partial(t)
        assert has and ctx.final_verify([part]) == ok
        got, stats = ctx.wait_jobs_node(t, 1 if ok else 0)
        assert [g[0] for g in got] == [0 if (not ok and i == 10) else 1 for i in range(300)]
    # a package without batchable sets contributes the identity partial
    t = ctx.submit_jobs([(sets[:3], 0)])
    part, has = ctx.jobs_partial(t)
    assert not has and ctx.final_verify([part])
    assert ctx.wait_jobs_node(t, 1)[0] == [(1, 0)]


def test_multi_device_context_duplicate_ids(keys):
    """lsg_init_devices over [0, 0] (the copy exchange; distinct ids use RCCL): whole jobs per
    device, the gathered node check, and localisation give the single-device verdicts."""
    from lodestar_amd._native import Context
    c1 = Context(0)
    c2 = Context(devices=[0, 0])
    try:
        assert c2.device_count() == 2
        sets = single_sets(c1, keys, b"multi", 512)
        bad, _ = corrupt(c1, keys, sets, 0.02, 5)
        per = oracle_each(bad)
        jobs = [([s], 1) for s in bad[:256]] + [(bad[256 + 4 * k:260 + 4 * k], 1) for k in range(64)]
        g1, s1 = c1.verify_jobs(jobs, seed=3)
        g2, s2 = c2.verify_jobs(jobs, seed=3)
        assert g1 == g2
        check_against_oracle(c2, jobs, per)
        good = [([s], 1) for s in sets]
        g, st = c2.verify_jobs(good)
        assert g == [(1, 0)] * 512 and st["batch_retries"] == 0
        # the node check over both devices' partials decides -- ONE final
        # exponentiation for a passing package (the devices' own checks are not launched)
        assert st["n_final_exps"] == 1, st
        # a lone batchable set per device: both randomised (a multi-device partial leaves its
        # slot), and an offset forgery split over the two devices is still rejected
        from tests.test_gpu_parity import _offset_pair
        fa, fb = _offset_pair(940, "multi-offs")
        g, st = c2.verify_jobs([([fa], 1), ([fb], 1)])
        assert g == [(0, 0), (0, 0)], (g, st)
    finally:
        c2.close()
        c1.close()


def test_rccl_exchange_single_device(keys, monkeypatch):
    """The RCCL all-gather path of lsg_init_devices exercised on one GPU
    (LSG_FORCE_EXCHANGE=1, A/B build: a one-rank communicator, the node check on the gathered
    partial, which decides: a passing package runs ONE final exponentiation, the node's)."""
    from lodestar_amd._native import AB_LIB_PATH, Context
    monkeypatch.setenv("LSG_FORCE_EXCHANGE", "1")
    c = Context(devices=[0], lib=AB_LIB_PATH)
    try:
        sets = single_sets(c, keys, b"rccl", 256)
        bad = list(sets)
        bad[5] = bd.corrupt_wrong_message(bad[5])
        g, st = c.verify_jobs([([s], 1) for s in sets])
        assert g == [(1, 0)] * 256 and st["n_final_exps"] == 1  # the node FE only
        g, st = c.verify_jobs([([s], 1) for s in bad])
        assert [x[0] for x in g] == [0 if i == 5 else 1 for i in range(256)]
        assert st["n_final_exps"] >= 2  # node check failed: the device's own check localises
    finally:
        c.close()


# ---- the fused Miller kernel (lines in LDS, four waves per item) and the one-set straight-line
# program items against the split kernels
@pytest.mark.parametrize("n", [1, 3, 4, 5, 37, 300])
def test_fused_miller_matches_split(ab_ctx, keys, n, monkeypatch):
    ctx = ab_ctx  # (A/B build: LSG_MILLER_FUSED, LSG_SLP_ITEMS)
    sets = single_sets(ctx, keys, b"fused", n)
    monkeypatch.setenv("LSG_MILLER_FUSED", "0")
    split, _, _ = ctx.batch_partial(sets, seed=11)
    monkeypatch.setenv("LSG_MILLER_FUSED", "1")
    monkeypatch.setenv("LSG_SLP_ITEMS", "0")
    fused, _, _ = ctx.batch_partial(sets, seed=11)
    names = [k for k, _ in ctx.last_kernel_times()]
    assert "k_miller_fused" in names and "k_miller_lines" not in names
    assert fused == split
    # one-set Miller items as straight-line programs (the small-package default)
    monkeypatch.setenv("LSG_SLP_ITEMS", "4096")
    slp, _, _ = ctx.batch_partial(sets, seed=11)
    names = [k for k, _ in ctx.last_kernel_times()]
    assert "k_slp_items1" in names and "k_miller_fused" not in names
    assert slp == split
    assert ctx.verify_sets(sets) == (1, 0)


def test_fresh_context_mostly_invalid_single_jobs(keys):
    """the per-job phase of a package whose retried jobs outnumber phase A's
    fallback buffer (single-set batchable jobs, most of them invalid) on a context that never
    called lsg_reserve -- verdicts and counters against the C oracle."""
    from lodestar_amd._native import Context
    for n, frac in ((32, 0.75), (200, 0.7)):
        c = Context(0)
        try:
            sets = single_sets(c, keys, b"mostbad%d" % n, n)
            bad = [bd.corrupt_wrong_message(s) if (i * 7919) % 100 < frac * 100 else s for i, s in enumerate(sets)]
            per = oracle_each(bad)
            assert per.count(0) >= n // 2
            check_against_oracle(c, [([s], 1) for s in bad], per)
            # two bad signatures in different 16-job chunks of an otherwise valid package
            two = list(sets)
            for i in (3, n - 2):
                two[i] = bd.corrupt_wrong_message(two[i])
            check_against_oracle(c, [([s], 1) for s in two], oracle_each(two))
        finally:
            c.close()


def test_multi_device_bad_key_rejects_package(keys):
    """a key that does not deserialize on device 1 of a [0, 0] context
    rejects EVERY job of the package (worker.ts:41-43 throws out of verifyManySignatureSets),
    with the first bad key's code in caller order, exactly as on one device."""
    from lodestar_amd._native import Context
    c1 = Context(0)
    c2 = Context(devices=[0, 0])
    try:
        sets = single_sets(c1, keys, b"badkey", 64)
        jobs = [([s], 1) for s in sets[:32]] + [(sets[32 + 2 * k:34 + 2 * k], 1 if k % 3 else 0) for k in range(16)]
        pk = bytearray(jobs[40][0][0][0][0])
        pk[95] ^= 1  # off the curve: BLST_POINT_NOT_ON_CURVE
        s0 = jobs[40][0][0]
        jobs[40] = ([([bytes(pk)], s0[1], s0[2])] + list(jobs[40][0][1:]), jobs[40][1])
        from lodestar_amd._native import assign_jobs
        owner = assign_jobs([len(j[0]) for j in jobs], 2)
        for c in (c1, c2):
            got, st = c.verify_jobs(jobs, seed=5)
            assert got == [(2, 2)] * len(jobs), got
            assert st["key_error"] == 2 and st["key_error_job"] == 40
        assert owner[40] == 1 and owner[0] == 0
    finally:
        c2.close()
        c1.close()


def test_node_mode_partials_device_resident(ctx, keys):
    """The one-process-per-GPU exchange without a host round trip (lsg_jobs_partial_device /
    lsg_final_submit_device over torch device buffers, as bench.py's RCCL path uses them): same
    partial bytes as the host copy, same node verdicts."""
    import torch
    sets = single_sets(ctx, keys, b"nodedev", 200)
    bad = list(sets)
    bad[77] = bd.corrupt_wrong_message(bad[77])
    for pkg, ok in ((sets, True), (bad, False)):
        t = ctx.submit_jobs([([s], 1) for s in pkg])
        host, has = ctx.jobs_partial(t)
        dev = torch.empty(3 * 576, dtype=torch.uint8, device="cuda:0")
        assert ctx.jobs_partial_device(t, dev.data_ptr()) == has
        dev[576:1152].copy_(dev[:576])  # a 3-rank "gather": this partial and two identities
        one = bytearray(576)
        one[47] = 1
        dev[1152:].copy_(torch.tensor(list(one), dtype=torch.uint8))
        torch.cuda.synchronize()
        assert bytes(dev[:576].cpu().numpy().tobytes()) == host
        assert ctx.final_wait(ctx.final_submit_device(dev[576:].data_ptr(), 2)) == ok
        got, _ = ctx.wait_jobs_node(t, 1 if ok else 0)
        assert [g[0] for g in got] == [0 if (not ok and i == 77) else 1 for i in range(200)]


# ---- coalesced launches (lsg_set_coalesce): many small packages in one launch, each with the
# reference's per-package semantics (multithread/index.ts:335 one package per worker,
# worker.ts:30-106 chunks, retries and the deserializeSet rule)
def test_coalesced_packages_match_separate_launches(keys):
    from lodestar_amd._native import Context
    c, ref = Context(0), Context(0)
    try:
        sets = single_sets(c, keys, b"coalesce", 260)
        bad, _ = corrupt(c, keys, sets, 0.03, 11)
        pk = bytearray(bad[200][0][0])
        pk[95] ^= 1  # off the curve: rejects every job of ITS package only
        badkey = ([bytes(pk)], bad[200][1], bad[200][2])
        pkgs = [
            [([s], 1) for s in bad[0:40]],                                  # gossip-like, some bad
            [(bad[40 + 5 * k:45 + 5 * k], 0) for k in range(3)],            # non-batchable jobs
            [([s], 1) for s in sets[60:80]],                                # all valid
            [([s], 1) for s in bad[180:200]] + [([badkey], 1)],             # a bad key
            [(sets[80:81], 1)],                                             # one set
            [(bad[81:114], 1), (sets[114:118], 0), ([], 1)],                # multi-set, mixed, empty
            [([s], 1) for s in bad[120:180]],                               # 60 jobs: 3 chunks
            [],                                                             # no jobs
        ]
        c.set_coalesce(4096, 1)  # one launch in flight: the rest wait and go out together
        tickets = [c.submit_jobs(p, seed=0) for p in pkgs]
        assert all(t is not None for t in tickets)
        got = {}
        for i in (3, 0, 7, 5, 1, 6, 2, 4):  # waits in any order
            got[i] = c.wait_jobs(tickets[i])
        for i, p in enumerate(pkgs):
            exp, est = ref.verify_jobs(p)
            res, st = got[i]
            assert res == exp, (i, res, exp)
            for k in ("batch_retries", "batch_sigs_success", "key_error", "key_error_job"):
                assert st[k] == est[k], (i, k, st[k], est[k])
        assert got[3][0] == [(2, 2)] * len(pkgs[3])
        # the oracle decides the packages without a bad key
        for i in (0, 2, 6):
            flat = [s for js, _ in pkgs[i] for s in js]
            exp, retries, success = co.expected_jobs([[k] for k in range(len(flat))], [True] * len(flat), oracle_each(flat))
            res, st = got[i]
            assert [(g[0], g[1] if g[0] == 2 else 0) for g in res] == exp
            assert (st["batch_retries"], st["batch_sigs_success"]) == (retries, success)
        # off again: later packages launch on their own
        c.set_coalesce(0, 1)
        t = c.submit_jobs(pkgs[2])
        assert t[0] >> 8 & 255 == 1 and c.wait_jobs(t)[0] == [(1, 0)] * 20
    finally:
        c.close()
        ref.close()


def test_held_merged_ticket_reports_busy(keys):
    """A coalesced package held while every pipeline slot is taken by un-waited tickets: its
    wait returns LSG_ERR_BUSY (the ticket stays live), and after another ticket's wait frees a
    slot the same wait launches and resolves it (the waiter used to get
    LSG_ERR_INVALID_ARG for a ticket that was still pending)."""
    from lodestar_amd._native import Context, LSG_ERR_BUSY
    c = Context(0)
    try:
        sets = single_sets(c, keys, b"busy", 6)
        c.set_coalesce(4, c.pipeline_slots())  # packages of > 4 sets launch on their own
        direct = []
        while True:
            t = c.submit_jobs([([s], 1) for s in sets[:5]])
            if t is None:
                break
            direct.append(t)
            assert len(direct) <= c.pipeline_slots()
        assert len(direct) == c.pipeline_slots()
        held = c.submit_jobs([([sets[5]], 1)])  # coalesced: held, no slot for it
        assert held is not None
        with pytest.raises(RuntimeError, match=r"\(%d\)" % LSG_ERR_BUSY):
            c.wait_jobs(held)
        assert c.wait_jobs(direct[0])[0] == [(1, 0)] * 5
        assert c.wait_jobs(held)[0] == [(1, 0)]
        for t in direct[1:]:
            assert c.wait_jobs(t)[0] == [(1, 0)] * 5
    finally:
        c.close()


def _splitmix(seed, n):
    M = (1 << 64) - 1
    s, out = seed, []
    while len(out) < n:
        s = (s + 0x9E3779B97F4A7C15) & M
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        if z:
            out.append(z)
    return out


@pytest.mark.parametrize("n", [1, 7, 264])
def test_shipped_jobs_partial_bit_exact_vs_oracle(ctx, keys, n):
    """The 576 bytes the SHIPPED library exports for the node exchange (lsg_jobs_partial, what
    crosses RCCL in SURVEY.md 8e) equal the oracle's partial byte for byte under the seeded
    splitmix randomizers: 264 sets take the bucket-MSM signature sum (groups >= 256), 7 the
    per-set scaling, and a lone set is exported unscaled then raised to its own randomizer
    (lsg_host.hip export_partial_dev)."""
    from oracle import verifier as ov
    from oracle.fields import f12_coeffs, f12_pow
    sets = single_sets(ctx, keys, b"xport%d" % n, n)
    seed = 0x5eed0000 + n
    t = ctx.submit_jobs([([s], 1) for s in sets], seed=seed)
    part, has = ctx.jobs_partial(t)
    assert has
    flat = [(p[0], m, s) for p, m, s in sets]
    if n == 1:
        exp, errs = ov.batch_partial(flat, [1])
        exp = f12_pow(exp, _splitmix(seed ^ 0x5851F42D4C957F2D, 1)[0])
    else:
        exp, errs = ov.batch_partial(flat, _splitmix(seed, n))
    assert errs == [0] * n
    want = b"".join(int(c[0]).to_bytes(48, "big") + int(c[1]).to_bytes(48, "big") for c in f12_coeffs(exp))
    assert part == want
    assert ctx.wait_jobs_node(t, 1)[0] == [(1, 0)] * n


def test_merged_nonbatchable_group_matches_per_job(ab_ctx, keys, monkeypatch):
    """A package's non-batchable jobs verified as one RLC group (default) and one group per job
    (LSG_NB_MERGE=0, A/B build) give identical per-job verdicts and counters, against the
    oracle's worker.ts:88-96 rules: a valid package takes one final exponentiation for all of
    its non-batchable jobs; a failing merged group is localised job by job (an invalid set, a
    one-set invalid job, an undecodable signature, an empty job, 300 sets in one job so the
    merged group takes the bucket MSM)."""
    ctx = ab_ctx
    sets = single_sets(ctx, keys, b"nbmerge", 340)
    sizes = [1, 2, 5, 300, 3, 1, 4, 8, 16]
    def jobs_of(ss):
        out, pos = [], 0
        for n in sizes:
            out.append((ss[pos:pos + n], 0))
            pos += n
        return out
    valid = jobs_of(sets)
    bad = list(sets)
    bad[3] = bd.corrupt_wrong_message(bad[3])      # job 2 (5 sets): invalid
    bad[311] = bd.corrupt_wrong_message(bad[311])  # job 5 (one set): invalid
    bad[320] = bd.corrupt_truncate(bad[320])       # job 7: undecodable -> LSG_ERROR
    mixed = jobs_of(bad) + [([], 0)] + [([s], 1) for s in sets[330:340]]
    for jobs, exp_fe in ((valid, 1), (mixed, None)):
        out = {}
        for merge in ("1", "0"):
            monkeypatch.setenv("LSG_NB_MERGE", merge)
            got, stats = ctx.verify_jobs(jobs, seed=23)
            out[merge] = (got, stats["batch_retries"], stats["batch_sigs_success"])
            if merge == "1" and exp_fe is not None:
                assert stats["n_final_exps"] == exp_fe, stats
        assert out["1"] == out["0"]
        flat = [s for js, _ in jobs for s in js]
        jsets, pos = [], 0
        for js, _ in jobs:
            jsets.append(list(range(pos, pos + len(js))))
            pos += len(js)
        exp, retries, success = co.expected_jobs(jsets, [bool(f & 1) for _, f in jobs], oracle_each(flat))
        got = out["1"][0]
        assert [(g[0], g[1] if g[0] == 2 else 0) for g in got] == exp
        assert out["1"][1:] == (retries, success)


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]], ids=["one-device", "three-duplicate-ids"])
def test_concurrent_submitters_match_oracle(keys, devices):
    """Packages are staged with the context lock released (lsg_host.hip submit_pkg / stage_pkg):
    four host threads submit and wait mixed packages at once -- on a one-device context and on
    one over three duplicate ids, whose devices' shares stage on threads of their own -- while a
    fifth thread rewrites the pubkey table that the packages' index sets read (it waits for the
    packages being staged).  Every job's verdict and every package's batch counters must be the
    oracle's (worker.ts:30-106) -- the counters over each device's share of the jobs."""
    import threading
    from lodestar_amd._native import Context, PkIndices, assign_jobs
    c0 = Context(0)
    c = Context(devices=devices)
    try:
        sks, pks = keys
        assert c.pubkey_table_set(0, pks) == [0] * N_KEYS
        sets = single_sets(c0, keys, b"concurrent", 1024)
        bad, _ = corrupt(c0, keys, sets, 0.03, 11)
        per = oracle_each(bad)
        packages = []
        for t in range(8):
            chunk = list(range(128 * t, 128 * t + 128))
            js = [[i] for i in chunk[:48]]                                   # gossip singles
            js += [chunk[48 + 4 * k:52 + 4 * k] for k in range(16)]          # 4-set batches
            js += [[i] for i in chunk[112:124]]                              # singles by validator index
            js += [chunk[124:128]]                                           # one non-batchable job
            flags = [1] * (len(js) - 1) + [0]
            jobs = []
            for q, idx in enumerate(js):
                if 64 <= q < 76:  # the index-named singles
                    i = idx[0]
                    jobs.append(([(PkIndices([i % N_KEYS]), bad[i][1], bad[i][2])], flags[q]))
                else:
                    jobs.append(([bad[i] for i in idx], flags[q]))
            # verdicts are the package's whatever the split; the batch counters are those of each
            # device's share of whole jobs (lsg_assign_jobs), chunked on its own, as a reference
            # pool's counters are those of each worker's jobs (multithread/index.ts:400-418)
            owner = assign_jobs([len(idx) for idx in js], len(devices))
            verd, retries, success = [None] * len(js), 0, 0
            for d in range(len(devices)):
                mine = [q for q in range(len(js)) if owner[q] == d]
                flat = [i for q in mine for i in js[q]]
                pos = {i: k for k, i in enumerate(flat)}
                e, r, sc = co.expected_jobs([[pos[i] for i in js[q]] for q in mine], [bool(flags[q]) for q in mine],
                                            [per[i] for i in flat])
                for q, v in zip(mine, e):
                    verd[q] = v
                retries += r
                success += sc
            packages.append((jobs, (verd, retries, success)))
        errors = []
        stop = threading.Event()

        def submitter(k):
            try:
                for rep in range(3):
                    jobs, (exp, retries, success) = packages[(2 * k + rep) % len(packages)]
                    got, st = c.verify_jobs(jobs)
                    got = [(s, e if s == 2 else 0) for s, e in got]
                    if got != exp:
                        errors.append(("verdicts", k, rep, [(j, g, x) for j, (g, x) in enumerate(zip(got, exp)) if g != x][:5]))
                    if (st["batch_retries"], st["batch_sigs_success"]) != (retries, success):
                        errors.append(("counters", k, rep, st, retries, success))
            except Exception as e:  # noqa: BLE001 -- reported below
                errors.append(("raised", k, repr(e)))

        def table_writer():
            while not stop.is_set():
                if c.pubkey_table_set(0, pks) != [0] * N_KEYS:
                    errors.append(("table", "pubkey_table_set failed"))
                    return

        th = [threading.Thread(target=submitter, args=(k,)) for k in range(4)]
        tw = threading.Thread(target=table_writer)
        tw.start()
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=150)
        stop.set()
        tw.join(timeout=60)
        assert not any(t.is_alive() for t in th) and not tw.is_alive(), "a submitter or the table writer hung"
        assert not errors, errors[:5]
    finally:
        c.close()
        c0.close()
