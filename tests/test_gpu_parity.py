"""GPU parity: the HIP path (through the C ABI, lodestar_amd/liblodestar_bls.so) against the
oracle and the committed golden fixtures.  Every test here needs an MI355X.

Reference behaviour pinned (file:line under /root/reference):
- packages/beacon-node/test/e2e/chain/bls/multithread.test.ts:25-103 (3 valid sets x 8 jobs;
  a 32-byte zero signature rejects with BLST_INVALID_SIZE without poisoning co-batched jobs)
- packages/beacon-node/test/e2e/interop/genesisState.test.ts:49-56 (genesis KAT signature)
- packages/beacon-node/src/chain/bls/multithread/worker.ts:30-106 (batch + retry verdicts)
"""
import json
import os

import pytest

from oracle.curves import E1, g1_serialize, g2_serialize, g2_uncompress, BlstError, in_g2
from oracle.interop import GENESIS_KAT, genesis_deposit_signing_root, interop_secret_key
from oracle import hash_to_curve as h2c
from oracle import verifier as ov
from tests import blsdata as bd

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd._native import Context
    c = Context(0)  # raises NativeUnavailable loudly if the HIP library or the GPU is missing
    yield c
    c.close()


def oracle_job_results(jobs):
    """Expected per-job (status, err_name) from the oracle's worker.ts restatement."""
    reqs = []
    for sets, flags in jobs:
        ss = []
        for pks, m, sig in sets:
            pts = [ov.public_key_from_bytes(p) for p in pks]
            agg = ov.aggregate_pubkeys(pts)
            ss.append({"publicKey": g1_serialize(agg), "message": m, "signature": sig})
        reqs.append({"opts": {"batchable": bool(flags & 1)}, "sets": ss})
    out = ov.verify_many_signature_sets(reqs)
    res = []
    for kind, val in out["results"]:
        if kind == "success":
            res.append((1 if val else 0, None))
        else:
            res.append((2, val))
    return res, out


def check_jobs(ctx, jobs, seed=7):
    """Per-job verdicts, error messages AND the BlsWorkResult counters against the oracle's
    worker.ts restatement."""
    from lodestar_amd._native import error_message
    got, stats = ctx.verify_jobs(jobs, seed=seed)
    exp, out = oracle_job_results(jobs)
    for i, ((gs, gc), (es, emsg)) in enumerate(zip(got, exp)):
        assert gs == es, (i, got, exp)
        if es == 2:
            assert error_message(gc) == emsg or error_message(gc).split(": ")[-1] in emsg, (i, gc, emsg)
    assert stats["batch_retries"] == out["batch_retries"], (stats, out["batch_retries"])
    assert stats["batch_sigs_success"] == out["batch_sigs_success"], (stats, out["batch_sigs_success"])
    return got, stats


def test_device_is_gfx950(ctx):
    assert "gfx950" in ctx.device_name()


def test_hash_to_g2_matches_oracle_and_golden(ctx):
    gold = json.load(open(os.path.join(GOLDEN, "hash_to_g2.json")))
    msgs = [bytes.fromhex(c["msg"]) for c in gold["cases"]]
    out = ctx.hash_to_g2(msgs)
    for c, o in zip(gold["cases"], out):
        assert o.hex() == c["out"]
    extra = [bd.msg("h2c", i) for i in range(16)]
    for m, o in zip(extra, ctx.hash_to_g2(extra)):
        assert o == g2_serialize(h2c.hash_to_g2(m))


def test_sig_decode_matches_oracle(ctx):
    gold = json.load(open(os.path.join(GOLDEN, "sig_decode.json")))
    groups = {}
    for c in gold["cases"]:
        groups.setdefault(len(bytes.fromhex(c["sig"])), []).append(c)
    for ln, cases in groups.items():
        out = ctx.sig_decode([bytes.fromhex(c["sig"]) for c in cases])
        for c, (pt, err) in zip(cases, out):
            assert err == c["err"], c
            if err == 0:
                assert pt.hex() == c["point"]


def test_aggregate_pubkeys(ctx):
    gold = json.load(open(os.path.join(GOLDEN, "aggregate_pubkeys.json")))
    for c in gold["cases"]:
        pks = [bytes.fromhex(p) for p in c["pks"]]
        out, err = ctx.aggregate_pubkeys(pks)
        assert err == c["err"]
        if err == 0:
            assert out.hex() == c["out"]


def test_genesis_kat_verifies_on_gpu(ctx):
    sk = interop_secret_key(0)
    pk = bytes.fromhex(GENESIS_KAT["pubkey"])
    _, root = genesis_deposit_signing_root(pk)
    sig = bytes.fromhex(GENESIS_KAT["signature"])
    assert ctx.verify_sets([([pk], root, sig)], seed=1) == (1, 0)
    assert ctx.verify_sets([([pk], bytes(32), sig)], seed=1)[0] == 0


def test_multithread_e2e_cases(ctx):
    # multithread.test.ts:25-37: sk = 0x(i+1)^32, msg = 0x(i+1)^32, 3 sets
    from oracle.curves import g1_serialize as ser, g2_compress
    from oracle.verifier import sign, sk_to_pk
    sets = []
    for i in range(3):
        sk = int.from_bytes(bytes([i + 1]) * 32, "big")
        m = bytes([i + 1]) * 32
        sets.append(([ser(sk_to_pk(sk))], m, g2_compress(sign(sk, m))))
    for flags in (0, 1):
        got, _ = check_jobs(ctx, [(sets, flags)] * 8)
        assert all(g == (1, 0) for g in got)
    # invalid first: 32-byte zero signature, batchable, plus 8 valid batchable jobs
    bad = [(sets[0][0], sets[0][1], bytes(32))]
    got, stats = check_jobs(ctx, [(bad, 1)] + [(sets, 1)] * 8)
    assert got[0] == (2, 10)  # BLST_INVALID_SIZE
    assert all(g == (1, 0) for g in got[1:])
    assert stats["batch_retries"] == 1


def test_single_and_batch_verdicts(ctx):
    good = [bd.single_set(i) for i in range(6)]
    assert ctx.verify_sets(good[:1], seed=3) == (1, 0)
    assert ctx.verify_sets(good, seed=3) == (1, 0)
    bad = list(good)
    bad[2] = bd.corrupt_wrong_message(bad[2])
    assert ctx.verify_sets(bad, seed=3) == (0, 0)
    assert ctx.verify_sets([bad[2]], seed=3) == (0, 0)
    # infinity signature -> false, truncated -> BLST_INVALID_SIZE error
    assert ctx.verify_sets([bd.corrupt_infinity(good[0])], seed=3) == (0, 0)
    assert ctx.verify_sets([bd.corrupt_truncate(good[0])], seed=3) == (2, 10)
    assert ctx.verify_sets([bd.corrupt_not_in_group(good[0])], seed=3) == (2, 3)
    assert ctx.verify_sets([], seed=3) == (2, 100)


def test_aggregate_sets(ctx):
    sets = [bd.aggregate_set(i, list(range(5 * i, 5 * i + 5 + i))) for i in range(4)]
    assert ctx.verify_sets(sets, seed=5) == (1, 0)
    assert ctx.verify_sets(sets[:1], seed=5) == (1, 0)
    wrong = (sets[1][0][:-1], sets[1][1], sets[1][2])  # one signer missing
    assert ctx.verify_sets([sets[0], wrong], seed=5) == (0, 0)


def test_adversarial_jobs_match_oracle(ctx):
    import random
    rng = random.Random(11)
    jobs = []
    for j in range(24):
        n = rng.choice([1, 1, 2, 3])
        sets = [bd.single_set(100 + 4 * j + k) for k in range(n)]
        if rng.random() < 0.3:
            k = rng.randrange(n)
            sets[k] = bd.CORRUPTIONS[rng.randrange(len(bd.CORRUPTIONS))](sets[k])
        jobs.append((sets, 1 if rng.random() < 0.7 else 0))
    check_jobs(ctx, jobs, seed=99)


@pytest.mark.parametrize("agg", ["0", "1"])
def test_shared_messages_match_oracle(ctx, ab_ctx, monkeypatch, agg):
    """Sets that sign one message (a committee's attestations) share one hash_to_G2 per
    package (stage_sets message table, k_h2c_gather) and, with LSG_MSG_AGG=1, one Miller pair
    (the masked sum of their scaled keys): verdicts, errors and counters stay the oracle's,
    with corrupted sets inside the shared groups and sets whose corruption gives them a
    message of their own."""
    import random
    if agg == "0":  # one Miller pair per set: the A/B build's LSG_MSG_AGG=0
        monkeypatch.setenv("LSG_MSG_AGG", agg)
        ctx = ab_ctx
    rng = random.Random(5)
    msgs = [bd.msg("committee", c) for c in range(3)]
    sets = []
    for c, m in enumerate(msgs):
        for k in range(6):
            key = 300 + 6 * c + k
            sets.append(([bd.pk_bytes(key)], m, g2_serialize_compressed(bd.sig_point((key,), m))))
    jobs = [([s], 1) for s in sets]
    check_jobs(ctx, jobs, seed=21)
    bad = list(sets)
    bad[1] = bd.corrupt_wrong_message(bad[1])       # leaves its group: a message of its own
    bad[7] = bd.corrupt_infinity(bad[7])            # stays in its group
    bad[8] = (bad[8][0], bad[8][1], bad[9][2])      # another signer's signature of the same message
    bad[14] = bd.corrupt_not_in_group(bad[14])
    bad[15] = bd.corrupt_truncate(bad[15])
    jobs = [([s], 1 if rng.random() < 0.8 else 0) for s in bad]
    jobs.append((bad[12:18], 1))                    # a multi-set job inside one shared group
    check_jobs(ctx, jobs, seed=22)
    assert ctx.verify_sets(sets, seed=23) == (1, 0)
    assert ctx.verify_sets([sets[0], sets[1], bad[8]], seed=23) == (0, 0)


def g2_serialize_compressed(pt):
    from oracle.curves import g2_compress
    return g2_compress(pt)


def test_batch_partial_and_final_verify(ctx):
    sets = [bd.single_set(200 + i) for i in range(10)]
    p1, e1, a1 = ctx.batch_partial(sets[:5], seed=1)
    p2, e2, a2 = ctx.batch_partial(sets[5:], seed=2)
    assert not a1 and not a2
    assert ctx.final_verify([p1, p2])
    bad = sets[5:]
    bad[0] = bd.corrupt_wrong_message(bad[0])
    p3, _, _ = ctx.batch_partial(bad, seed=2)
    assert not ctx.final_verify([p1, p3])
    assert ctx.final_verify([p1]) and not ctx.final_verify([p3])


def _offset_pair(i, tag):
    """Two sets whose signatures are sig_a + D and sig_b - D (D in G2): each one invalid, their
    unrandomised sum valid -- the forgery an exported partial without RLC would pass."""
    from oracle.curves import E2, G2_GEN, g2_compress, g2_uncompress
    a, b = bd.single_set(i, tag=tag), bd.single_set(i + 1, tag=tag)
    D = E2.mul(G2_GEN, 123456789)
    sa = E2.add(g2_uncompress(a[2]), D)
    sb = E2.add(g2_uncompress(b[2]), E2.neg(D))
    return (a[0], a[1], g2_compress(sa)), (b[0], b[1], g2_compress(sb))


def test_one_set_shards_offset_forgery_rejected(ctx):
    """a one-set shard's exported partial keeps a random RLC coefficient.
    Two shards holding sig_a + D and sig_b - D: every local check fails, and so must the
    product of their partials -- through lsg_batch_partial and through lsg_jobs_partial(_device)
    (a lone batchable set is verified unscaled inside its package, and its partial leaves the
    slot raised to a fresh randomizer)."""
    fa, fb = _offset_pair(880, "offs")
    pa, _, ea = ctx.batch_partial([fa], seed=5)
    pb, _, eb = ctx.batch_partial([fb], seed=6)
    assert not ea and not eb
    assert not ctx.final_verify([pa]) and not ctx.final_verify([pb])
    assert not ctx.final_verify([pa, pb])
    # the jobs path: each package one batchable single-set job (the lone-set shortcut)
    parts = []
    for s in (fa, fb):
        t = ctx.submit_jobs([([s], 1)])
        part, has = ctx.jobs_partial(t)
        assert has
        parts.append(part)
        got, _ = ctx.wait_jobs(t)
        assert got == [(0, 0)]
    assert not ctx.final_verify(parts)
    # valid lone sets still pass through the randomised export
    va, vb = bd.single_set(890, tag="offs"), bd.single_set(891, tag="offs")
    parts = []
    for s in (va, vb):
        t = ctx.submit_jobs([([s], 1)])
        parts.append(ctx.jobs_partial(t)[0])
        assert ctx.wait_jobs(t)[0] == [(1, 0)]
    assert ctx.final_verify(parts)


def test_probe_rate_positive(ctx):
    fp, mad = ctx.probe_fp_mul_rate()
    assert fp > 1e9 and mad == pytest.approx(fp * 300)


def test_async_jobs_two_slots_match_sync(ctx):
    import random
    rng = random.Random(5)
    pkgs = []
    for p in range(2):
        jobs = []
        for j in range(20):
            n = rng.choice([1, 2, 3])
            sets = [bd.single_set(300 + 40 * p + 2 * j + k) for k in range(n)]
            if rng.random() < 0.25:
                k = rng.randrange(n)
                sets[k] = bd.CORRUPTIONS[rng.randrange(len(bd.CORRUPTIONS))](sets[k])
            jobs.append((sets, 1 if rng.random() < 0.8 else 0))
        pkgs.append(jobs)
    t0 = ctx.submit_jobs(pkgs[0], seed=21)
    t1 = ctx.submit_jobs(pkgs[1], seed=22)
    assert t0 is not None and t1 is not None
    extra = []
    while True:  # fill the remaining pipeline slots; then every slot is outstanding -> LSG_ERR_BUSY
        t = ctx.submit_jobs(pkgs[0], seed=23)
        if t is None:
            break
        extra.append(t)
        assert len(extra) < 64
    r1, _ = ctx.wait_jobs(t1)  # out of order
    r0, _ = ctx.wait_jobs(t0)
    for t in extra:
        assert [g[0] for g in ctx.wait_jobs(t)[0]] == [g[0] for g in r0]
    for jobs, got in ((pkgs[0], r0), (pkgs[1], r1)):
        exp, _ = oracle_job_results(jobs)
        assert [g[0] for g in got] == [e[0] for e in exp]
    assert ctx.verify_jobs(pkgs[0], seed=21)[0] == r0


def test_partials_and_async_finals(ctx):
    """lsg_batch_partial partials and the final-exponentiation entries (lsg_final_*): single,
    grouped (one launch for several groups) and empty tickets."""
    sets = [bd.single_set(400 + i) for i in range(24)]
    bad = list(sets)
    bad[13] = bd.corrupt_wrong_message(bad[13])
    parts = [ctx.batch_partial(pkg[8 * g:8 * g + 8], seed=31 + g)[0] for pkg in (sets, bad) for g in range(3)]
    expect = [True, True, True, True, False, True]
    assert [ctx.final_verify([p]) for p in parts] == expect
    assert ctx.final_wait_groups(ctx.final_submit_groups([[p] for p in parts])) == expect
    pairs = [[parts[g], parts[(g + 1) % 3]] for g in range(3)] + [[parts[3], parts[4]]]
    assert ctx.final_wait_groups(ctx.final_submit_groups(pairs)) == [True, True, True, False]
    fs = [ctx.final_submit(parts[:3]), ctx.final_submit(parts[3:]), ctx.final_submit([])]
    assert [ctx.final_wait(t) for t in fs] == [True, False, False]
    # the same sets as one partial equal the product of the three (same randomizers)
    whole = ctx.batch_partial(sets, seed=31)[0]
    assert ctx.final_verify([whole])


def test_batch_partial_excludes_errored_sets(ctx):
    sets = [bd.single_set(500 + i) for i in range(6)]
    sets[3] = bd.corrupt_truncate(sets[3])
    sets[4] = bd.corrupt_not_in_group(sets[4])
    part, errs, anyerr = ctx.batch_partial(sets, seed=9)
    assert anyerr and errs == [0, 0, 0, 10, 3, 0]
    assert ctx.final_verify([part])  # the remaining sets are valid; errored ones are identities


def test_node_host_on_gpu(ctx, tmp_path):
    """BlsGpuVerifier (Node) -> N-API addon -> C ABI on the GPU: multithread.test.ts:25-103."""
    import shutil
    import subprocess
    if shutil.which("node") is None:
        pytest.skip("node not installed")
    addon = os.path.join(HERE, "..", "lodestar_amd", "napi", "lsg_napi.node")
    assert os.path.exists(addon), "N-API addon not built"
    from oracle.curves import g1_serialize, g2_serialize
    valid = [bd.single_set(900 + i, tag="node") for i in range(3)]
    agg = bd.aggregate_set(5, [11, 12, 13], tag="node")
    wrong = bd.corrupt_wrong_message(bd.single_set(904, tag="node"))
    sm_msg = bd.msg("node-same", 0)
    sm_sets, sm_exp = [], []
    for k in range(4):
        pks, _, sig = bd.single_set(920 + k, tag="x")
        good = k != 2
        m = sm_msg if good else bd.msg("node-other", k)
        s = bd.single_set(920 + k, tag="x")
        sig = bd.g2_compress(bd.sig_point((920 + k,), m))
        sm_sets.append({"pk": pks[0].hex(), "sig": sig.hex()})
        sm_exp.append(good)
    pts = [ov.public_key_from_bytes(p) for p in agg[0]]
    h2c_msg = bd.msg("node-h2c", 0)
    dst = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"
    from oracle import interop as oi
    sr_data = bytes((7 * k + 3) & 255 for k in range(3 * 128))
    sr_dom = bytes(range(32, 64))
    cases = {
        "valid": [{"pks": [p.hex() for p in s[0]], "msg": s[1].hex(), "sig": s[2].hex()} for s in valid],
        "wrong_message": {"pks": [p.hex() for p in wrong[0]], "msg": wrong[1].hex(), "sig": wrong[2].hex()},
        "aggregate": {"pks": [p.hex() for p in agg[0]], "msg": agg[1].hex(), "sig": agg[2].hex()},
        "aggregate_pk": g1_serialize(ov.aggregate_pubkeys(pts)).hex(),
        "same_message": {"msg": sm_msg.hex(), "sets": sm_sets, "expected": sm_exp},
        "h2c": {"msg": h2c_msg.hex(), "dst": dst.decode(), "out": g2_serialize(h2c.hash_to_g2(h2c_msg, dst)).hex()},
        "signing_roots": {"data": sr_data.hex(), "domain": sr_dom.hex(),
                          "roots": b"".join(oi.attestation_signing_root(sr_data[128 * k:128 * k + 128], sr_dom)
                                            for k in range(3)).hex()},
    }
    f = tmp_path / "cases.json"
    f.write_text(json.dumps(cases))
    r = subprocess.run(["node", os.path.join(HERE, "js", "test_verifier_gpu.js"), str(f)], capture_output=True,
                       text=True, timeout=180)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr


def test_sharded_verifier_gpu_backend(ctx):
    """lodestar_amd/sharded.py on one GPU: node check passes for a valid package; a corrupted
    set localises to this rank and the per-job fallback matches the worker.ts verdicts."""
    from lodestar_amd.sharded import ShardedVerifier, GpuBackend
    sv = ShardedVerifier(GpuBackend(ctx))
    jobs = [([bd.single_set(800 + 3 * j + k, tag="sv") for k in range(1 + j % 3)], 1) for j in range(6)]
    ok = sv.verify_jobs(jobs, seed=5)
    assert ok.combined_ok and [r[0] for r in ok.results] == [1] * 6
    bad = list(jobs)
    s = list(bad[4][0])
    s[0] = bd.corrupt_wrong_message(s[0])
    bad[4] = (s, 1)
    t = list(bad[1][0])
    t[1] = bd.corrupt_truncate(t[1])
    bad[1] = (t, 1)
    out = sv.verify_jobs(bad, seed=5)
    exp, _ = oracle_job_results(bad)
    assert not out.combined_ok and out.retried_ranks == [0]
    # aggregate and multi-key sets share the batched shard (no per-job detour)
    agg = [([bd.aggregate_set(k, list(range(3 * k, 3 * k + 5)), tag="sv")], 1) for k in range(4)]
    res = sv.verify_jobs(agg + jobs, seed=0)
    assert res.combined_ok and [r[0] for r in res.results] == [1] * 10
    assert [r[0] for r in out.results] == [e[0] for e in exp]


def _splitmix_rands(seed, n):
    """The randomizers lsg_batch_partial derives from a nonzero seed on a single-device
    context (lsg_host.hip stage_sets: splitmix64, zero draws skipped)."""
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


def _f12_bytes(f):
    from oracle.fields import f12_coeffs
    return b"".join(int(c[0]).to_bytes(48, "big") + int(c[1]).to_bytes(48, "big") for c in f12_coeffs(f))


def test_msm_signature_sums_match_scalar_path(ab_ctx, monkeypatch):
    """Bucket MSM vs per-set [r_i] sig_i for the package group's signature sum: identical
    partials, including an infinite and an undecodable signature (identity contributions).
    (A/B build: LSG_MSM_MIN_GROUP.)"""
    ctx = ab_ctx
    sets = [bd.single_set(700 + i, tag="msm") for i in range(40)]
    sets[5] = bd.corrupt_infinity(sets[5])
    sets[22] = bd.corrupt_truncate(sets[22])
    sets[31] = bd.corrupt_wrong_message(sets[31])
    out = {}
    for mode, thr in (("msm", "1"), ("scalar", "1000000")):
        monkeypatch.setenv("LSG_MSM_MIN_GROUP", thr)
        part, errs, anyerr = ctx.batch_partial(sets, seed=1234)
        out[mode] = part
        assert anyerr and errs[22] == 10 and errs[5] == 0
    assert out["msm"] == out["scalar"]
    assert not ctx.final_verify([out["msm"]])  # 5: infinity sig; 31: wrong msg


def test_batch_partial_bit_exact_vs_oracle(ab_ctx, monkeypatch):
    """The per-shard Miller product (SURVEY 8e partial) equals the oracle's, byte for byte,
    with the same randomizers, through the MSM signature sum (A/B build: LSG_MSM_MIN_GROUP)."""
    ctx = ab_ctx
    monkeypatch.setenv("LSG_MSM_MIN_GROUP", "1")
    sets = [bd.single_set(760 + i, tag="msm") for i in range(7)]
    sets[2] = bd.corrupt_infinity(sets[2])
    sets[4] = bd.corrupt_not_in_group(sets[4])
    seed = 4242
    part, errs, anyerr = ctx.batch_partial(sets, seed=seed)
    rands = _splitmix_rands(seed, len(sets))
    exp, exp_errs = ov.batch_partial([(p[0], m, s) for p, m, s in sets], rands)
    assert errs == exp_errs and anyerr
    assert part == _f12_bytes(exp)


# ---- validator pubkey table resident in HBM, sets naming keys by index
# (index2pubkey, state-transition/src/cache/pubkeyCache.ts:60-75, epochContext.ts:701-704)
def _table_context(lib=None):
    from lodestar_amd._native import Context
    c = Context(0, lib=lib)
    # indices 0..23 uncompressed, 24..39 compressed (two loads, the second one past the end)
    assert c.pubkey_table_set(0, [bd.pk_bytes(i) for i in range(24)]) == [0] * 24
    assert c.pubkey_table_set(24, [bd.pk_bytes(i, compressed=True) for i in range(24, 40)]) == [0] * 16
    return c


@pytest.fixture(scope="module")
def table_ctx():
    c = _table_context()
    yield c
    c.close()


@pytest.fixture(scope="module")
def table_ab_ctx():
    from lodestar_amd._native import AB_LIB_PATH
    c = _table_context(AB_LIB_PATH)
    yield c
    c.close()


def test_pubkey_table_aggregation_by_index(table_ctx):
    from lodestar_amd._native import PkIndices, LSG_ERR_BAD_INDEX
    c = table_ctx
    assert c.pubkey_table_size() == 40
    for idx in ([7], [0, 1, 2], list(range(40)), [39, 3, 3, 17, 24]):
        out, err = c.aggregate_pubkeys(PkIndices(idx))
        assert err == 0
        assert out == g1_serialize(ov.aggregate_pubkeys([bd.pk_point(i) for i in idx])), idx
    assert c.aggregate_pubkeys(PkIndices([1, 40]))[1] == LSG_ERR_BAD_INDEX
    assert c.aggregate_pubkeys(PkIndices([]))[1] == 101  # EMPTY_AGGREGATE_ARRAY


@pytest.mark.parametrize("form", ["fold", "tree"])
def test_aggregation_tree_edge_cases(table_ctx, table_ab_ctx, monkeypatch, form):
    """PublicKey.aggregate of large packages (>= 32768 keys) against the oracle, bit-exact, in
    both forms: the shipped fused gather + mixed-addition fold (lsg_k_pk.hip k_pk_agg_seg) and
    the batch-affine tree (k_agg_*, A/B build with LSG_AGG_TREE=1), on the cases the tree's
    affine additions must route around: P + P (doubling), P + (-P) (infinity), infinity keys in
    the table, lone last points, sets summed directly (few keys), a key list of period 40 whose
    higher levels are full of equal pairs, bad indices and empty sets."""
    from lodestar_amd._native import PkIndices, LSG_ERR_BAD_INDEX
    from oracle.curves import E1, G1_GEN
    c = table_ctx
    if form == "tree":
        c = table_ab_ctx
        monkeypatch.setenv("LSG_AGG_TREE", "1")
    # rows 40 = -pk(3), 41 = the infinity key (uncompressed encoding)
    neg3 = g1_serialize(E1.neg(bd.pk_point(3)))
    assert c.pubkey_table_set(40, [neg3, bytes([0x40]) + bytes(95)]) == [0, 0]
    sk = {i: bd.sk(i) for i in range(40)}
    from oracle.fields import R as ORDER
    sk[40] = (-bd.sk(3)) % ORDER
    sk[41] = 0

    def expect(ix):
        t = sum(sk[i] for i in ix) % ORDER
        return g1_serialize(E1.mul(G1_GEN, t) if t else None)

    cases = [
        [3, 40],                          # P + (-P): infinity (final kernel)
        [3, 40] * 6 + [9],                # 13 points: six P - P pairs in a level, then 9
        [5] * 9,                          # doublings in the levels
        [5] * 16,
        [41] * 12,                        # only infinity keys
        [41, 7, 41, 8, 41, 41, 9, 10, 11, 41, 12],
        list(range(40)),
        [7],
        [0, 1],
        list(range(9)),                   # 9: one level with a lone last point
        [i % 40 for i in range(33000)],   # period 40: equal pairs from level 3 on
        [i % 7 for i in range(300)] + [40, 3],
    ]
    got = c.aggregate_pubkeys_multi([PkIndices(ix) for ix in cases] + [PkIndices([1, 99999]), PkIndices([])])
    for k, ix in enumerate(cases):
        assert got[k] == (expect(ix), 0), (k, len(ix))
    assert got[-2][1] == LSG_ERR_BAD_INDEX and got[-1][1] == 101
    # the same through byte-encoded keys (decoded in the tree's gather), below and above the
    # tree's threshold
    few = [bd.pk_bytes(i % 40) for i in range(50)]
    many = [bd.pk_bytes(i % 40, compressed=(i >= 16500)) for i in range(33000)]  # (one encoding per set)
    g2 = c.aggregate_pubkeys_multi([few, many[:33000 // 2], many[33000 // 2:]])
    assert g2[0] == (expect([i % 40 for i in range(50)]), 0)
    assert g2[1] == (expect([i % 40 for i in range(16500)]), 0)
    assert g2[2] == (expect([i % 40 for i in range(16500, 33000)]), 0)


def test_pubkey_table_rejects_bad_keys_and_grows(table_ctx):
    from lodestar_amd._native import PkIndices, LSG_ERR_BAD_INDEX
    c = table_ctx
    bad = bytearray(bd.pk_bytes(1))
    bad[50] ^= 1  # y no longer on the curve
    errs = c.pubkey_table_set(5000, [bd.pk_bytes(41), bytes(bad), bd.pk_bytes(43)])
    assert errs[0] == 0 and errs[1] == 2 and errs[2] == 0  # BLST_POINT_NOT_ON_CURVE
    assert c.pubkey_table_size() == 5003
    assert c.aggregate_pubkeys(PkIndices([5000, 5002]))[0] == g1_serialize(
        ov.aggregate_pubkeys([bd.pk_point(41), bd.pk_point(43)]))
    assert c.aggregate_pubkeys(PkIndices([5001]))[1] == LSG_ERR_BAD_INDEX  # undecodable key: index unset
    assert c.aggregate_pubkeys(PkIndices([4999]))[1] == LSG_ERR_BAD_INDEX  # gap: never set
    assert c.aggregate_pubkeys(PkIndices([0, 39]))[0] == g1_serialize(
        ov.aggregate_pubkeys([bd.pk_point(0), bd.pk_point(39)]))  # rows kept across growth


def test_index_sets_match_byte_sets(table_ctx):
    """Verdicts of sets naming keys by index equal those of the same sets with encoded keys,
    through maybeBatch (lsg_verify_sets) and the worker's batch + retry path (lsg_verify_jobs)."""
    from lodestar_amd._native import PkIndices, LSG_ERR_BAD_INDEX
    c = table_ctx

    def by_index(s, keys):
        return (PkIndices(keys), s[1], s[2])

    agg_keys = [list(range(3 * i, 3 * i + 4 + i)) for i in range(4)]
    agg = [by_index(bd.aggregate_set(i, k), k) for i, k in enumerate(agg_keys)]
    single = [by_index(bd.single_set(i), [i]) for i in range(4)]
    assert c.verify_sets(agg + single, seed=11) == (1, 0)
    wrong = by_index(bd.corrupt_wrong_message(bd.single_set(5)), [5])
    assert c.verify_sets(agg + [wrong], seed=11) == (0, 0)
    miss = (PkIndices(agg_keys[1][:-1]), agg[1][1], agg[1][2])  # one signer missing
    assert c.verify_sets([miss], seed=11) == (0, 0)
    jobs = [(agg[:2], 1), ([wrong], 1), (single, 1), (agg[2:], 0)]
    got, stats = c.verify_jobs(jobs, seed=12)
    assert [g[0] for g in got] == [1, 0, 1, 1]
    # deserializeSet semantics (worker.ts:108-114): an unknown index rejects the package
    got, _ = c.verify_jobs([(agg[:1], 1), ([(PkIndices([7, 4096]), agg[0][1], agg[0][2])], 1)], seed=13)
    assert got == [(2, LSG_ERR_BAD_INDEX), (2, LSG_ERR_BAD_INDEX)]


# ---- batched KeyValidate (PublicKey.fromBytes(pk, affine, true),
# processDeposit.ts:57-65) against oracle/verifier.py:public_key_validate
def test_pubkey_validate_matches_oracle(ctx):
    from oracle.curves import g1_compress
    from oracle.fields import P
    flip = bytearray(bd.pk_bytes(2, compressed=True))
    flip[47] ^= 4
    big_x = bytearray((P + 5).to_bytes(48, "big"))
    big_x[0] |= 0x80
    cases = {
        48: [bd.pk_bytes(i, compressed=True) for i in range(3)] + [g1_compress(None), bytes(flip), bytes(big_x),
                                                                   g1_compress(bd.g1_not_in_group(1))],
        96: [bd.pk_bytes(i) for i in range(3, 6)] + [g1_serialize(None), g1_serialize(bd.g1_not_in_group(2)),
                                                     bytes(96)],
    }
    for ln, pks in cases.items():
        got = ctx.pubkey_validate(pks)
        for pk, (out, err) in zip(pks, got):
            try:
                pt = ov.public_key_validate(pk)
                exp = 0
            except BlstError as e:
                exp = e.code
            assert err == exp, (ln, pk.hex(), err, exp)
            if exp == 0:
                assert out == g1_serialize(pt)


def test_aggregate_signatures_matches_golden(ctx):
    """Op-pool Signature.aggregate: every golden case of one encoding in one
    batched call, plus an empty group, against the oracle's fixture."""
    from lodestar_amd._native import LSG_ERR_EMPTY_AGGREGATE
    gold = json.load(open(os.path.join(GOLDEN, "aggregate_signatures.json")))
    by_len = {}
    for c in gold["cases"]:
        by_len.setdefault(len(c["sigs"][0]) // 2, []).append(c)
    for ln, cases in by_len.items():
        groups = [[bytes.fromhex(x) for x in c["sigs"]] for c in cases] + [[]]
        out = ctx.aggregate_signatures(groups)
        for c, (o, err) in zip(cases, out):
            assert err == c["err"], c
            if err == 0:
                assert o.hex() == c["out"]
        assert out[-1][1] == LSG_ERR_EMPTY_AGGREGATE
    (o, err), = ctx.aggregate_signatures([[bytes(32)]])
    assert err == 10  # BLST_INVALID_SIZE


def test_aggregate_signatures_linearity_at_scale(ctx):
    """4096 signatures (sync-committee / attestation-committee sizes mixed) in 40 groups over
    one message per group: each aggregate must equal the signature of the group's summed key
    (size-independent property; the signatures and the expected values come from lsg_sign)."""
    from oracle.fields import R
    import random
    rng = random.Random(5)
    sizes = [512] * 4 + [128] * 10 + [64] * 8 + [1, 2, 3, 7] * 4
    sizes.append(4096 - sum(sizes))
    assert sizes[-1] > 0
    sks = [rng.randrange(1, R) for _ in range(4096)]
    msgs, sums, pos = [], [], 0
    for g, n in enumerate(sizes):
        m = bd.msg("oppool-scale", g)
        msgs += [m] * n
        sums.append(sum(sks[pos:pos + n]) % R)
        pos += n
    sigs = ctx.sign(sks, msgs)
    groups, pos = [], 0
    for n in sizes:
        groups.append(sigs[pos:pos + n])
        pos += n
    out = ctx.aggregate_signatures(groups)
    expect = ctx.sign(sums, [bd.msg("oppool-scale", g) for g in range(len(sizes))])
    for g, ((o, err), e) in enumerate(zip(out, expect)):
        assert err == 0 and o == e, g


def test_signing_roots_pinned_by_genesis_kat(ctx):
    """computeSigningRoot on the GPU reproduces the deposit signing root the
    reference's genesis KAT signs (test/e2e/interop/genesisState.test.ts:49-56), and the
    AttestationData form matches the oracle for per-object and shared domains."""
    import random
    from oracle import interop as oi
    pk = bytes.fromhex(GENESIS_KAT["pubkey"])
    wc, root = genesis_deposit_signing_root(pk)
    domain = oi.compute_domain(oi.DOMAIN_DEPOSIT, oi.GENESIS_FORK_VERSION_MINIMAL, bytes(32))
    obj = oi.deposit_message_root(pk, wc, oi.MAX_EFFECTIVE_BALANCE)
    assert ctx.signing_roots([obj], domain) == [root]
    rng = random.Random(11)
    datas = [bytes(rng.getrandbits(8) for _ in range(128)) for _ in range(300)]
    doms = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(300)]
    assert ctx.attestation_signing_roots(datas, doms) == [oi.attestation_signing_root(d, m) for d, m in zip(datas, doms)]
    assert ctx.attestation_signing_roots(datas[:5], doms[0]) == [oi.attestation_signing_root(d, doms[0])
                                                                  for d in datas[:5]]
    objs = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(65)]
    assert ctx.signing_roots(objs, doms[:65]) == [oi.compute_signing_root(o, m) for o, m in zip(objs, doms)]


def test_attestation_signing_roots_feed_verification(ctx):
    """The GPU's attestation signing roots are the messages the verifier checks: sets signed
    over them verify, and a set whose AttestationData changes by one bit does not."""
    import random
    from oracle.fields import R
    rng = random.Random(12)
    n = 64
    datas = [bytes(rng.getrandbits(8) for _ in range(128)) for _ in range(n)]
    domain = bytes(rng.getrandbits(8) for _ in range(32))
    roots = ctx.attestation_signing_roots(datas, domain)
    sks = [bd.sk(i) for i in range(n)]
    sigs = ctx.sign(sks, roots)
    sets = [([bd.pk_bytes(i)], roots[i], sigs[i]) for i in range(n)]
    assert ctx.verify_sets(sets, seed=3)[0] == 1
    bad = bytearray(datas[7])
    bad[0] ^= 1
    sets[7] = (sets[7][0], ctx.attestation_signing_roots([bytes(bad)], domain)[0], sets[7][2])
    assert ctx.verify_sets(sets, seed=3)[0] == 0


def test_device_fp2_leaf_at_lazy_bounds(ctx):
    """The device Fp2 product leaf (lsg_fp_pair.hpp pair_fp2_mul_v, the SOP form) at the lazy
    bounds of its inputs: limbs at the edges of [-8, 2^29 + 8), signed top limbs with
    |v| < 2^12.6 p -- on gfx950 an accumulator column lives 7 steps per lane and the argued bound
    is |t| < 2^62.6, which random field elements never approach -- against exact integers:
    out = (a0 b0 - a1 b1, a0 b1 + a1 b0) / 2^406 mod p, |out| < 3p, limbs 0..12 normalised
    (lsg_check_fp2_mul runs the leaf the kernels call)."""
    import itertools
    import random
    P = h2c.P
    Rinv = pow(1 << 406, -1, P)
    bound = int(2 ** 12.6 * P)
    top_max = bound >> (29 * 13)

    def value(limbs):
        return sum(v << (29 * k) for k, v in enumerate(limbs))

    def clamp(limbs):  # the top limb's magnitude lowered until |value| < 2^12.6 p
        while abs(value(limbs)) >= bound:
            limbs[13] += -1 if limbs[13] > 0 else 1
        return limbs

    patterns = [clamp([lo] * 13 + [top]) for lo, top in
                itertools.product(((1 << 29) + 7, -8, 0, (1 << 29) - 1), (top_max, -top_max, 0, 1))]
    r = random.Random(77)
    patterns += [clamp([r.randrange(-8, (1 << 29) + 8) for _ in range(13)] + [r.randrange(-top_max, top_max + 1)])
                 for _ in range(60)]
    # alternating extremes: the largest positive and negative partial products in one column
    patterns += [clamp([((1 << 29) + 7) if k % 2 else -8 for k in range(13)] + [top_max]),
                 clamp([-8 if k % 2 else ((1 << 29) + 7) for k in range(13)] + [-top_max])]

    def pair_words(limbs):  # pair layout of one element: limb L at word 2 (L mod 7) + L / 7
        w = [0] * 14
        for L, v in enumerate(limbs):
            w[2 * (L % 7) + L // 7] = v & 0xFFFFFFFF
        return w

    def from_words(w):
        limbs = [w[2 * (L % 7) + L // 7] for L in range(14)]
        return [x - (1 << 32) if x >= (1 << 31) else x for x in limbs]

    items = []
    n = len(patterns)
    for k in range(4 * n):
        items.append((patterns[k % n], patterns[(3 * k + 1) % n], patterns[(5 * k + 2) % n], patterns[(7 * k + 3) % n]))
    words = [w for it in items for e in it for w in pair_words(e)]
    out = ctx.check_fp2_mul(words)
    for i, (a0, a1, b0, b1) in enumerate(items):
        va0, va1, vb0, vb1 = map(value, (a0, a1, b0, b1))
        c0, c1 = from_words(out[28 * i:28 * i + 14]), from_words(out[28 * i + 14:28 * i + 28])
        v0, v1 = value(c0), value(c1)
        assert (v0 - (va0 * vb0 - va1 * vb1) * Rinv) % P == 0, i
        assert (v1 - (va0 * vb1 + va1 * vb0) * Rinv) % P == 0, i
        assert abs(v0) < 3 * P and abs(v1) < 3 * P, i
        assert all(0 <= c < (1 << 29) for c in c0[:13] + c1[:13]), i
