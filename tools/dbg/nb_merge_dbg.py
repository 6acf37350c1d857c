"""Dev diagnostic (not product): chunk mode after a merged-group package on one context."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lodestar_amd._native import Context, AB_LIB_PATH  # noqa: E402
AB_LIB_PATH = os.environ.get("DBG_LIB", AB_LIB_PATH)
from oracle.interop import interop_secret_key  # noqa: E402
import hashlib  # noqa: E402

def sets_for(ctx, n):
    sks = [interop_secret_key(i) for i in range(64)]
    pks = ctx.sk_to_pk(sks)
    msgs = [hashlib.sha256(b"dbg" + i.to_bytes(8, "little")).digest() for i in range(n)]
    sigs = ctx.sign([sks[i % 64] for i in range(n)], msgs)
    return [([pks[i % 64]], msgs[i], sigs[i]) for i in range(n)]

def run(label, seq, reserve=False):
    ctx = Context(0, lib=AB_LIB_PATH)
    if reserve:
        ctx.reserve(1024, 1024, 32 * 1024, n_slots=2)
    sets = sets_for(ctx, 600)
    jobs = [([s], 1) for s in sets[:300]] + [(sets[300 + 2 * k:302 + 2 * k], 1 if k % 4 else 0) for k in range(150)]
    out = []
    for env in seq:
        for k, v in env.items():
            os.environ[k] = v
        got, st = ctx.verify_jobs(jobs, seed=17)
        out.append((sum(1 for g in got if g[0] != 1), st["batch_retries"], st["batch_sigs_success"], st["n_final_exps"]))
    print(label, out, flush=True)
    ctx.close()

P0 = {"LSG_PACKAGE_GROUP": "0"}
P1 = {"LSG_PACKAGE_GROUP": "1", "LSG_NB_MERGE": "1"}
P1n = {"LSG_PACKAGE_GROUP": "1", "LSG_NB_MERGE": "0"}
run("chunk alone x2", [P0, P0])
run("merge then chunk", [P1, P0])
run("merge then chunk (reserved)", [P1, P0], reserve=True)
run("nomerge then chunk", [P1n, P0])
run("merge x2", [P1, P1])
run("chunk then merge", [P0, P1])
run("merge, chunk, merge, chunk", [P1, P0, P1, P0])
