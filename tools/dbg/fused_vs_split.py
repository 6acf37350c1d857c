"""Debug: batch partials of the same sets under the Miller variants (split K=1/2/4, fused)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests import test_gpu_configs as T  # noqa: E402
from lodestar_amd._native import Context  # noqa: E402
from oracle.interop import interop_secret_key  # noqa: E402

ctx = Context(0)
sks = [interop_secret_key(i) for i in range(T.N_KEYS)]
keys = (sks, ctx.sk_to_pk(sks))
for n in [2, 5, 8, 9, 37]:
    sets = T.single_sets(ctx, keys, b"dbg", n)
    out = {}
    for name, env in [("k1", {"LSG_MILLER_FUSED": "0", "LSG_MILLER_K": "1"}),
                      ("k2", {"LSG_MILLER_FUSED": "0", "LSG_MILLER_K": "2"}),
                      ("k4", {"LSG_MILLER_FUSED": "0", "LSG_MILLER_K": "4"}),
                      ("fused", {"LSG_MILLER_FUSED": "1"})]:
        os.environ.update(env)
        out[name] = ctx.batch_partial(sets, seed=11)[0]
        os.environ.pop("LSG_MILLER_K", None)
    print(n, {k: (v == out["k1"]) for k, v in out.items()}, ctx.verify_sets(sets), flush=True)
