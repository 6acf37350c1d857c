"""PublicKey.aggregate of one block package alone on the GPU (config C's pubkey side): 64
blocks x 128 aggregate sets of 440-460 random signers named by index into a pubkey table
(validator v holds key v mod 1024), through lsg_aggregate_pubkeys_multi -- the same tree the
verification packages run (lsg_host.hip launch_agg_tree), with nothing else on the device.
Prints one JSON line: per-call wall time and the library's per-kernel times (HIP events).

  python tools/agg_probe.py [--sets 8192] [--validators 1048576] [--reps 5]
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=8192)
    ap.add_argument("--validators", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", type=int, default=16, help="sets compared against the serial fold (A/B library)")
    args = ap.parse_args()
    from lodestar_amd import _native
    from bench import interop_sk

    ctx = _native.Context(0)
    pks = ctx.sk_to_pk([interop_sk(i) for i in range(1024)])
    for first in range(0, args.validators, 65536):
        n = min(65536, args.validators - first)
        ctx.pubkey_table_set(first, [pks[v % 1024] for v in range(first, first + n)])
    rng = random.Random(7)
    sets = [_native.PkIndices(rng.sample(range(args.validators), rng.randint(440, 460))) for _ in range(args.sets)]
    ctx.aggregate_pubkeys_multi(sets)  # warm: buffers sized
    wall, kern = [], {}
    for _ in range(args.reps):
        t0 = time.perf_counter()
        out = ctx.aggregate_pubkeys_multi(sets)
        wall.append((time.perf_counter() - t0) * 1e3)
        for name, ms in ctx.last_kernel_times():
            kern[name] = kern.get(name, 0.0) + ms / args.reps
    assert all(e == 0 for _, e in out)
    # spot check: small lists (below the tree's threshold) run the serial fold + butterfly
    bad = 0
    for i in range(min(args.check, args.sets)):
        ref = ctx.aggregate_pubkeys_multi([sets[i]])[0][0]
        bad += ref != out[i][0]
    print(json.dumps({"sets": args.sets, "keys": sum(len(s) for s in sets), "wall_ms": [round(w, 3) for w in wall],
                      "kernel_ms": {k: round(v, 4) for k, v in sorted(kern.items(), key=lambda x: -x[1])},
                      "checked": min(args.check, args.sets), "mismatches": bad}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
