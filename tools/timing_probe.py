"""Dev tool: per-kernel timing of one sharded batch on the GPU (not part of the product).
usage: python tools/timing_probe.py [n_sets]"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lodestar_amd._native import Context  # noqa: E402

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def interop_sk(i):
    return int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    ctx = Context(0)
    print(ctx.device_name(), flush=True)
    t = time.time()
    fp, mad = ctx.probe_fp_mul_rate()
    print(f"probe: {fp:.3e} fp_mul/s  {mad:.3e} mad/s ({time.time()-t:.2f}s)", flush=True)
    nk = min(n, 1024)
    sks = [interop_sk(i) for i in range(nk)]
    t = time.time()
    pks = ctx.sk_to_pk(sks)
    print(f"keygen {nk}: {time.time()-t:.2f}s", flush=True)
    msgs = [hashlib.sha256(b"lodestar-mi355x" + b"firehose" + i.to_bytes(8, "little")).digest() for i in range(n)]
    t = time.time()
    sigs = ctx.sign([sks[i % nk] for i in range(n)], msgs)
    print(f"sign {n}: {time.time()-t:.2f}s", flush=True)
    for k in ctx.last_kernel_times():
        print("   ", k)
    sets = [([pks[i % nk]], msgs[i], sigs[i]) for i in range(n)]
    for rep in range(2):
        t = time.time()
        part, errs, anyerr = ctx.batch_partial(sets, seed=1 + rep)
        dt = time.time() - t
        kt = ctx.last_kernel_times()
        t = time.time()
        ok = ctx.final_verify([part])
        dfe = time.time() - t
        print(f"rep {rep}: batch_partial {dt*1e3:.1f} ms anyerr={anyerr} final_verify {dfe*1e3:.1f} ms ok={ok}", flush=True)
        for name, ms in kt:
            print(f"    {name:20s} {ms:9.3f} ms")
    res = {"n": n, "fp_mul_per_s": fp, "mad_per_s": mad}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "timing_probe.json"), "w"))


if __name__ == "__main__":
    main()
