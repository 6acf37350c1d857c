"""Per-kernel HBM traffic per dispatch from the two rocprofv3 --pmc passes of tools/gpu_traffic.sh.

FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit one TCC group)
and reported by rocprofv3 in KiB per dispatch.  Corrections follow
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE counts half the
bytes of a wide coalesced read, so fetched bytes = 2 x FETCH_SIZE; WRITE_SIZE is taken as is.
Both derive from the L2's memory-side request counters, so Infinity-Cache hits are included:
the figure is an upper bound on HBM bytes.

    python tools/pmc_traffic.py gpurun_out/traffic_fetch gpurun_out/traffic_write \
        --sets-per-launch 24576 -o profiles/r01_pmc_traffic.json
"""
import argparse
import csv
import json
import os
import re


def per_kernel(d, counter):
    acc = {}
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = re.split(r"[(<]", row["Kernel_Name"])[0].split()[-1]
            a = acc.setdefault(name, [0.0, 0])
            a[0] += float(row["Counter_Value"])
            a[1] += 1
    return {k: (v[0] / v[1], v[1]) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--sets-per-launch", type=int, required=True,
                    help="sets one per-set kernel launch covers in the profiled run (groups x sets per group)")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    fe = per_kernel(a.fetch_dir, "FETCH_SIZE")
    wr = per_kernel(a.write_dir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fe) & set(wr)):
        fb = 2 * fe[k][0] * 1024
        wb = wr[k][0] * 1024
        kernels[k] = {"dispatches": fe[k][1], "fetch_size_kib": round(fe[k][0], 1),
                      "write_size_kib": round(wr[k][0], 1), "hbm_bytes_per_dispatch": round(fb + wb),
                      "hbm_bytes_per_set": round((fb + wb) / a.sets_per_launch, 1)}
    out = {"source": "tools/gpu_traffic.sh (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes)",
           "correction": "bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; gfx950 FETCH_SIZE halving)",
           "sets_per_launch": a.sets_per_launch, "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for k, v in kernels.items():
        print(f"{k:28s} {v['dispatches']:5d} {v['hbm_bytes_per_dispatch']:>14,d} B/dispatch "
              f"{v['hbm_bytes_per_set']:>10.1f} B/set")


if __name__ == "__main__":
    main()
