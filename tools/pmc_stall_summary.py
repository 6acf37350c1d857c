#!/usr/bin/env python3
"""Per-kernel stall profile from tools/gpu_pmc_stall.sh's two PMC passes (rocprofv3 csv):
the average over dispatches of each counter, and derived shares -- waiting cycles (SQ_WAIT_ANY)
and issue-wait cycles per wave cycle, LDS-wait share, LDS bank conflicts per LDS instruction.
Usage: python tools/pmc_stall_summary.py gpurun_out [kernel-substring ...]"""
import collections
import csv
import json
import os
import sys


def load(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0]
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main(d, picks):
    out = {}
    for part in ("stall_a", "stall_b"):
        for k, cs in load(os.path.join(d, part, "run_counter_collection.csv")).items():
            o = out.setdefault(k, {})
            for c, v in cs.items():
                o[c] = sum(v) / len(v)
    res = {}
    for k, o in out.items():
        if picks and not any(p in k for p in picks):
            continue
        wc = o.get("SQ_WAVE_CYCLES", 0) or 1
        res[k] = {
            "wave_cycles": o.get("SQ_WAVE_CYCLES"),
            "wait_any_share": round(o.get("SQ_WAIT_ANY", 0) / wc, 3),
            "wait_inst_any_share": round(o.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
            "wait_inst_lds_share": round(o.get("SQ_WAIT_INST_LDS", 0) / wc, 3),
            "valu_active_share": round(o.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3),
            "lds_active_share": round(o.get("SQ_ACTIVE_INST_LDS", 0) / wc, 3),
            "lds_bank_conflict_per_lds_inst": round(o.get("SQ_LDS_BANK_CONFLICT", 0) / max(o.get("SQ_INSTS_LDS", 0), 1), 3),
            "ifetch_per_kvalu": round(1e3 * o.get("SQ_IFETCH", 0) / max(o.get("SQ_INSTS_VALU", 0), 1), 3),
            "raw": {c: v for c, v in sorted(o.items())},
        }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
