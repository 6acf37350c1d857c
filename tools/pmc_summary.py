#!/usr/bin/env python3
"""Per-kernel isolation profile from tools/gpu_pmc.sh (depth-1 bench: one package at a time).

Inputs (gpurun_out/): iso_trace/run_results.db (kernel durations), iso_sq*/ and iso_fetch/,
iso_write/ (rocprofv3 --pmc CSVs).  For every kernel, per dispatch:
  - isolated duration (kernel trace), VALU instructions and their 64-bit share,
  - VALU issue share of the waves' lifetime: SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (both in
    quad-cycles, MI355X_MICROARCH.md PMC table),
  - HBM traffic: 2 x FETCH_SIZE + WRITE_SIZE (KiB per dispatch in rocprofv3's CSV; the gfx950
    FETCH_SIZE halving of the guide's HBM section; Infinity-Cache hits included, so an upper
    bound),
  - algorithmic work (bench/opcount.json stage counts x sets per launch) -> achieved mad/s and
    the fraction of the measured v_mad_u64_u32 peak.
Writes profiles/<tag>_pmc_isolation.json, profiles/<tag>_pmc_traffic.json (read by bench.py
for roofline.traffic) and a text table on stdout.

    python tools/pmc_summary.py gpurun_out --sets 32768 --tag r06   (--peak: override the run's probe)
"""
import argparse
import csv
import glob
import json
import os
import re
import sqlite3

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kname(s):
    s = s.replace("(anonymous namespace)::", "")
    return re.split(r"[(]", s)[0].replace("void ", "").strip()


def durations(db):
    c = sqlite3.connect(db)
    out = {}
    for name, n, avg in c.execute("select name, count(*), avg(end - start) from kernels group by name"):
        out[kname(name)] = {"calls": n, "avg_ns": avg}
    return out


def counters(d):
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = kname(row["Kernel_Name"])
                a = acc.setdefault(k, {}).setdefault(row["Counter_Name"], [0.0, 0])
                a[0] += float(row["Counter_Value"])
                a[1] += 1
    return {k: {c: v[0] / v[1] for c, v in cs.items()} for k, cs in acc.items()}


def serial_durations(d):
    """per-kernel average dispatch duration in a --pmc pass: counter collection serialises the
    dispatches, so these are each kernel alone on the GPU (the kernel trace of the depth-1 run
    still overlaps the package's two streams)"""
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Dispatch_Id"] in seen:
                    continue
                seen.add(row["Dispatch_Id"])
                a = acc.setdefault(kname(row["Kernel_Name"]), [0.0, 0])
                a[0] += int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                a[1] += 1
    return {k: v[0] / v[1] for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--sets", type=int, required=True, help="sets per package in the profiled run")
    ap.add_argument("--peak", type=float, default=None,
                    help="v_mad_u64_u32 peak, mad/s (default: the profiled run's own probe, roofline.peak of the "
                         "bench line in <dir>/iso_trace.log)")
    ap.add_argument("--tag", default="r02")
    a = ap.parse_args()
    peak_source = "--peak"
    if a.peak is None:  # the same run's probe (lsg_probe_mad_peak, measured live by bench.py)
        lines = [l for l in open(os.path.join(a.dir, "iso_trace.log")) if l.startswith("{")]
        a.peak = json.loads(lines[-1])["roofline"]["peak"] * 1e12
        peak_source = "probe of the profiled run (iso_trace.log roofline.peak)"
    dur = durations(os.path.join(a.dir, "iso_trace", "run_results.db"))
    ser = serial_durations(os.path.join(a.dir, "iso_sq"))
    cnt = {}
    for sub in ("iso_sq", "iso_sq2", "iso_fetch", "iso_write"):
        for k, cs in counters(os.path.join(a.dir, sub)).items():
            cnt.setdefault(k, {}).update(cs)
    opc = json.load(open(os.path.join(ROOT, "bench", "opcount.json")))
    mk = os.environ.get("LSG_MILLER_K", "4")
    stage = {"k_miller_accum<4>": [f"miller_accum{mk}_per_set"], "k_miller_lines": ["miller_lines"],
             "k_miller_fused": ["miller_fused_per_set"],
             "k_sig_subgroup": ["sig_subgroup"], "k_sig_decode": ["sig_decode"], "k_pk_scale": ["pk_scale"]}
    rows, traffic = {}, {}
    for k in sorted(set(dur) | set(cnt), key=lambda x: -dur.get(x, {}).get("avg_ns", 0)):
        d, c = dur.get(k, {}), cnt.get(k, {})
        r = {"calls": d.get("calls"), "avg_us": round(d.get("avg_ns", 0) / 1e3, 2)}
        if "SQ_INSTS_VALU" in c:
            r["valu_instr"] = c["SQ_INSTS_VALU"]
            r["int64_share"] = round(c.get("SQ_INSTS_VALU_INT64", 0) / max(c["SQ_INSTS_VALU"], 1), 3)
            r["valu_issue_share"] = round(c.get("SQ_ACTIVE_INST_VALU", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1), 3)
            # wave cycles (SQ_WAVE_CYCLES is in quad-cycles) per VALU instruction: ~4-6 means
            # the wave issues back to back (instruction-bound), much more means it waits
            r["wave_cycles_per_valu"] = round(4 * c.get("SQ_WAVE_CYCLES", 0) / max(c["SQ_INSTS_VALU"], 1), 2)
        if k in ser:
            r["serial_us"] = round(ser[k] / 1e3, 2)
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            b = 1024.0 * (2 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0))
            r["hbm_bytes"] = round(b)
            r["hbm_bytes_per_set"] = round(b / a.sets, 1)
            traffic[k.split("<")[0]] = {"hbm_bytes_per_dispatch": round(b)}
        if k in stage and all(x in opc["stage_fp_muls"] for x in stage[k]) and d.get("avg_ns"):
            mads = sum(opc["stage_fp_muls"][x] for x in stage[k]) * a.sets * opc["mads_per_fp_mul"]
            r["achieved_tmad_s"] = round(mads / (d["avg_ns"] * 1e-9) / 1e12, 3)
            r["frac_of_peak"] = round(mads / (d["avg_ns"] * 1e-9) / a.peak, 4)
            if k in ser:
                r["frac_of_peak_serial"] = round(mads / (ser[k] * 1e-9) / a.peak, 4)
        rows[k] = r
    out = {"sets_per_launch": a.sets, "peak_mad_per_s": a.peak, "peak_source": peak_source, "kernels": rows,
           "source": "tools/gpu_pmc.sh (depth-1 bench, one package at a time) -> tools/pmc_summary.py",
           "columns": "avg_us: kernel trace of the depth-1 run (the package's two streams overlap); serial_us: the "
                      "same dispatches under --pmc, which serialises them (each kernel alone on the GPU); "
                      "frac_of_peak / frac_of_peak_serial: algorithmic mads over those durations / peak"}
    with open(os.path.join(ROOT, "profiles", f"{a.tag}_pmc_isolation.json"), "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.join(ROOT, "profiles", f"{a.tag}_pmc_traffic.json"), "w") as f:
        json.dump({"sets_per_launch": a.sets, "kernels": traffic,
                   "correction": "2 x FETCH_SIZE + WRITE_SIZE (gfx950, MI355X_MICROARCH.md HBM section)"}, f, indent=1)
    print(f"{'kernel':28s} {'calls':>5s} {'avg_us':>9s} {'alone_us':>9s} {'VALU/disp':>10s} {'i64':>5s} {'cyc/VALU':>8s} {'B/set':>8s} {'frac':>6s} {'alone':>6s}")
    for k, r in rows.items():
        print(f"{k[:28]:28s} {r.get('calls') or 0:5d} {r['avg_us']:9.1f} {r.get('serial_us', 0):9.1f} {r.get('valu_instr', 0):10.3g} "
              f"{r.get('int64_share', 0):5.2f} {r.get('wave_cycles_per_valu', 0):8.2f} {r.get('hbm_bytes_per_set', 0):8.1f} "
              f"{r.get('frac_of_peak', 0):6.3f} {r.get('frac_of_peak_serial', 0):6.3f}")


if __name__ == "__main__":
    main()
