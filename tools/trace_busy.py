#!/usr/bin/env python3
"""GPU busy fraction and kernel concurrency inside a bench run's timed window, from a
rocprofv3 kernel trace (rocpd database) and the bench line's timed_window_monotonic_ns.
    python tools/trace_busy.py gpurun_out/ntrace_plain/run_results.db gpurun_out/ntrace_plain.json"""
import json
import sqlite3
import sys


def main(db, bench):
    w0, w1 = json.loads(open(bench).read().splitlines()[-1])["timed_window_monotonic_ns"]
    c = sqlite3.connect(db)
    iv = [(max(s, w0), min(e, w1), n) for s, e, n in c.execute("select start, end, name from kernels")
          if e > w0 and s < w1]
    ev = sorted([(s, 1) for s, e, _ in iv] + [(e, -1) for s, e, _ in iv])
    busy = 0
    area = 0
    cur = 0
    last = w0
    for t, d in ev:
        if cur > 0:
            busy += t - last
        area += cur * (t - last)
        cur += d
        last = t
    span = w1 - w0
    by = {}
    for s, e, n in iv:
        k = n.split("(")[0].replace("void ", "")
        by[k] = by.get(k, 0) + (e - s)
    print(f"window {span / 1e6:.1f} ms, kernels {len(iv)}, busy {busy / span:.3f}, mean concurrency {area / max(busy, 1):.2f}")
    for k, v in sorted(by.items(), key=lambda x: -x[1])[:12]:
        print(f"  {k:40s} {v / 1e6:9.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
