#!/usr/bin/env python3
"""Count HIP allocation / free API calls inside bench.py's timed window, from a
`rocprofv3 --hip-trace --output-format csv` run of the same command (the bench line's
timed_window_monotonic_ns and rocprofv3's timestamps are both CLOCK_MONOTONIC).

    python tools/hip_alloc_window.py gpurun_out/alloc_trace gpurun_out/alloc_bench.log > profiles/r02_hip_alloc_window.json
"""
import collections
import csv
import glob
import json
import os
import sys

ALLOC = ("hipMalloc", "hipFree", "hipHostMalloc", "hipHostFree", "hipMallocAsync", "hipFreeAsync", "hipHostRegister",
         "hipExtMallocWithFlags", "hipMallocManaged", "hipHostAlloc", "hipMallocHost", "hipFreeHost")


def main():
    tdir, log = sys.argv[1], sys.argv[2]
    line = json.loads([x for x in open(log).read().splitlines() if x.startswith("{")][-1])
    w0, w1 = line["timed_window_monotonic_ns"]
    inside, outside, api_total = collections.Counter(), collections.Counter(), collections.Counter()
    files = glob.glob(os.path.join(tdir, "**", "*hip_api_trace.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                fn = row.get("Function") or row.get("Operation") or ""
                t = int(row["Start_Timestamp"])
                if w0 <= t <= w1:
                    api_total[fn] += 1
                if fn in ALLOC:
                    (inside if w0 <= t <= w1 else outside)[fn] += 1
    print(json.dumps({"trace_files": [os.path.relpath(f) for f in files], "timed_window_ns": [w0, w1],
                      "timed_steps": line["steps"], "alloc_calls_in_window": dict(inside),
                      "alloc_calls_outside_window": dict(outside),
                      "hip_api_calls_in_window": dict(api_total.most_common())}, indent=1))


if __name__ == "__main__":
    main()
