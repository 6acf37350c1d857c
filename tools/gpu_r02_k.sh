#!/bin/bash
# diagnose run-to-run pipelining variance: environment, CPU share, repeated runs, a kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
{ env | grep -E '^(HIP|AMD|GPU|HSA|ROC|OMP)' | sort; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/loadavg; uptime; } > gpurun_out/bk_env.txt 2>&1
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'])" "$1" "$2"; }
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --waits inline > gpurun_out/bk_$i.log 2>&1 && summ gpurun_out/bk_$i.log run$i || exit 1
  cat /proc/loadavg
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bk_trace -o run -- python3 -u bench.py --no-cpu-baseline --waits inline --steps 12 > gpurun_out/bk_trace.log 2>&1 && summ gpurun_out/bk_trace.log traced
