#!/bin/bash
# jobs bench vs the number of HW queues HIP maps the library's streams onto
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'])" "$1" "$2"; }
echo "env GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
for q in 4 4 8 8 16 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 60 > gpurun_out/bj_$q.log 2>&1 && summ gpurun_out/bj_$q.log q$q || exit 1
done
