#!/bin/bash
# pipeline depth / package size sweep of the jobs workload (default 32,768 sets, depth 4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'])" "$1" "$2"; }
for cfg in "4 32768" "3 32768" "6 32768" "8 32768" "4 49152" "4 65536" "4 32768"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --depth $1 --sets-per-step $2 > gpurun_out/z_$1_$2.log 2>&1 && summ gpurun_out/z_$1_$2.log "depth$1_sets$2" || exit 1
done
