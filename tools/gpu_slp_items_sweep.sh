#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/slpsweep
for rep in 1 2; do
for v in 2048 4096 1024; do
  for w in gossip sync; do
    LSG_SLP_ITEMS=$v timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/slpsweep/${w}_${v}_${rep}.log 2>&1 || exit $?
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/slpsweep/${w}_${v}_${rep}.log').read().strip().splitlines()[-1]); print('$w slp_items=$v', d['value'], d['p50_batch_latency_ms'])"
  done
done
done
