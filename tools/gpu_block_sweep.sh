#!/bin/bash
# Block-body (config C) throughput against pipeline depth and package size (blocks per package).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${LSG_TAG:-r04}
for cfg in ${BLOCK_SWEEP:-"4:64" "6:64" "8:64" "4:128" "6:128"}; do
  d=${cfg%%:*}; b=${cfg#*:}
  echo "== depth $d blocks $b ($(date +%T))"
  timeout -k 10 300 python -u bench.py --workload block --depth "$d" --blocks "$b" --no-cpu-baseline \
    > "gpurun_out/${TAG}_block_d${d}_b${b}.json" 2> "gpurun_out/${TAG}_block_d${d}_b${b}.err" || { tail -5 "gpurun_out/${TAG}_block_d${d}_b${b}.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], d['whole_path_mad_frac'], d['kernel_ms'].get('g1_aggregate'))" "gpurun_out/${TAG}_block_d${d}_b${b}.json"
done
echo "== all ok"
