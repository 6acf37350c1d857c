#!/bin/bash
# Firehose (config D, workload jobs) throughput against pipeline depth and package size.
#   JOBS_SWEEP="depth:sets ..." bash tools/gpu_jobs_sweep.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${LSG_TAG:-r04}
for cfg in ${JOBS_SWEEP:-"6:32768" "8:32768" "10:32768" "4:65536"}; do
  d=${cfg%%:*}; n=${cfg#*:}
  o="gpurun_out/${TAG}_${WL:-jobs}_d${d}_n${n}"
  echo "== ${WL:-jobs} depth $d sets $n ($(date +%T))"
  timeout -k 10 300 python -u bench.py --workload "${WL:-jobs}" --depth "$d" --sets-per-step "$n" --no-cpu-baseline \
    > "$o.json" 2> "$o.err" || { tail -5 "$o.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], d['whole_path_mad_frac'])" "$o.json"
done
echo "== all ok"
