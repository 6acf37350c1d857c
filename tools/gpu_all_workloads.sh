#!/bin/bash
# GPU-box: one bench record per workload with the current build -> gpurun_out/<tag>_bench_<workload>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${ALL_TAG:-r05}
for w in ${ALL_WORKLOADS:-jobs committees block adversarial gossip sync single node}; do
  out="gpurun_out/${T}_bench_$w"
  echo "== $w ($(date +%T))"
  timeout -k 10 400 python -u bench.py --workload "$w" ${ALL_ARGS:-} > "$out.json" 2> "$out.err" || { tail -5 "$out.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$out.json').read().splitlines()[-1]); print(d['value'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], d['whole_path_mad_frac'])"
done
echo "== all ok"
