#!/bin/bash
# GPU-box: smaller coalesced launches for gossip / sync: launches of <= 2048
# sets take the straight-line-program Miller items (k_slp_items1, ~0.6 ms of latency) instead of
# the fused kernel (a whole 64-step loop, ~4.9 ms, whatever the launch size).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/co2
for rep in 1 2; do
  for cfg in "--coalesce 4096 --coalesce-inflight 4" "--coalesce 2048 --coalesce-inflight 4" "--coalesce 2048 --coalesce-inflight 8" \
             "--coalesce 1024 --coalesce-inflight 8" "--coalesce 1024 --coalesce-inflight 12"; do
    for w in gossip sync; do
      out=gpurun_out/co2/${w}_$(echo $cfg | tr -d ' -')_$rep.json
      timeout -k 10 300 python3 -u bench.py --workload $w --no-cpu-baseline $cfg > $out 2> ${out%.json}.err || { tail -3 ${out%.json}.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$out').read().splitlines()[-1]); print('$w', '$cfg', d['value'], d['p50_batch_latency_ms'], d['host_cpu_cores_busy'])"
    done
  done
done
