# GPU-box sweep of the coalescing parameters for gossip and sync (bench.py --coalesce / --coalesce-inflight)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in "--coalesce 4096" "--coalesce 8192" "--coalesce 4096 --coalesce-inflight 6" "--coalesce 8192 --coalesce-inflight 3"; do
  for w in gossip sync; do
    out=gpurun_out/r05_co_${w}_$(echo $cfg | tr -d ' -')_$rep.json
    timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline $cfg > $out 2> /dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$out').read().splitlines()[-1]); print('$w', '$cfg', d['value'], d['p50_batch_latency_ms'])"
  done
done
done
