#!/bin/bash
# GPU-box sweep for the small-package workloads (gossip-128, sync): the straight-line-program
# threshold (LSG_SLP_ITEMS, A/B build) x coalesced launches in flight.  -> gpurun_out/r05_small_*.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in ${SW_WORKLOADS:-gossip sync}; do
  for slp in ${SW_SLP:-2048 512 256}; do
    for f in ${SW_INFLIGHT:-4 8}; do
      out="gpurun_out/r05_small_${w}_slp${slp}_f${f}"
      echo "== $w slp=$slp inflight=$f ($(date +%T))"
      LSG_LIB=lodestar_amd/liblodestar_bls_ab.so LSG_SLP_ITEMS=$slp timeout -k 10 300 python -u bench.py --workload "$w" \
        --coalesce-inflight "$f" --no-cpu-baseline > "$out.json" 2> "$out.err" || { tail -5 "$out.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$out.json').read().splitlines()[-1]); print(d['value'], d['p50_batch_latency_ms'], d['whole_path_mad_frac'])"
    done
  done
done
echo "== all ok"
