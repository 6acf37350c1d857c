#!/bin/bash
# Coalesced small packages (gossip-128, sync contributions): one package group per
# sub-package against one group per 16-job chunk (A/B build, LSG_SUB_GROUPS), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in ${SUBAB_WORKLOADS:-gossip sync}; do
  for c in 1a 0a 1b 0b; do
    o="gpurun_out/r04_subab_${w}_${c}"
    LSG_LIB=lodestar_amd/liblodestar_bls_ab.so LSG_SUB_GROUPS=${c:0:1} timeout -k 10 300 python -u bench.py \
      --workload "$w" --no-cpu-baseline > "$o.json" 2> "$o.err" || { tail -5 "$o.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['p50_batch_latency_ms'], d['final_exps'])" "$o.json" "$w $c"
  done
done
echo "== all ok"
