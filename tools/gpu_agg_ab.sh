#!/bin/bash
# Block bodies (config C): the batch-affine aggregation tree against the serial fold
# (A/B build, LSG_AGG_TREE) over AGG_AB="validators:tree[:hw_queues] ..." cases.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${AGG_AB:-"1048576:1" "1048576:0" "1024:1" "1024:0"}; do
  IFS=: read -r v t q <<< "$c"
  o="gpurun_out/r04_aggab_v${v}_t${t}_q${q:-def}"
  echo "== validators $v tree $t hw_queues ${q:-default} ($(date +%T))"
  ( [ -n "$q" ] && export GPU_MAX_HW_QUEUES=$q
    LSG_LIB=lodestar_amd/liblodestar_bls_ab.so LSG_AGG_TREE=$t timeout -k 10 300 python -u bench.py --workload block \
      --validators "$v" --no-cpu-baseline ${AGG_AB_ARGS:-} > "$o.json" 2> "$o.err" ) || { tail -5 "$o.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; print(round(d['value']), d['ms_per_step'], d['p50_unloaded_latency_ms'], d['host_submit_ms_per_package'], {x: k.get(x) for x in ('k_pk_gather_aff','k_pk_decode','g1_aggregate','binv_agg')})" "$o.json"
done
echo "== all ok"
