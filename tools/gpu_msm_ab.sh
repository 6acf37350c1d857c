#!/bin/bash
# Block bodies (config C): the bucket MSM for the RLC signature sums against per-set [r_i] sig_i
# (A/B build: LSG_MSM_MIN_GROUP=1000000 disables the MSM), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${MSMAB:-"4:a" "1000000:a" "4:b" "1000000:b"}; do
  m=${c%%:*}; t=${c#*:}
  o="gpurun_out/r04_msmab_${WL:-block}_m${m}_${t}"
  echo "== msm_min_group $m ($t, $(date +%T))"
  LSG_LIB=lodestar_amd/liblodestar_bls_ab.so LSG_MSM_MIN_GROUP=$m timeout -k 10 300 python -u bench.py \
    --workload "${WL:-block}" --no-cpu-baseline > "$o.json" 2> "$o.err" || { tail -5 "$o.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; print(round(d['value']), d['ms_per_step'], d['p50_unloaded_latency_ms'], d['host_submit_ms_per_package'])" "$o.json"
done
echo "== all ok"
