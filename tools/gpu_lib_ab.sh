#!/bin/bash
# GPU-box A/B of two library builds, interleaved:  AB_LIB=<path> AB_TAG=<name> bash tools/gpu_lib_ab.sh
#   (AB_ENV="VAR=value ...": environment of the alternative's runs, e.g. an A/B-build switch)
#   -> gpurun_out/<round>_ab_<tag>_<workload>_{dflt,alt}<rep>.json (AB_WORKLOADS, AB_REPS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${AB_ROUND:-r05}
one() {  # tag workload lib
  local out="gpurun_out/${R}_ab_${AB_TAG}_${2}_$1"
  echo "== $1 $2 ($(date +%T))"
  env LSG_LIB=$3 $4 timeout -k 10 300 python -u bench.py --workload "$2" --no-cpu-baseline ${AB_ARGS:-} > "$out.json" 2> "$out.err"
  local rc=$?
  python3 -c "import json; d=json.loads(open('$out.json').read().splitlines()[-1]); r=d['roofline']; print(d['value'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], r['kernel'], r['kernel_ms'], d['whole_path_mad_frac'])" || true
  if [ $rc -ne 0 ]; then tail -5 "$out.err"; echo "== FAILED rc=$rc"; exit $rc; fi
}
for w in ${AB_WORKLOADS:-jobs block gossip single}; do
  for k in $(seq 1 ${AB_REPS:-2}); do
    one "dflt$k" "$w" lodestar_amd/liblodestar_bls.so
    one "alt$k" "$w" "$AB_LIB" ${AB_ENV:-}
  done
done
echo "== all ok"
