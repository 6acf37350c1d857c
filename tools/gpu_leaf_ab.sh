#!/bin/bash
# GPU-box A/B of the Montgomery leaf: the default library (DPP moves folded
# into the ands) against lodestar_amd/liblodestar_bls_dppand0.so (-DLSG_LEAF_DPP_AND=0, the
# round-2 moves), interleaved on the latency-bound workloads (gossip-128, single, sync).
#   bash tools/gpu_leaf_ab.sh            -> gpurun_out/r04_leafab_*.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=lodestar_amd/liblodestar_bls_dppand0.so
one() {  # tag workload lib
  local tag=$1 w=$2 lib=$3
  echo "== $tag $w ($(date +%T))"
  LSG_LIB=$lib timeout -k 10 300 python -u bench.py --workload "$w" --no-cpu-baseline \
    > "gpurun_out/r04_leafab_${w}_${tag}.json" 2> "gpurun_out/r04_leafab_${w}_${tag}.err"
  local rc=$?
  tail -c 400 "gpurun_out/r04_leafab_${w}_${tag}.json"; echo
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/r04_leafab_${w}_${tag}.err"; echo "== FAILED rc=$rc"; exit $rc; fi
}
for w in ${LEAFAB_WORKLOADS:-gossip single sync}; do
  one dflt1 "$w" lodestar_amd/liblodestar_bls.so
  one and01 "$w" "$AB"
  one dflt2 "$w" lodestar_amd/liblodestar_bls.so
  one and02 "$w" "$AB"
done
echo "== all ok"
