#!/bin/bash
# GPU-box A/B of k_miller_fused's register budget: the default library (LSG_MF_WAVES=2: 256
# registers, so other kernels' waves can share a SIMD with the LDS-bound workgroup) against
# lodestar_amd/liblodestar_bls_mf1.so (-DLSG_MF_WAVES=1: 512 registers, no scratch spill),
# interleaved on MFAB_WORKLOADS (default: the firehose and block bodies).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
one() {  # tag workload lib
  local tag=$1 w=$2 lib=$3
  echo "== $tag $w ($(date +%T))"
  LSG_LIB=$lib timeout -k 10 300 python -u bench.py --workload "$w" --no-cpu-baseline \
    > "gpurun_out/r04_mfab_${w}_${tag}.json" 2> "gpurun_out/r04_mfab_${w}_${tag}.err"
  local rc=$?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'], d.get('p50_batch_latency_ms'), d['kernel_ms'].get('k_miller_fused'))" "gpurun_out/r04_mfab_${w}_${tag}.json"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/r04_mfab_${w}_${tag}.err"; echo "== FAILED rc=$rc"; exit $rc; fi
}
for w in ${MFAB_WORKLOADS:-jobs block}; do
  one dflt1 "$w" lodestar_amd/liblodestar_bls.so
  one mf1a "$w" lodestar_amd/liblodestar_bls_mf1.so
  one dflt2 "$w" lodestar_amd/liblodestar_bls.so
  one mf1b "$w" lodestar_amd/liblodestar_bls_mf1.so
done
echo "== all ok"
