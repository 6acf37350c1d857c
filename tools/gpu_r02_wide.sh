#!/bin/bash
# serial stages: one-item-per-row build from LSG_ROW_WIDE_MIN (512) groups on (default) vs the
# row-split build for every group count (liblodestar_bls_r4only.so): parity suite, then the
# adversarial (per-job fallback groups) and jobs workloads, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], 'fe', k.get('k_row_final_exp'), 'negg1', k.get('k_row_miller_neg_g1'))" "$1" "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in wide r4only; do
    lib=lodestar_amd/liblodestar_bls.so; [ $v = r4only ] && lib=lodestar_amd/liblodestar_bls_r4only.so
    LSG_LIB=$lib timeout -k 10 300 python -u bench.py --workload adversarial --no-cpu-baseline > gpurun_out/wd_adv_${v}_$rep.log 2>&1 && summ gpurun_out/wd_adv_${v}_$rep.log adv_${v}_$rep || exit 1
  done
done
for v in wide r4only; do
  lib=lodestar_amd/liblodestar_bls.so; [ $v = r4only ] && lib=lodestar_amd/liblodestar_bls_r4only.so
  LSG_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/wd_jobs_$v.log 2>&1 && summ gpurun_out/wd_jobs_$v.log jobs_$v || exit 1
done
