#!/bin/bash
# Fp12 products folded 4 terms per lane pair per pass (SEG_FOLD_FP12): parity suite, then
# pipelined and depth-1 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], 'horner', k.get('k_row_horner_miller'), 'fe', k.get('k_row_final_exp'), 'prod', k.get('fp12_product'), 'allocs', d.get('allocations_in_timed_region'))" "$1" "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/sx_$rep.log 2>&1 || exit 1
  summ gpurun_out/sx_$rep.log pipe_$rep || exit 1
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --depth 1 --steps 8 > gpurun_out/sx_d1_$rep.log 2>&1 || exit 1
  summ gpurun_out/sx_d1_$rep.log d1_$rep || exit 1
done
