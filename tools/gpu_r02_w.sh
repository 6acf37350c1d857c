#!/bin/bash
# serial per-group stages with one item per wave (four rows share the item's product batches)
# vs one item per row (-DLSG_ROWS_PER_ITEM=1): GPU parity suite, then pipelined and depth-1
# benches of both, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], 'horner', k.get('k_row_horner_miller'), 'fe', k.get('k_row_final_exp'), 'prod', k.get('fp12_product'))" "$1" "$2"; }
lib() { [ $1 = r4 ] && echo lodestar_amd/liblodestar_bls.so || echo lodestar_amd/liblodestar_bls_$1.so; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in r4 r1; do
    LSG_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/rw_${v}_$rep.log 2>&1 || exit 1
    summ gpurun_out/rw_${v}_$rep.log ${v}_$rep || exit 1
    LSG_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu-baseline --depth 1 --steps 8 > gpurun_out/rw_${v}_d1_$rep.log 2>&1 || exit 1
    summ gpurun_out/rw_${v}_d1_$rep.log ${v}_d1_$rep || exit 1
  done
done
