#!/bin/bash
# leaf-mode A/B: LSG_LEAF_MODE 1 (multi-product leaves, products one after another; default)
# vs 0 (one product per call) vs 2 (interleaved multi-product leaves): throughput
# interleaved twice, then per-kernel memory-side traffic at depth 1 (FETCH_SIZE, WRITE_SIZE)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], r['kernel'], r['frac'], r['kernel_ms'])" "$1" "$2"; }
lib() { [ $1 = m1 ] && echo lodestar_amd/liblodestar_bls.so || echo lodestar_amd/liblodestar_bls_$1.so; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_cfg_m1.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_cfg_m1.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in m1 m0; do
    LSG_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/lm_${v}_$rep.log 2>&1 || exit 1
    summ gpurun_out/lm_${v}_$rep.log ${v}_$rep || exit 1
  done
done
B="bench.py --steps 4 --warmup 2 --depth 1 --no-cpu-baseline"
for v in m1 m0; do
  LSG_LIB=$(lib $v) timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/lt_f_$v -o run -- python3 $B > gpurun_out/lt_f_$v.log 2>&1 || exit 1
  LSG_LIB=$(lib $v) timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/lt_w_$v -o run -- python3 $B > gpurun_out/lt_w_$v.log 2>&1 || exit 1
  echo TRAFFIC_$v
done
