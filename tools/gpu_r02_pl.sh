#!/bin/bash
# fused Miller kernel with paired line products (l0 l1, l2 l3 before multiplying into f):
# partial products against the split kernels, GPU parity suite, then A/B against the
# previous build (liblodestar_bls_old.so) pipelined and at depth 1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], 'fused', k.get('k_miller_fused'), r['frac'])" "$1" "$2"; }
timeout -k 10 200 python -u tools/dbg/fused_vs_split.py > gpurun_out/pl_fvs.log 2>&1; rc=$?; cat gpurun_out/pl_fvs.log | tail -6; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in new old; do
    lib=lodestar_amd/liblodestar_bls.so; [ $v = old ] && lib=lodestar_amd/liblodestar_bls_old.so
    LSG_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/pl_${v}_$rep.log 2>&1 && summ gpurun_out/pl_${v}_$rep.log ${v}_$rep || exit 1
  done
done
for v in new old; do
  lib=lodestar_amd/liblodestar_bls.so; [ $v = old ] && lib=lodestar_amd/liblodestar_bls_old.so
  LSG_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pl_pmc_$v -o run -- python3 bench.py --steps 4 --warmup 2 --depth 1 --no-cpu-baseline > gpurun_out/pl_pmc_$v.log 2>&1 || exit 1
  echo PMC_$v
done
for v in new old; do
  lib=lodestar_amd/liblodestar_bls.so; [ $v = old ] && lib=lodestar_amd/liblodestar_bls_old.so
  LSG_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/plt_f_$v -o run -- python3 bench.py --steps 4 --warmup 2 --depth 1 --no-cpu-baseline > gpurun_out/plt_f_$v.log 2>&1 || exit 1
  LSG_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/plt_w_$v -o run -- python3 bench.py --steps 4 --warmup 2 --depth 1 --no-cpu-baseline > gpurun_out/plt_w_$v.log 2>&1 || exit 1
  echo TRAFFIC_$v
done
