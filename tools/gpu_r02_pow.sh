#!/bin/bash
# one-call fixed exponentiation with its table written out (default) vs the previous build
# (-DLSG_NO_POW_LEAF): parity suite, then jobs benches interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_unloaded_latency_ms'], 'dec', k.get('k_sig_decode'), 'map', k.get('k_h2c_map'))" "$1" "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in pow nopow; do
    lib=lodestar_amd/liblodestar_bls.so; [ $v = nopow ] && lib=lodestar_amd/liblodestar_bls_nopow.so
    LSG_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/pw_${v}_$rep.log 2>&1 && summ gpurun_out/pw_${v}_$rep.log ${v}_$rep || exit 1
  done
done
for v in pow nopow; do
  lib=lodestar_amd/liblodestar_bls.so; [ $v = nopow ] && lib=lodestar_amd/liblodestar_bls_nopow.so
  LSG_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pw_pmc_$v -o run -- python3 bench.py --steps 4 --warmup 2 --depth 1 --no-cpu-baseline > gpurun_out/pw_pmc_$v.log 2>&1 || exit 1
  echo PMC_$v
done
