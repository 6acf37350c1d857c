#!/bin/bash
# GPU tests, then the jobs bench: default build vs h2c kernels at 1 wave/SIMD (A/B library)
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], {x: k.get(x) for x in ('k_pk_scale','k_h2c_map','k_h2c_clear')})" "$1" "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bm_def$i.log 2>&1 && summ gpurun_out/bm_def$i.log default &&
LSG_LIB=lodestar_amd/liblodestar_bls_h2c1.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bm_h2c1_$i.log 2>&1 && summ gpurun_out/bm_h2c1_$i.log h2c1 || exit 1
done
