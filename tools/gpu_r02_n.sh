#!/bin/bash
# fused Miller kernel: GPU tests, then the jobs bench fused vs split (LSG_MILLER_FUSED=0)
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], r['kernel'], r['frac'], r['kernel_ms'], {x: k.get(x) for x in ('k_miller_fused','k_miller_accum','k_miller_lines')})" "$1" "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bn_fused.log 2>&1 && summ gpurun_out/bn_fused.log fused &&
LSG_MILLER_FUSED=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bn_split.log 2>&1 && summ gpurun_out/bn_split.log split &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --depth 1 --steps 8 > gpurun_out/bn_fused_d1.log 2>&1 && summ gpurun_out/bn_fused_d1.log fused_d1
