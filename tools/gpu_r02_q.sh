#!/bin/bash
# fused Miller kernel, rebalanced M phase: parity vs split, jobs bench, depth-1 isolation
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], r['kernel'], r['frac'], r['kernel_ms'])" "$1" "$2"; }
timeout -k 10 200 python -u tools/dbg/fused_vs_split.py &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_cfg.log 2>&1 && tail -1 gpurun_out/pytest_cfg.log &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bq_fused.log 2>&1 && summ gpurun_out/bq_fused.log fused &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --depth 1 --steps 8 > gpurun_out/bq_fused_d1.log 2>&1 && summ gpurun_out/bq_fused_d1.log fused_d1
