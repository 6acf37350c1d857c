#!/bin/bash
# fused Miller kernel (dynamic LDS, 2 waves/SIMD register budget): parity vs split, then benches
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], r['kernel'], r['frac'], r['kernel_ms'])" "$1" "$2"; }
timeout -k 10 200 python -u tools/dbg/fused_vs_split.py &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bo_fused.log 2>&1 && summ gpurun_out/bo_fused.log fused &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --depth 1 --steps 8 > gpurun_out/bo_fused_d1.log 2>&1 && summ gpurun_out/bo_fused_d1.log fused_d1 &&
LSG_MILLER_FUSED=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bo_split.log 2>&1 && summ gpurun_out/bo_split.log split
