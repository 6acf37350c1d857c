#!/bin/bash
# one GPU: jobs bench under the three wait strategies (inline, threads spinning, threads sleeping)
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], d['host_submit_ms_per_package'])" "$1" "$2"; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --waits inline > gpurun_out/bh_inline.log 2>&1 && summ gpurun_out/bh_inline.log inline &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --waits thread > gpurun_out/bh_thread.log 2>&1 && summ gpurun_out/bh_thread.log thread &&
LSG_BLOCKING_WAITS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --waits thread > gpurun_out/bh_tblock.log 2>&1 && summ gpurun_out/bh_tblock.log thread_blocking &&
LSG_BLOCKING_WAITS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --waits inline > gpurun_out/bh_iblock.log 2>&1 && summ gpurun_out/bh_iblock.log inline_blocking
