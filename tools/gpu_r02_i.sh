#!/bin/bash
# every workload's bench line with its CPU baseline, then the driver's short run vs a long run
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))" "$1" "$2"; }
for w in jobs adversarial block sync gossip; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/bi_$w.log 2>&1 && summ gpurun_out/bi_$w.log $w || exit 1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bi_short.log 2>&1 && summ gpurun_out/bi_short.log short &&
timeout -k 10 300 python -u bench.py --steps 300 --warmup 5 --no-cpu-baseline > gpurun_out/bi_long.log 2>&1 && summ gpurun_out/bi_long.log long
