#!/bin/bash
# pipelining variance: threaded vs inline waits, spinning vs sleeping completion events
set -o pipefail
mkdir -p gpurun_out
cat /proc/loadavg
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], d['host_submit_ms_per_package'], d['submit_call_ms_p50_max'])" "$1" "$2"; }
i=0
for mode in thread inline thread-b thread inline thread-b thread; do
  i=$((i+1)); w=${mode%-b}; b=0; [ "$mode" != "$w" ] && b=1
  LSG_BLOCKING_WAITS=$b timeout -k 10 200 python -u bench.py --no-cpu-baseline --waits $w > gpurun_out/bl_$i.log 2>&1 && summ gpurun_out/bl_$i.log $mode || exit 1
done
cat /proc/loadavg
