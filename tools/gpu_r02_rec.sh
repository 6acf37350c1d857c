#!/bin/bash
# round-2 records of the final build: GPU parity suite, every workload's bench line with its
# CPU baseline, the driver's short run against a long run, rocprofv3 kernel stats of the
# default bench, then the depth-1 isolation PMC passes (tools/gpu_pmc.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))" "$1" "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit 1
for w in jobs adversarial block sync gossip; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/rec_$w.log 2>&1 && summ gpurun_out/rec_$w.log $w || exit 1
done
timeout -k 10 400 python -u bench.py --workload block --no-cpu-baseline > gpurun_out/rec_block2.log 2>&1 && summ gpurun_out/rec_block2.log block_repeat &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/rec_short.log 2>&1 && summ gpurun_out/rec_short.log short &&
timeout -k 10 300 python -u bench.py --steps 300 --warmup 5 --no-cpu-baseline > gpurun_out/rec_long.log 2>&1 && summ gpurun_out/rec_long.log long &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/def_trace -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/def_bench.log 2>&1 && echo DEF_OK &&
bash tools/gpu_pmc.sh
