#!/bin/bash
# segmented reductions (throughput-mode chunking for work-bound passes):
# parity suite, then the block, sync and jobs workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], 'agg', k.get('g1_aggregate'), 'msm', k.get('msm_buckets'), k.get('msm_bits'))" "$1" "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for w in block sync jobs block sync; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/lds_$w.log 2>&1 && summ gpurun_out/lds_$w.log $w || exit 1
done
