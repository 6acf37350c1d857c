#!/bin/bash
# round-2 record of the current build: GPU parity suite, default bench (with CPU baseline),
# rocprofv3 kernel stats of the default bench, then the depth-1 isolation PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log | cut -c1-300 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/def_trace -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/def_bench.log 2>&1 && echo DEF_OK &&
bash tools/gpu_pmc.sh
