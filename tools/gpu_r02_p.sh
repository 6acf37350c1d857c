#!/bin/bash
# round-2 profiles of the default bench: kernel stats of the bench command itself, a HIP API
# trace (no allocations inside the timed window), then the depth-1 isolation PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/def_trace -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/def_bench.log 2>&1 && echo DEF_OK &&
timeout -k 10 300 rocprofv3 --hip-trace --output-format csv -d gpurun_out/alloc_trace -o run -- python3 bench.py --no-cpu-baseline --steps 10 > gpurun_out/alloc_bench.log 2>&1 && echo ALLOC_OK &&
bash tools/gpu_pmc.sh
