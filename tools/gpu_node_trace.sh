#!/bin/bash
# GPU-box: kernel traces of the plain one-GPU path and the one-rank node-protocol rehearsal
# (bench.py run directly with the torch.distributed env of one rank, no launcher)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ntrace_plain -o run -- python3 bench.py --steps 30 --no-cpu-baseline \
  > gpurun_out/ntrace_plain.json 2> gpurun_out/ntrace_plain.err && echo PLAIN_OK &&
LSG_BENCH_REHEARSE=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 \
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ntrace_node -o run -- python3 bench.py --steps 30 --no-cpu-baseline \
  > gpurun_out/ntrace_node.json 2> gpurun_out/ntrace_node.err && echo NODE_OK
