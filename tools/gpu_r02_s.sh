#!/bin/bash
# instruction-supply check of the per-set kernels (depth-1 bench, one package at a time):
# instruction-cache hits/misses and instruction fetches against issued VALU instructions
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps 4 --warmup 2 --depth 1 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d gpurun_out/ic -o run -- python3 $B > gpurun_out/ic.log 2>&1 && echo IC_OK &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU --kernel-trace --output-format csv -d gpurun_out/ic2 -o run -- python3 $B > gpurun_out/ic2.log 2>&1 && echo IC2_OK
