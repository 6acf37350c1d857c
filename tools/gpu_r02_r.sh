#!/bin/bash
# round-2 re-entry: full GPU parity suite, the default bench (with CPU baseline), then an A/B
# of the interleaved Fp2 leaves (default) against three separate product calls
# (liblodestar_bls_nofp2.so, -DLSG_NO_FP2_LEAF), pipelined and depth 1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], r['kernel'], r['frac'], r['kernel_ms'], json.dumps(k))" "$1" "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 && summ gpurun_out/bench_default.log fp2leaf &&
LSG_LIB=lodestar_amd/liblodestar_bls_nofp2.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_nofp2.log 2>&1 && summ gpurun_out/bench_nofp2.log nofp2 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --depth 1 --steps 8 > gpurun_out/bench_d1.log 2>&1 && summ gpurun_out/bench_d1.log fp2leaf_d1 &&
LSG_LIB=lodestar_amd/liblodestar_bls_nofp2.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --depth 1 --steps 8 > gpurun_out/bench_nofp2_d1.log 2>&1 && summ gpurun_out/bench_nofp2_d1.log nofp2_d1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_short.log 2>&1 && summ gpurun_out/bench_short.log short
