#!/bin/bash
# register-budget A/B (512-register waves instead of spilling): default vs -DLSG_MF_WAVES=1
# (fused Miller kernel) vs -DLSG_H2C_WAVES=1 (hash map / cofactor clearing), interleaved,
# then the memory-side traffic of the fused kernel at depth 1 for default and MF_WAVES=1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']; r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], r['kernel'], r['frac'], r['kernel_ms'])" "$1" "$2"; }
for rep in 1 2; do
  for v in default mf1 h1; do
    lib=lodestar_amd/liblodestar_bls.so; [ $v != default ] && lib=lodestar_amd/liblodestar_bls_$v.so
    LSG_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab_${v}_$rep.log 2>&1 || exit 1
    summ gpurun_out/ab_${v}_$rep.log ${v}_$rep || exit 1
  done
done
B="bench.py --steps 4 --warmup 2 --depth 1 --no-cpu-baseline"
for v in default mf1; do
  lib=lodestar_amd/liblodestar_bls.so; [ $v != default ] && lib=lodestar_amd/liblodestar_bls_$v.so
  LSG_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/tr_f_$v -o run -- python3 $B > gpurun_out/tr_f_$v.log 2>&1 || exit 1
  LSG_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/tr_w_$v -o run -- python3 $B > gpurun_out/tr_w_$v.log 2>&1 || exit 1
  echo TRAFFIC_$v
done
