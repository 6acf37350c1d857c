# A/B: the same bench on alternative builds of the library (LSG_LIB), unloaded and loaded
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for lib in ${LIBS}; do for k in ${KS:-2}; do
LSG_LIB=$PWD/lodestar_amd/$lib LSG_MILLER_K=$k timeout -k 10 200 python -u bench.py --steps 32 --warmup 8 --no-cpu-baseline ${BARGS} > gpurun_out/ab_${lib}_${k}.log 2>&1 || { tail -5 gpurun_out/ab_${lib}_${k}.log; exit 1; }
tail -1 gpurun_out/ab_${lib}_${k}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib K$k', d['value'], 'p50', d['p50_batch_latency_ms'], 'unloaded', d['p50_unloaded_latency_ms'], {k: v for k, v in d['kernel_ms'].items() if v > 1})"
done; done
