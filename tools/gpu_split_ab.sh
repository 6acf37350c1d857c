# Split Miller loop bring-up: GPU parity suite on the default build, then the bench over
# SPECS = "lib:K:split" (split=0: fused k_miller_multi; 1: k_miller_lines + k_miller_accum)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/split_pytest.log 2>&1 || { tail -40 gpurun_out/split_pytest.log; exit 1; }
tail -1 gpurun_out/split_pytest.log
for spec in ${SPECS}; do IFS=: read lib k sp <<< "$spec"
LSG_LIB=$PWD/lodestar_amd/$lib LSG_MILLER_K=$k LSG_MILLER_SPLIT=$sp timeout -k 10 200 python -u bench.py --steps ${STEPS:-96} --warmup 12 --no-cpu-baseline ${BARGS} > gpurun_out/split_${lib}_${k}_${sp}.log 2>&1 || { tail -5 gpurun_out/split_${lib}_${k}_${sp}.log; exit 1; }
tail -1 gpurun_out/split_${lib}_${k}_${sp}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', d['value'], 'p50', d['p50_batch_latency_ms'], 'unloaded', d['p50_unloaded_latency_ms'], {k: v for k, v in d['kernel_ms'].items() if v > 1})"
done
