set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for cfg in ${CFGS:-1x6 2x3 4x2 4x3 8x2}; do set -- ${cfg/x/ }
timeout -k 10 200 python -u bench.py --steps 32 --warmup 8 --groups $1 --depth $2 --no-cpu-baseline > gpurun_out/ms_$1_$2.log 2>&1 || { tail -5 gpurun_out/ms_$1_$2.log; exit 1; }
tail -1 gpurun_out/ms_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('groups', $1, 'depth', $2, d['value'], 'p50', d['p50_batch_latency_ms'], 'ms/step', d['ms_per_step'])"
done
