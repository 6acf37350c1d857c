# GPU check: parity tests (stop at first failure), then one bench line (default shape unless
# BENCH_ARGS is set)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_check.log 2>&1 || { tail -5 gpurun_out/bench_check.log; exit 1; }
tail -1 gpurun_out/bench_check.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'p50', d['p50_batch_latency_ms'], 'ms/step', d['ms_per_step'], 'frac', d['whole_path_mad_frac'], 'cpu', d['cpu_baseline']); print({k: v for k, v in d['kernel_ms'].items() if v > 0.2})"
