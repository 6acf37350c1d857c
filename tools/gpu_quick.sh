# quick GPU check: parity tests (stop at first failure), then a short bench per depth
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for d in ${DEPTHS:-4}; do
timeout -k 10 200 python -u bench.py --steps 24 --warmup 6 --depth $d --no-cpu-baseline > gpurun_out/bench_d$d.log 2>&1 || { tail -5 gpurun_out/bench_d$d.log; exit 1; }
tail -1 gpurun_out/bench_d$d.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('depth', $d, d['value'], 'p50', d['p50_batch_latency_ms'], 'ms/step', d['ms_per_step'], 'probe', '%.3g'%d['probe_lane_fp_mul_per_s'], {k: v for k, v in d['kernel_ms'].items() if v > 0.2})"
done
