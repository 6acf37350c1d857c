set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for k in 1 2 4; do for d in 4 6; do
LSG_MILLER_K=$k timeout -k 10 200 python -u bench.py --steps 24 --warmup 6 --depth $d --no-cpu-baseline > gpurun_out/bench_k${k}_d$d.log 2>&1 || { tail -5 gpurun_out/bench_k${k}_d$d.log; exit 1; }
tail -1 gpurun_out/bench_k${k}_d$d.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('K', $k, 'depth', $d, d['value'], 'p50', d['p50_batch_latency_ms'], 'miller', d['kernel_ms']['k_miller_multi'])"
done; done
