set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for k in ${KS:-1 2}; do for d in ${DEPTHS:-6 8 12}; do
LSG_MILLER_K=$k timeout -k 10 200 python -u bench.py --steps 24 --warmup 6 --depth $d --no-cpu-baseline > gpurun_out/sw_k${k}_d$d.log 2>&1 || { tail -5 gpurun_out/sw_k${k}_d$d.log; exit 1; }
tail -1 gpurun_out/sw_k${k}_d$d.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('K', $k, 'depth', $d, d['value'], 'p50', d['p50_batch_latency_ms'], 'ms/step', d['ms_per_step'])"
done; done
