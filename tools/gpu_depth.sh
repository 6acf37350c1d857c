set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for d in 2 4 6; do
timeout -k 10 200 python -u bench.py --steps 24 --warmup 6 --depth $d --no-cpu-baseline > gpurun_out/bench_d$d.log 2>&1 || exit 1
tail -1 gpurun_out/bench_d$d.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($d, d['value'], d['p50_batch_latency_ms'], d['ms_per_step'])"
done
