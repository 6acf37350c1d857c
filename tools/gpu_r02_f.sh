# round 2: short distinct-set soak, then one bench line per workload (A-E) with its CPU baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tests/soak.py --sets 400000 > gpurun_out/soak_short.log 2>&1; echo "SOAK rc=$?"; tail -2 gpurun_out/soak_short.log
for w in jobs adversarial block sync gossip; do
  timeout -k 10 300 python -u bench.py --workload $w > gpurun_out/bench_$w.log 2>&1 || { echo "BENCH $w FAILED"; tail -5 gpurun_out/bench_$w.log; exit 1; }
  tail -1 gpurun_out/bench_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['value'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], d['roofline']['kernel'], d['roofline']['frac'], d['whole_path_mad_frac'], (d['cpu_baseline'] or {}).get('value'))"
done
