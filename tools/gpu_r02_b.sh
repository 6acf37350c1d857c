# round 2: allocation trace of the reserve test; package size / depth / K sweep of the jobs bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
LSG_TRACE_ALLOC=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -k "reserve" -v -s --timeout 240 --timeout-method thread > gpurun_out/alloc_trace.log 2>&1; echo "reserve rc=$?"
for cfg in "16384 3" "32768 2" "32768 4" "49152 3" "65536 2" "65536 3"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --steps 16 --warmup 4 --sets-per-step $1 --depth $2 --no-cpu-baseline > gpurun_out/sweep_$1_$2.log 2>&1 || { echo "FAIL $cfg"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_$1_$2.log').read().strip().splitlines()[-1]); print('$1 $2', d['value'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], d['roofline']['kernel_ms'], d['allocations_in_timed_region'])"
done
LSG_MILLER_K=2 timeout -k 10 200 python -u bench.py --steps 16 --warmup 4 --sets-per-step 32768 --depth 3 --no-cpu-baseline > gpurun_out/sweep_k2.log 2>&1 && python3 -c "import json; d=json.loads(open('gpurun_out/sweep_k2.log').read().strip().splitlines()[-1]); print('K2 32768 3', d['value'], d['p50_batch_latency_ms'], d['roofline']['kernel_ms'])"
