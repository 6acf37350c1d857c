# round 2: full GPU tests (alloc trace on the reserve test), K x depth sweep at 32k packages
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "PYTEST rc=$?"; tail -3 gpurun_out/pytest_gpu.log
grep -q "Fatal\|core dumped\|Segmentation" gpurun_out/pytest_gpu.log && exit 3
LSG_TRACE_ALLOC=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -k "reserve" -v -s --timeout 240 --timeout-method thread > gpurun_out/alloc_trace.log 2>&1; echo "reserve rc=$?"
for cfg in "4 32768 3" "2 32768 3" "2 32768 4" "2 49152 3" "4 49152 4"; do
  set -- $cfg
  LSG_MILLER_K=$1 timeout -k 10 200 python -u bench.py --steps 16 --warmup 4 --sets-per-step $2 --depth $3 --no-cpu-baseline > gpurun_out/sweep_$1_$2_$3.log 2>&1 || { echo "FAIL $cfg"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_$1_$2_$3.log').read().strip().splitlines()[-1]); print('K$1 $2 d$3', d['value'], d['p50_batch_latency_ms'], d['p50_unloaded_latency_ms'], d['roofline']['kernel_ms'], d['host_submit_ms_per_package'], d['allocations_in_timed_region'])"
done
