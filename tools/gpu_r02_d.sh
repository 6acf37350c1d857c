# round 2: instruction-rate probe, GPU tests, jobs bench 32k x depth 4 with rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/irate_probe > gpurun_out/irate.log 2>&1; cat gpurun_out/irate.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "PYTEST rc=$?"; tail -3 gpurun_out/pytest_gpu.log
grep -q "Fatal\|core dumped\|Segmentation" gpurun_out/pytest_gpu.log && exit 3
timeout -k 10 300 python -u bench.py --steps 24 --warmup 4 --depth 4 > gpurun_out/bench_d4.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench_d4.log | cut -c1-600 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d -o run -- python -u bench.py --steps 24 --warmup 4 --depth 4 --no-cpu-baseline > gpurun_out/bench_prof_d.log 2>&1 && echo PROF_OK
