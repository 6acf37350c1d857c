# round 2, first GPU pass: parity tests (all, verbose), a short jobs bench, its rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "PYTEST rc=$?"; tail -5 gpurun_out/pytest_gpu.log
grep -q "Fatal\|core dumped\|Segmentation" gpurun_out/pytest_gpu.log && exit 3
timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 && echo PROF_OK
