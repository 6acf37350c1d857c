# round 2: GPU tests, then the kernel isolation profile (tools/gpu_pmc.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "PYTEST rc=$?"; tail -3 gpurun_out/pytest_gpu.log
grep -q "Fatal\|core dumped\|Segmentation" gpurun_out/pytest_gpu.log && exit 3
bash tools/gpu_pmc.sh
