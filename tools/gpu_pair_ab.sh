# Pair-backend bring-up: GPU parity suite on one pair build, then the A/B bench over builds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LSG_LIB=$PWD/lodestar_amd/${PARITY_LIB:-ab_pair_w2.so} timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pair_pytest.log 2>&1 || { tail -40 gpurun_out/pair_pytest.log; exit 1; }
tail -3 gpurun_out/pair_pytest.log
LIBS="${LIBS}" KS="${KS:-2}" bash tools/gpu_ab.sh
