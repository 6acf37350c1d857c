# kernel-trace timeline of a short bench run (for overlap / queue analysis)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- python3 bench.py --steps 32 --warmup 8 --depth ${DEPTH:-3} --groups ${NGROUPS:-4} --no-cpu-baseline > gpurun_out/trace.log 2>&1 && tail -1 gpurun_out/trace.log | cut -c1-200
