# GPU-box: the default bench line REPS times back to back (the headline's spread on one box),
# then a kernel trace of the lone-set workload.  -> gpurun_out/<tag>_bench_rep<k>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${REP_TAG:-r05}
for k in $(seq 1 ${REPS:-3}); do
  timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench_rep$k.json 2> gpurun_out/${T}_bench_rep$k.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${T}_bench_rep$k.json').read().splitlines()[-1]); print('rep $k', d['value'], d['p50_batch_latency_ms'], d['whole_path_mad_frac'], d['roofline']['frac'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_single_prof -o single -- python3 bench.py --workload single --steps 40 --no-cpu-baseline > gpurun_out/${T}_single_prof.log 2>&1
