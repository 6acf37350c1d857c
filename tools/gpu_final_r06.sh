#!/bin/bash
# GPU-box: the round-6 final records, in named parts (each step under its own time limit,
# stopping at the first failure).  Outputs under gpurun_out/final/; the ones kept are copied
# into profiles/r06_*.
#   tools/gpu_final_r06.sh core        GPU suite, smoke, default bench x3, Node drop-in x3
#   tools/gpu_final_r06.sh workloads   every bench workload once, lone set, 2 x committees
#   tools/gpu_final_r06.sh prof        rocprofv3 kernel stats of the default bench + PMC isolation
#   tools/gpu_final_r06.sh soak        10^7-set verdict soak (soak-threads: 4 submitters, 3 duplicate device ids)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/final
mkdir -p $out
run() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  tail -2 "$out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
}
for part in "$@"; do
  case $part in
    core)
      run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread
      run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
      for k in 1 2 3; do run "bench_$k" 400 python -u bench.py; done
      for k in 1 2 3; do run "bench_node_$k" 400 python -u bench.py --workload node --no-cpu-baseline; done
      LSG_NODE_CPUPROF=$PWD/$out/node.cpuprofile run bench_node_prof 400 python -u bench.py --workload node --no-cpu-baseline
      python3 tools/node_prof_summary.py $out/node.cpuprofile 30 > $out/node_prof.txt ;;
    workloads)
      for w in block gossip sync adversarial committees single; do run "bench_$w" 400 python -u bench.py --workload $w --no-cpu-baseline; done ;;
    prof)
      run rocprof 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
      run pmc 900 bash tools/gpu_pmc.sh ;;
    soak)
      run soak 1100 python -u tests/soak.py --sets 10000000 ;;
    soak-threads)  # four submitting threads on a context over three duplicate ids of the GPU
      run soak_threads 1100 python -u tests/soak.py --sets 10000000 --seed 2 --devices 3 --submitters 4 ;;
    *) echo "unknown part $part"; exit 2 ;;
  esac
done
echo "== all parts ok"
