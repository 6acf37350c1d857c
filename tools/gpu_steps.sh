#!/bin/bash
# GPU-box runner: named steps, each under its own time limit, stopping at the first failure.
#   tools/gpu_steps.sh test smoke bench prof ...
# Outputs go to gpurun_out/ (merged back by gpurun); copy the ones to keep into profiles/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${LSG_TAG:-r03}
run() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/${TAG}_$name.log"
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
}
for step in "$@"; do
  # row:<step> / pair:<step> run <step> with the row / pair serial kernels (A/B against the
  # straight-line-program default); w4:<step> with the 4-bit-window signature scaling kernel;
  # nodedup:<step> hashing every set's message (no per-package message table); noagg:<step>
  # one Miller pair per set even when sets share a message; agg:<step> one pair per message
  if [ "${step#pair:}" != "$step" ]; then export LSG_SERIAL=pair TAG=${LSG_TAG:-r03}_pair; step=${step#pair:};
  elif [ "${step#row:}" != "$step" ]; then export LSG_SERIAL=row TAG=${LSG_TAG:-r03}_row; step=${step#row:};
  elif [ "${step#w4:}" != "$step" ]; then export LSG_SIG_SCALE=4 TAG=${LSG_TAG:-r03}_w4; step=${step#w4:};
  elif [ "${step#nodedup:}" != "$step" ]; then export LSG_MSG_DEDUP=0 TAG=${LSG_TAG:-r03}_nodedup; step=${step#nodedup:};
  elif [ "${step#noagg:}" != "$step" ]; then export LSG_MSG_AGG=0 TAG=${LSG_TAG:-r03}_noagg; step=${step#noagg:};
  elif [ "${step#agg:}" != "$step" ]; then export LSG_MSG_AGG=1 TAG=${LSG_TAG:-r03}_agg; step=${step#agg:};
  else unset LSG_SERIAL LSG_SIG_SCALE LSG_MSG_DEDUP LSG_MSG_AGG; TAG=${LSG_TAG:-r03}; fi
  case $step in
    test) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ;;
    test-*) run "pytest_${step#test-}" 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -k "${step#test-}" ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python -u bench.py ;;
    bench-short) run bench_short 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    bench-*) w=${step#bench-}; run "bench_$w" 400 python -u bench.py --workload "$w" --no-cpu-baseline ;;
    depth-*) a=${step#depth-}; w=${a%%:*}; d=${a#*:}; run "bench_${w}_d$d" 400 python -u bench.py --workload "$w" --depth "$d" --no-cpu-baseline ;;
    co-*) a=${step#co-}; w=${a%%:*}; r=${a#*:}; d=${r%%:*}; f=${r#*:}; run "bench_${w}_d${d}_f$f" 400 python -u bench.py --workload "$w" --depth "$d" --coalesce-inflight "$f" --no-cpu-baseline ;;
    devices1) run bench_devices1 400 python -u bench.py --devices 1 --steps 20 --warmup 5 --no-cpu-baseline ;;
    devhost-*) n=${step#devhost-}; run "bench_devhost_$n" 400 python -u bench.py --devices "$n" --devices-same --depth 3 --steps 12 --warmup 3 --packages 2 --no-cpu-baseline ;;
    node) run bench_node 400 python -u bench.py --workload node --no-cpu-baseline ;;
    node-semi128) run bench_node_semi128 400 python -u bench.py --workload node --no-cpu-baseline "--node-flags=--max-old-space-size=4096 --max-semi-space-size=128" ;;
    node-semi256) run bench_node_semi256 400 python -u bench.py --workload node --no-cpu-baseline "--node-flags=--max-old-space-size=4096 --max-semi-space-size=256" ;;
    node-s128p98k) run bench_node_s128p98k 400 python -u bench.py --workload node --no-cpu-baseline "--node-flags=--max-old-space-size=4096 --max-semi-space-size=128" --node-max-pending 98304 ;;
    node-mm128) run bench_node_mm128 400 python -u bench.py --workload node --no-cpu-baseline "--node-flags=--max-old-space-size=4096 --min-semi-space-size=128 --max-semi-space-size=128" ;;
    node-mm64) run bench_node_mm64 400 python -u bench.py --workload node --no-cpu-baseline "--node-flags=--max-old-space-size=4096 --min-semi-space-size=64 --max-semi-space-size=64" ;;
    node-gc) run node_gc 300 node --max-old-space-size=4096 --max-semi-space-size=64 --trace-gc bench/bench_node.js --steps 150 --warmup 10 ;;
    node-long) run bench_node_long 400 python -u bench.py --workload node --no-cpu-baseline --steps 150 --warmup 10 ;;
    node-long128) run bench_node_long128 400 python -u bench.py --workload node --no-cpu-baseline --steps 150 --warmup 10 "--node-flags=--max-old-space-size=4096 --min-semi-space-size=128 --max-semi-space-size=128" ;;
    hwq32-*) w=${step#hwq32-}; export LSG_HW_QUEUES=32 && run "bench_${w}_hwq32" 400 python -u bench.py --workload "$w" --depth 16 --no-cpu-baseline && unset LSG_HW_QUEUES ;;
    node-p98k) run bench_node_p98k 400 python -u bench.py --workload node --no-cpu-baseline --node-max-pending 98304 ;;
    node-nosemi) run bench_node_nosemi 400 python -u bench.py --workload node --no-cpu-baseline --node-flags=--max-old-space-size=4096 ;;
    node-prof) mkdir -p gpurun_out/nodeprof && export LSG_NODE_CPUPROF=gpurun_out/nodeprof/bench_node.cpuprofile &&
               run bench_node_prof 400 python -u bench.py --workload node --no-cpu-baseline --steps 15 && unset LSG_NODE_CPUPROF ;;
    prof) run rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    pmc) run pmc 900 bash tools/gpu_pmc.sh ;;
    trace-*) w=${step#trace-}; run "trace_$w" 400 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/trace_$w" -o run -- python3 bench.py --workload "$w" --steps 20 --warmup 4 --no-cpu-baseline ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all steps ok"
