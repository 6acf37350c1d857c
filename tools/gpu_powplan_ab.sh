#!/bin/bash
# GPU-box: A/B of the fixed-exponent power (lsg_fp_pair.hpp): the compile-time plan
# (pair_pow_plan, shipped) against the bit-scanning leaf (pair_pow_fixed, built with
# -DLSG_NO_POW_PLAN into lodestar_amd/liblodestar_bls_noplan.so).  Default bench and lone set,
# alternating, then kernel stats of both.  Outputs under gpurun_out/powplan/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/powplan
mkdir -p $out
NOPLAN=$PWD/lodestar_amd/liblodestar_bls_noplan.so
run() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  tail -1 "$out/$name.log" | cut -c1-260
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
}
[ "${SKIP_TESTS:-0}" = 1 ] || run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread
for k in 1 2; do
  LSG_LIB=$NOPLAN run "noplan_bench_$k" 400 python -u bench.py --no-cpu-baseline
  run "plan_bench_$k" 400 python -u bench.py --no-cpu-baseline
done
LSG_LIB=$NOPLAN run noplan_single 300 python -u bench.py --workload single --no-cpu-baseline
run plan_single 300 python -u bench.py --workload single --no-cpu-baseline
run plan_prof 400 rocprofv3 --kernel-trace --stats -d $out/plan_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
LSG_LIB=$NOPLAN run noplan_prof 400 rocprofv3 --kernel-trace --stats -d $out/noplan_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo "== all ok"
