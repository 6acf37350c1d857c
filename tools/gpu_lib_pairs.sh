#!/bin/bash
# GPU-box: pairs of runs of an alternative build of the library (argument 1, an in-tree .so built with
# extra flags) against the shipped one, alternating on the same box.  Argument 2 names the
# output directory under gpurun_out/; further arguments are the workloads (default: jobs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ALT=$PWD/$1
tag=$2
shift 2
workloads=${*:-jobs}
out=gpurun_out/$tag
mkdir -p $out
run() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -3 "$out/$name.log"; exit $rc; fi
  python3 -c "
import json; d=json.loads(open('$out/$name.log').read().strip().splitlines()[-1])
print('%-22s %12.1f  p50 %s ms' % ('$name', d['value'], d['p50_batch_latency_ms']))"
}
for k in $(seq 1 ${REPS:-3}); do
  for w in $workloads; do
    LSG_LIB=$ALT run "alt_${w}_$k" 300 python -u bench.py --workload $w --no-cpu-baseline
    run "base_${w}_$k" 300 python -u bench.py --workload $w --no-cpu-baseline
  done
done
echo "== all ok"
