#!/bin/bash
# GPU-box: round-robin of several builds of the library on the same box.  Argument 1 names the
# output directory under gpurun_out/, argument 2 the workload, the rest are in-tree .so files
# ("base" = the shipped library).  REPS rounds (default 4), each build once per round.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1
w=$2
shift 2
out=gpurun_out/$tag
mkdir -p $out
for k in $(seq 1 ${REPS:-4}); do
  for lib in "$@"; do
    name=$(basename $lib .so)_$k
    if [ "$lib" = base ]; then
      timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $out/$name.log 2>&1
    else
      LSG_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $out/$name.log 2>&1
    fi
    rc=$?
    if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -3 $out/$name.log; exit $rc; fi
    python3 -c "
import json; d=json.loads(open('$out/$name.log').read().strip().splitlines()[-1])
print('%-28s %12.1f  p50 %s ms' % ('$name', d['value'], d['p50_batch_latency_ms']))"
  done
done
echo "== all ok"
