#!/bin/bash
# GPU-box A/B of the hardware-queue count: the library's own setting
# (lsg_init_devices sets GPU_MAX_HW_QUEUES=16 before its first HIP call) against LSG_HW_QUEUES=4
# (HIP's default) and 16, interleaved, for the jobs, gossip and Node workloads.
#   bash tools/gpu_hwq_ab.sh      -> gpurun_out/r05_hwq_<workload>_<setting>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "box environment: GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-<unset>}"
unset LSG_HW_QUEUES
one() {  # setting workload
  local q=$1 w=$2 out="gpurun_out/r05_hwq_${2}_${1}"
  echo "== hwq=$q $w ($(date +%T))"
  if [ "$q" = lib ]; then  # the library's own setting, over whatever the box exports
    timeout -k 10 300 python -u bench.py --workload "$w" --no-cpu-baseline > "$out.json" 2> "$out.err"
  else
    LSG_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --workload "$w" --no-cpu-baseline > "$out.json" 2> "$out.err"
  fi
  local rc=$?
  python3 -c "import json,sys; d=json.loads(open('$out.json').read().splitlines()[-1]); print(d['value'], d['p50_batch_latency_ms'])" || true
  if [ $rc -ne 0 ]; then tail -5 "$out.err"; echo "== FAILED rc=$rc"; exit $rc; fi
}
for w in ${HWQ_WORKLOADS:-jobs gossip node}; do
  for q in lib 4 16; do one "$q" "$w"; done
done
echo "== all ok"
