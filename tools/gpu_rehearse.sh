#!/bin/bash
# One-GPU rehearsal of the multi-rank node protocol: bench.py under
# torch.distributed.run with LSG_BENCH_REHEARSE=1 (gloo exchange through host memory, every
# rank on device 0), against the plain one-GPU path.  -> gpurun_out/r05_rehearse_*.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${REH_TAG:-r05}
one() {  # name ranks extra-args...
  local name=$1 n=$2; shift 2
  echo "== $name ($(date +%T))"
  LSG_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
    --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus "$n" --no-cpu-baseline "$@" \
    > "gpurun_out/${R}_rehearse_$name.json" 2> "gpurun_out/${R}_rehearse_$name.err"
  local rc=$?
  python3 -c "import json; d=json.loads(open('gpurun_out/${R}_rehearse_$name.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['node_check_host_ms_per_package'])" || true
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/${R}_rehearse_$name.err"; echo "== FAILED rc=$rc"; exit $rc; fi
}
plain() {
  echo "== plain ($(date +%T))"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > "gpurun_out/${R}_rehearse_plain.json" 2> "gpurun_out/${R}_rehearse_plain.err" || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${R}_rehearse_plain.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['p50_batch_latency_ms'])"
}
plain
one rank1 1
for n in ${REH_RANKS:-}; do one "ranks$n" "$n"; done
for extra in ${REH_EXTRA:-}; do one "rank1_$extra" 1 --depth "$extra"; done
for lag in ${REH_LAG:-}; do LSG_BENCH_NODE_LAG=$lag one "rank1_lag$lag" 1; done
echo "== all ok"
