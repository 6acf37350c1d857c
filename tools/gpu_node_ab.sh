#!/bin/bash
# GPU-box: the Node drop-in (bench.py --workload node) with the round-6 JS host against earlier
# builds (tools/ab/blsGpuVerifier_*.js), interleaved, plus a CPU profile of the JS thread
# (LSG_NODE_CPUPROF) -- VERDICT r5 item 1.  Records under gpurun_out/node_ab/.
# usage: tools/gpu_node_ab.sh "<name>:<verifier or ->:<max pending sigs>" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/node_ab
mkdir -p $out
for spec in "$@"; do
  IFS=: read -r name ver pend <<< "$spec"
  env=(X=1)
  [ "$ver" != "-" ] && env=(LSG_VERIFIER_JS=$PWD/$ver)
  [ "$name" = "prof" ] && env+=(LSG_NODE_CPUPROF=$PWD/$out/prof.cpuprofile)
  echo "== $name $ver $pend $(date +%T)"
  env "${env[@]}" timeout -k 10 240 python3 bench.py --workload node --no-cpu-baseline --node-max-pending "$pend" \
    > $out/$name.json 2> $out/$name.err || exit 1
  python3 -c "import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['p50_batch_latency_ms'], d['mean_package_sets'])"
done
if [ -f $out/prof.cpuprofile ]; then python3 tools/node_prof_summary.py $out/prof.cpuprofile 30 > $out/prof.txt && cat $out/prof.txt; fi
