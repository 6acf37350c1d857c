#!/bin/bash
# GPU-box: host staging of a multi-device context rehearsed on one GPU (duplicate device ids,
# bench.py --devices N --devices-same): submit-call wall time and host submit time per package
# for LSG_STAGE_PAR = 0 (devices staged one after another, round 5), 1 (part 1 on threads),
# 2 (parts 1 and 2 on threads; shipped) -- VERDICT r5 item 3.  A/B build (liblodestar_bls_ab.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/devhost
mkdir -p $out
one() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --devices-same --depth 3 --steps 12 --warmup 3 --packages 2 \
    --no-cpu-baseline $BARGS > $out/$name.json 2> $out/$name.err || { echo "$name FAILED"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], 'host_submit', d['host_submit_ms_per_package'], 'call_p50_max', d['submit_call_ms_p50_max'], 'cores', d['host_cpu_cores_busy'])"
}
AB=LSG_LIB=$PWD/lodestar_amd/liblodestar_bls_ab.so
for rep in 1 2 3; do
  BARGS="--devices 1" one "n1_r$rep" X=1
  for n in 2 4 8; do
    for par in 0 1 2; do BARGS="--devices $n" one "n${n}_par${par}_r$rep" $AB LSG_STAGE_PAR=$par; done
  done
done
