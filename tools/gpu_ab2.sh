set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for spec in ${SPECS}; do IFS=: read lib g d <<< "$spec"
LSG_LIB=$PWD/lodestar_amd/$lib timeout -k 10 200 python -u bench.py --steps ${STEPS:-192} --warmup 24 --groups $g --depth $d --no-cpu-baseline > gpurun_out/ab2.log 2>&1 || { tail -5 gpurun_out/ab2.log; exit 1; }
tail -1 gpurun_out/ab2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', d['value'], 'p50', d['p50_batch_latency_ms'])"
done
