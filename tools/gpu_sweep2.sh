# bench sweep over (groups per submission) x (submissions in flight); no parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in ${CFGS:-6x4 6x6 6x8 8x6 12x4 4x8}; do set -- ${cfg/x/ }
timeout -k 10 200 python -u bench.py --steps $((8 * $1 * $2)) --warmup $((2 * $1)) --groups $1 --depth $2 --no-cpu-baseline > gpurun_out/sw_$1_$2.log 2>&1 || { tail -5 gpurun_out/sw_$1_$2.log; exit 1; }
tail -1 gpurun_out/sw_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('groups', $1, 'depth', $2, d['value'], 'p50', d['p50_batch_latency_ms'], 'ms/step', d['ms_per_step'])"
done
