# Interleaved repeats of the default bench at a few (groups x depth) shapes, 384 steps each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do for cfg in ${CFGS:-6x4 12x3 12x4}; do set -- ${cfg/x/ }
timeout -k 10 200 python -u bench.py --steps 384 --warmup 48 --groups $1 --depth $2 --no-cpu-baseline > gpurun_out/shape_$1_$2_$rep.log 2>&1 || { tail -5 gpurun_out/shape_$1_$2_$rep.log; exit 1; }
tail -1 gpurun_out/shape_$1_$2_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rep $rep groups', $1, 'depth', $2, d['value'], 'p50', d['p50_batch_latency_ms'])"
done; done
