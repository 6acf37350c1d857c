cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/devtrace
LSG_TRACE_HOST=1 timeout -k 10 200 python3 bench.py --devices 1 --devices-same --depth 3 --steps 12 --warmup 3 --packages 2 --no-cpu-baseline > gpurun_out/devtrace/n1.json 2> gpurun_out/devtrace/n1.err &&
LSG_TRACE_HOST=1 timeout -k 10 200 python3 bench.py --devices 8 --devices-same --depth 3 --steps 12 --warmup 3 --packages 2 --no-cpu-baseline > gpurun_out/devtrace/n8.json 2> gpurun_out/devtrace/n8.err && echo done
