# HBM traffic per kernel dispatch (MI355X_MICROARCH.md HBM/rocprofv3 section): FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes over a short default-shaped bench run (12 groups x 4096
# sets per submission), each pass under its own kill timer.  tools/pmc_traffic.py turns the
# CSVs into profiles/<round>_pmc_traffic.json, which bench.py reads for roofline.traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/traffic_fetch -o run -- python3 bench.py --steps 24 --warmup 12 --depth 2 --no-cpu-baseline > gpurun_out/traffic_fetch.log 2>&1 && echo FETCH_OK &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/traffic_write -o run -- python3 bench.py --steps 24 --warmup 12 --depth 2 --no-cpu-baseline > gpurun_out/traffic_write.log 2>&1 && echo WRITE_OK
