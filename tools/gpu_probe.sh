# Fp-multiplication microbenchmarks of candidate backends (tools/micro/probe_fpmul.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/micro/fpmul_probe 256 > gpurun_out/fpmul_probe.log 2>&1 || { cat gpurun_out/fpmul_probe.log; exit 1; }
grep RATE gpurun_out/fpmul_probe.log
python3 tools/micro/check_fpmul.py gpurun_out/fpmul_probe.log
