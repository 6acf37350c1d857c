# PMC passes over a short bench run (one counter group per pass, each under its own kill timer)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmc1 -o run -- python3 bench.py --steps 6 --warmup 1 --depth 4 --no-cpu-baseline > gpurun_out/pmc1.log 2>&1 && echo PMC1_OK &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d gpurun_out/pmc2 -o run -- python3 bench.py --steps 6 --warmup 1 --depth 4 --no-cpu-baseline > gpurun_out/pmc2.log 2>&1 && echo PMC2_OK
