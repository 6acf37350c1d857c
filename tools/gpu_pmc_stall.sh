# (see tools/pmc_stall_summary.py)
# Stall profile of the jobs path at depth 1 (one package at a time): where the waves wait
# (any / instruction issue / LDS), LDS bank conflicts, instruction-fetch requests.  One PMC
# pass per counter group, each under its own kill timer (MI355X_MICROARCH.md: separate --pmc
# passes, no trace domains with --pmc).  tools/pmc_stall_summary.py reads the outputs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps 6 --warmup 2 --depth 1 --no-cpu-baseline --sets-per-step 32768"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_IFETCH SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/stall_a -o run -- python3 $B > gpurun_out/stall_a.log 2>&1 && echo STALL_A_OK &&
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM --kernel-trace --output-format csv -d gpurun_out/stall_b -o run -- python3 $B > gpurun_out/stall_b.log 2>&1 && echo STALL_B_OK
