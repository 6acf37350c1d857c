# Kernel isolation profile of the jobs path (depth 1: one package at a time, so each kernel's
# duration is its own, not a share of the chip): kernel stats, then one PMC group per pass
# (MI355X_MICROARCH.md: separate --pmc passes, no trace domains with --pmc), each under its own
# kill timer.  tools/pmc_summary.py turns the outputs into profiles/<round>_pmc_*.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps 6 --warmup 2 --depth 1 --no-cpu-baseline --sets-per-step ${LSG_PMC_SETS:-32768}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/iso_trace -o run -- python3 $B > gpurun_out/iso_trace.log 2>&1 && echo TRACE_OK &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d gpurun_out/iso_sq -o run -- python3 $B > gpurun_out/iso_sq.log 2>&1 && echo SQ_OK &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_THREAD_CYCLES_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/iso_sq2 -o run -- python3 $B > gpurun_out/iso_sq2.log 2>&1 && echo SQ2_OK &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/iso_fetch -o run -- python3 $B > gpurun_out/iso_fetch.log 2>&1 && echo FETCH_OK &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/iso_write -o run -- python3 $B > gpurun_out/iso_write.log 2>&1 && echo WRITE_OK
