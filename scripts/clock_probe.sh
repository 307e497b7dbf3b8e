#!/bin/bash
# Effective GPU clock of the write-pattern probe kernels: kernel durations (kernel trace) and
# GRBM_GUI_ACTIVE (GPU-busy cycles per dispatch) in separate rocprofv3 passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/clk_trace gpurun_out/clk_pmc
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/clk_trace -- scripts/_write_pattern6 > gpurun_out/clk_trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/clk_pmc -- scripts/_write_pattern6 > gpurun_out/clk_pmc.log 2>&1 || exit $?
echo done
