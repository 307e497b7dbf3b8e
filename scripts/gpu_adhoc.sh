cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
timeout -k 10 300 python scripts/sweep.py --config cfg2 --regs 2 --grid 'PU_VARIANT=0,8' > gpurun_out/sweep_keep.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/sweep.py --config cfg2 --lnl-only --regs 0,2,4,6,8 > gpurun_out/sweep_lnlonly.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/sweep.py --config cfg3 --regs 0,1,2 > gpurun_out/sweep_cfg3.txt 2>&1 || exit $?
PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS|SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC|GRBM_GUI_ACTIVE GRBM_COUNT" bash scripts/pmc.sh --config cfg2 --regs 2
cat gpurun_out/sweep_keep.txt gpurun_out/sweep_lnlonly.txt gpurun_out/sweep_cfg3.txt
