#!/bin/bash
# PMC sets for the KEEP and LNL_ONLY traversal (one rocprofv3 pass per set); results in
# gpurun_out/pmc_keep and gpurun_out/pmc_lnl (summarise with scripts/pmc_summary.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE|SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS|SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU|SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU|SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INSTS_BRANCH|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQC_DCACHE_MISSES SQC_DCACHE_REQ|WRITE_SIZE|FETCH_SIZE"
PMC_SETS="$SETS" bash scripts/pmc.sh --config ${CFG:-cfg2} --grid "PU_LDS_SLOTS=${KEEP_SLOTS:-2}" || exit $?
rm -rf gpurun_out/pmc_keep && mv gpurun_out/pmc gpurun_out/pmc_keep
PMC_SETS="$SETS" bash scripts/pmc.sh --config ${CFG:-cfg2} --lnl-only --grid "PU_LDS_SLOTS=${LNL_SLOTS:-2}" || exit $?
rm -rf gpurun_out/pmc_lnl && mv gpurun_out/pmc gpurun_out/pmc_lnl
