#!/bin/bash
# PMC sets for the KEEP and LNL_ONLY traversal (cfg2), one rocprofv3 pass per set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE|SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS|SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU|SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQ_INST_LEVEL_SMEM|SQ_INST_CYCLES_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS|SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INSTS_BRANCH"
PMC_SETS="$SETS" bash scripts/pmc.sh --config ${CFG:-cfg2} --grid "PU_REGS:PU_LDS_SLOTS=${KEEP_SLOTS:-3:0}" || exit $?
mv gpurun_out/pmc gpurun_out/pmc_keep
PMC_SETS="$SETS" bash scripts/pmc.sh --config ${CFG:-cfg2} --lnl-only --grid "PU_REGS:PU_LDS_SLOTS=${LNL_SLOTS:-2:0}" || exit $?
mv gpurun_out/pmc gpurun_out/pmc_lnl
