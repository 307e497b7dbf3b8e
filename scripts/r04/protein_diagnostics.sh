# r04: protein diagnostics -- per-phase s_memtime ticks of one wave (timing build) and the TA
# path beside the matrix cores (PMC), installed build and the LDS-staged variant
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/phylo_utils_amd
PHYLO_HIP_LIB=$L/libphylo_hip_timing.so PU_TIMING=1 timeout -k 10 300 \
  python bench.py --config cfg3 --steps 50 --warmup 5 --no-cpu-baseline \
  > gpurun_out/timing_cfg3.json 2> gpurun_out/timing_cfg3.txt || exit $?
grep "pu timing" gpurun_out/timing_cfg3.txt | tail -2 || true
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc_avail.txt 2>&1 || true
SETS="TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE|SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
PMC_SETS="$SETS" bash scripts/pmc.sh --config cfg3 || exit $?
PHYLO_HIP_LIB=$L/libphylo_hip_ldsp.so PMC_DIR=pmc_ldsp PMC_SETS="$SETS" bash scripts/pmc.sh --config cfg3
