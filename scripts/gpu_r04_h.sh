# r04: (1) ptah = the lnL-only tip-product rows requested one op ahead (-DPU_PT_AHEAD): parity
# tests, then cfg5 A/B (one tree alone, sweep.py; the 125-tree bench); (2) protein diagnostics:
# per-phase s_memtime ticks of one wave (timing build) and the TA path beside the matrix cores
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/phylo_utils_amd
PHYLO_HIP_LIB=$L/libphylo_hip_ptah.so timeout -k 10 300 python -u -m pytest \
  tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_ptah.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ptah.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lib in libphylo_hip.so libphylo_hip_ptah.so; do
    PHYLO_HIP_LIB=$L/$lib timeout -k 10 300 python scripts/sweep.py --config cfg5 --lnl-only \
      --steps 200 --rounds 3 2>/dev/null | tail -1 | sed "s/^/$lib one tree: /" | tee -a gpurun_out/ab_r04h.txt
    PHYLO_HIP_LIB=$L/$lib timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 5 \
      --no-cpu-baseline > gpurun_out/ab_line.json 2> gpurun_out/ab_err.txt || exit $?
    python -c "
import json; d = json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1])
print('$lib cfg5 bench: step %.4f ms value %.1f lnl %r' % (d['ms_per_step'], d['value'], d.get('lnl')))" | tee -a gpurun_out/ab_r04h.txt
  done
done
PHYLO_HIP_LIB=$L/libphylo_hip_timing.so PU_TIMING=1 timeout -k 10 300 \
  python bench.py --config cfg3 --steps 50 --warmup 5 --no-cpu-baseline \
  > gpurun_out/timing_cfg3.json 2> gpurun_out/timing_cfg3.txt || exit $?
grep "pu timing" gpurun_out/timing_cfg3.txt | tail -2 || true
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc_avail.txt 2>&1 || true
SETS="TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE|SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
PMC_SETS="$SETS" bash scripts/pmc.sh --config cfg3 || exit $?
PHYLO_HIP_LIB=$L/libphylo_hip_ldsp.so PMC_DIR=pmc_ldsp PMC_SETS="$SETS" bash scripts/pmc.sh --config cfg3
