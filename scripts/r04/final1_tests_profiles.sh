# r04 final, call 1: GPU tests + smoke on the installed build, then per config the rocprofv3
# kernel trace, the PMC FETCH / WRITE passes and the instruction-mix pass (no bench lines:
# those are taken once these profiles are committed, so their roofline reads them)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
INSTS=1 BENCH=0 CONFIGS="cfg2 cfg3 cfg4 cfg5:--lnl-only:_lnl" bash scripts/gpu_profiles.sh
# ptah = the lnL-only tip-product rows requested one op ahead (-DPU_PT_AHEAD): parity tests,
# then cfg5 A/B (one tree alone, sweep.py; the 125-tree bench)
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
