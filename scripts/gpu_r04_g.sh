# r04 A/B builds, tested then timed on one box:
#   aasw: register stash slots (TV_RSLOTS) + the protein op's one-load descriptor / switch
#   ldsp: aasw + the protein A operands staged through LDS by LDS-DMA (-DPU_AA_LDSP)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/phylo_utils_amd
PHYLO_HIP_LIB=$L/libphylo_hip_aasw.so timeout -k 10 540 python -u -m pytest \
  tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_aasw.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_aasw.log; [ $rc -ne 0 ] && exit $rc
PHYLO_HIP_LIB=$L/libphylo_hip_ldsp.so timeout -k 10 300 python -u -m pytest \
  tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_ldsp.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ldsp.log; [ $rc -ne 0 ] && exit $rc
run() {  # label, then env assignments; one bench line, summarised
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-200} --warmup 20 \
      --no-cpu-baseline > gpurun_out/ab_line.json 2> gpurun_out/ab_err.txt
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/ab_err.txt; exit $rc; fi
  python -c "
import json; d = json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1])
t = d.get('timing', {})
print('%-6s %-8s step %.5f ms  kernel %.5f ms  value %.1f  lnl %r' % ('$CFG', '$label', d['ms_per_step'],
      t.get('kernel_ms_median', float('nan')), d['value'], d.get('lnl')))" | tee -a gpurun_out/ab_r04g.txt
}
CFG=cfg3
for i in 1 2 3; do
  run A PU_AB=A
  run aasw PHYLO_HIP_LIB=$L/libphylo_hip_aasw.so
  run ldsp PHYLO_HIP_LIB=$L/libphylo_hip_ldsp.so
  run ldsp2 PHYLO_HIP_LIB=$L/libphylo_hip_ldsp.so PU_LDS_SLOTS=2
done
CFG=cfg4 STEPS=60
for i in 1 2 3; do
  run A PU_AB=A
  run aasw PHYLO_HIP_LIB=$L/libphylo_hip_aasw.so
done
