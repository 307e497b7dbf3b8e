# r04: aast = protein CLVs stored as row pairs (two 16-byte + one 8-byte store per lane and op
# instead of five 8-byte ones): GPU tests on that build, cfg3 A/B; then the default-plan sweep
#  on the installed build
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/phylo_utils_amd
PHYLO_HIP_LIB=$L/libphylo_hip_aast.so timeout -k 10 540 python -u -m pytest \
  tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_aast.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_aast.log; [ $rc -ne 0 ] && exit $rc
run() {  # label, then env assignments; one bench line, summarised
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-200} --warmup 20 \
      --no-cpu-baseline $ARGS > gpurun_out/ab_line.json 2> gpurun_out/ab_err.txt
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/ab_err.txt; exit $rc; fi
  python -c "
import json; d = json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1])
t = d.get('timing', {})
print('%-6s %-8s step %.5f ms  kernel %.5f ms  value %.1f  lnl %r' % ('$CFG$ARGS', '$label', d['ms_per_step'],
      t.get('kernel_ms_median', float('nan')), d['value'], d.get('lnl')))" | tee -a gpurun_out/ab_r04i.txt
}
CFG=cfg3
for i in 1 2 3; do
  run A PU_AB=A
  run aast PHYLO_HIP_LIB=$L/libphylo_hip_aast.so
done
ARGS=--lnl-only
for i in 1 2; do
  run A PU_AB=A
  run aast PHYLO_HIP_LIB=$L/libphylo_hip_aast.so
done
bash scripts/gpu_r04_sweep.sh
