# r04: k_prune_mfma with two 16-site blocks per wave (PU_AA_NB=2, libphylo_hip_nb.so): the GPU
# suite with NB = 2 exported (every protein test on it) and the bitwise test, then cfg3 A/B
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/phylo_utils_amd
PHYLO_HIP_LIB=$L/libphylo_hip_nb.so PU_AA_NB=2 timeout -k 10 540 python -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_nb.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_nb.log; [ $rc -ne 0 ] && exit $rc
run() {  # label, then env assignments; one bench line, summarised
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config cfg3 --steps 200 --warmup 20 \
      --no-cpu-baseline $ARGS > gpurun_out/ab_line.json 2> gpurun_out/ab_err.txt
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/ab_err.txt; exit $rc; fi
  python -c "
import json; d = json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1])
t = d.get('timing', {})
print('cfg3%-10s %-6s step %.5f ms  kernel %.5f ms  value %.1f  lnl %r' % ('$ARGS', '$label', d['ms_per_step'],
      t.get('kernel_ms_median', float('nan')), d['value'], d.get('lnl')))" | tee -a gpurun_out/ab_r04m.txt
}
for i in 1 2 3; do
  run nb1 PHYLO_HIP_LIB=$L/libphylo_hip_nb.so PU_AA_NB=1
  run nb2 PHYLO_HIP_LIB=$L/libphylo_hip_nb.so PU_AA_NB=2
  run nb2s2 PHYLO_HIP_LIB=$L/libphylo_hip_nb.so PU_AA_NB=2 PU_LDS_SLOTS=2
done
ARGS=--lnl-only
for i in 1 2; do
  run nb1 PHYLO_HIP_LIB=$L/libphylo_hip_nb.so PU_AA_NB=1
  run nb2 PHYLO_HIP_LIB=$L/libphylo_hip_nb.so PU_AA_NB=2
done
