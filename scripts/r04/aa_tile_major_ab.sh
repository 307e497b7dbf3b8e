# r04 late: tile-major protein rows too (experiment build libphylo_hip_aatm.so:
# `make -C phylo_utils_amd/csrc ab VARIANT=aatm FLAGS=-DPU_AA_TILE_MAJOR`) against
# category-major protein rows: protein GPU tests on the experiment library, then cfg3 A/B
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/aatm
export TMPDIR=/tmp
L=$PWD/phylo_utils_amd
PHYLO_HIP_LIB=$L/libphylo_hip_aatm.so timeout -k 10 600 python -u -m pytest tests -m gpu -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "protein or aa or K20 or cfg3 or lg or wag" \
  > gpurun_out/aatm/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/aatm/pytest.log; [ $rc -ne 0 ] && exit $rc
run() {  # label, then env assignments; one bench line, summarised
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-200} --warmup 20 \
      --no-cpu-baseline > gpurun_out/ab_line.json 2> gpurun_out/ab_err.txt
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/ab_err.txt; exit $rc; fi
  python -c "
import json; d = json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1])
t = d.get('timing', {})
print('%-5s %-4s step %.5f ms  kernel %.5f ms  value %.1f  lnl %r' % ('$CFG', '$label', d['ms_per_step'],
      t.get('kernel_ms_median', float('nan')), d['value'], d.get('lnl')))" | tee -a gpurun_out/aatm/ab.txt
}
CFG=cfg3
for i in 1 2 3 4; do run row PU_AB=A; run tm PHYLO_HIP_LIB=$L/libphylo_hip_aatm.so; done
