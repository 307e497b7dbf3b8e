# r04 late: tile-major DNA rows (k_prune's row = tile * C + category, experiment build
# libphylo_hip_tm.so: `make -C phylo_utils_amd/csrc ab VARIANT=tm FLAGS=-DPU_TILE_MAJOR`;
# traversal-consistent only, so the getters are not used here) against the row layout
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/tm
export TMPDIR=/tmp
L=$PWD/phylo_utils_amd
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
      t.get('kernel_ms_median', float('nan')), d['value'], d.get('lnl')))" | tee -a gpurun_out/tm/ab.txt
}
CFG=cfg2
for i in 1 2 3; do run row PU_AB=A; run tm PHYLO_HIP_LIB=$L/libphylo_hip_tm.so; done
CFG=cfg4 STEPS=60
for i in 1 2; do run row PU_AB=A; run tm PHYLO_HIP_LIB=$L/libphylo_hip_tm.so; done
for v in row tm; do
  if [ $v = tm ]; then export PHYLO_HIP_LIB=$L/libphylo_hip_tm.so; fi
  timeout -k 10 300 python -u scripts/sweep.py --config cfg2 \
    --sites 50000,62500,75000,87500,100000,112500,125000,131072,137500,150000 --steps 100 --rounds 3 \
    --json gpurun_out/tm/sweep_$v.json > gpurun_out/tm/sweep_$v.txt 2>&1 || exit $?
  echo "sweep $v done"
done
