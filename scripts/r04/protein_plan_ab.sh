# r04: protein plan knobs on the final build -- stash slots (LDS per workgroup: 3 slots = 3
# workgroups per CU, 2 slots = 4) and the split target, cfg3, three alternating rounds
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # label, then env assignments; one bench line, summarised
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config cfg3 --steps 200 --warmup 20 \
      --no-cpu-baseline > gpurun_out/ab_line.json 2> gpurun_out/ab_err.txt
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/ab_err.txt; exit $rc; fi
  python -c "
import json; d = json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1])
t = d.get('timing', {})
print('cfg3 %-10s step %.5f ms  kernel %.5f ms  value %.1f  lnl %r' % ('$label', d['ms_per_step'],
      t.get('kernel_ms_median', float('nan')), d['value'], d.get('lnl')))" | tee -a gpurun_out/ab_protein_plan.txt
}
for i in 1 2 3; do
  run default PU_AB=A
  run slots2 PU_LDS_SLOTS=2
  run slots1 PU_LDS_SLOTS=1
  run split4 PU_SPLIT=4
  run split5 PU_SPLIT=5
  run s2sp4 PU_LDS_SLOTS=2 PU_SPLIT=4
done
