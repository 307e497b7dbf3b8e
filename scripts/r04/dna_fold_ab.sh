# r04: DNA grid reduction folded into k_prune (no k_reduce launch) -- GPU tests, smoke, then
# an A/B against the k_reduce launch (PU_NO_FOLD=1) on cfg2, cfg4 and cfg5; lnL must match bitwise
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_fold.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_fold.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_fold.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_fold.log
run() {  # label, then env assignments; one bench line, summarised
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-200} --warmup 20 \
      --no-cpu-baseline > gpurun_out/ab_line.json 2> gpurun_out/ab_err.txt
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/ab_err.txt; exit $rc; fi
  python -c "
import json; d = json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1])
t = d.get('timing', {})
print('%-5s %-6s step %.5f ms  kernel %.5f ms  value %.1f  lnl %r' % ('$CFG', '$label', d['ms_per_step'],
      t.get('kernel_ms_median', float('nan')), d['value'], d.get('lnl')))" | tee -a gpurun_out/ab_fold.txt
}
CFG=cfg2
for i in 1 2 3; do run fold PU_AB=A; run reduce PU_NO_FOLD=1; done
CFG=cfg5 STEPS=20
for i in 1 2 3; do run fold PU_AB=A; run reduce PU_NO_FOLD=1; done
CFG=cfg4 STEPS=60
for i in 1 2; do run fold PU_AB=A; run reduce PU_NO_FOLD=1; done
