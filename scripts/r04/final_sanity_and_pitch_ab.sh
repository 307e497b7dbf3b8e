# r04 final sanity on the library built by __graft_entry__.build() from the committed source:
# GPU tests, smoke, the default bench line
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_n.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_n.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_n.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_n.log
timeout -k 10 600 python bench.py > gpurun_out/bench_n.json 2> gpurun_out/bench_n.err || exit $?
tail -c 400 gpurun_out/bench_n.json
# A/B: extra unused tiles per layout row (-DPU_PITCH_EXTRA=e builds) on cfg2 and cfg4
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
      t.get('kernel_ms_median', float('nan')), d['value'], d.get('lnl')))" | tee -a gpurun_out/ab_pitch.txt
}
CFG=cfg2
for i in 1 2 3; do
  run A PU_AB=A
  for e in 1 3 8; do run p$e PHYLO_HIP_LIB=$L/libphylo_hip_p$e.so; done
done
CFG=cfg4 STEPS=60
for i in 1 2; do
  run A PU_AB=A
  for e in 1 3; do run p$e PHYLO_HIP_LIB=$L/libphylo_hip_p$e.so; done
done
