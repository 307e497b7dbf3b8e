#!/bin/bash
# Same-box A/B of whole bench steps: bench.py alternately on libphylo_hip.so (A),
# libphylo_hip_$B.so (B) and, when AENV is set, A under that environment (A+env),
# ROUNDS times each.  CFG / BENCH_ARGS select the workload.  Prints ms_per_step,
# the traversal's event median and the value of every run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=${B:-old}
run() {  # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config ${CFG:-cfg3} --steps ${STEPS:-200} --warmup 20 \
      --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_line.json 2> gpurun_out/ab_err.txt
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -5 gpurun_out/ab_err.txt; exit $rc; fi
  python -c "
import json; d = json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1])
t = d.get('timing', {})
print('%-8s step %.5f ms  kernel %.5f ms  value %.1f  lnl %r' % ('$label', d['ms_per_step'],
      t.get('kernel_ms_median', float('nan')), d['value'], d.get('lnl')))"
}
for i in $(seq 1 ${ROUNDS:-3}); do
  run A PU_AB=A || exit $?
  if [ "$B" != none ]; then run B PHYLO_HIP_LIB=$PWD/phylo_utils_amd/libphylo_hip_$B.so || exit $?; fi
  if [ -n "$AENV" ]; then run A+env $AENV || exit $?; fi
done
