#!/bin/bash
# r06: same-box A/B of kernel builds: bench.py --config $CFG alternately on each LIBS entry
# (libphylo_hip_<name>.so; "new" = libphylo_hip.so), ROUNDS rounds.  Prints ms_per_step, the
# traversal's event median and lnL of every run (-> gpurun_out/r06_ab/<tag>.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_ab; mkdir -p $O
TAG=${TAG:-ab}
for i in $(seq 1 ${ROUNDS:-3}); do
  for n in ${LIBS:-new old}; do
    lib=$PWD/phylo_utils_amd/libphylo_hip.so
    [ "$n" != new ] && lib=$PWD/phylo_utils_amd/libphylo_hip_$n.so
    PHYLO_HIP_LIB=$lib timeout -k 10 300 python bench.py --config ${CFG:-cfg3} --steps ${STEPS:-200} \
        --warmup 20 --no-cpu-baseline $BENCH_ARGS > $O/line.json 2> $O/err.txt
    rc=$?
    if [ $rc -ne 0 ]; then echo "$n rc=$rc"; tail -5 $O/err.txt; exit $rc; fi
    python -c "
import json; d = json.loads(open('$O/line.json').read().strip().splitlines()[-1])
t = d.get('timing', {}); r = d.get('roofline', {})
print('%-6s %-5s step %.5f ms  kernel %.5f ms  value %.1f  lnl %r' % ('$n', '${CFG:-cfg3}', d['ms_per_step'],
      t.get('kernel_ms_median', r.get('kernel_ms', float('nan'))), d['value'], d.get('lnl')))" | tee -a $O/$TAG.txt
  done
done
