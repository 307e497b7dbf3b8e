# r06 call 5: kernel traces + PMC byte passes + bench lines for cfg2, cfg3 and cfg5 (batch) on
# the r06 build (scripts/gpu_profiles.sh; scripts/collect_profiles.py --round r06 afterwards)
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call5; mkdir -p $O
export TMPDIR=/tmp
CONFIGS="cfg2 cfg3 cfg5::_batch" BENCH_STEPS=200 INSTS=1 bash scripts/gpu_profiles.sh > $O/profiles.log 2>&1 || { tail -30 $O/profiles.log; exit 1; }
grep -E "^== |rc=" $O/profiles.log
for t in cfg2 cfg3 cfg5_batch; do
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_$t.json').read().splitlines() if l.startswith('{')][-1]); r=d['roofline']
print('$t', d['value'], d['ms_per_step'], r.get('frac'), r.get('kernel_ms'), r.get('ceiling_GBps'), r.get('frac_of_ceiling'), d.get('lnl_rel_err_vs_cpu'))"
done
