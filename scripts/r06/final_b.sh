# r06 final evidence, call B: per config a kernel trace + PMC passes + bench line
# (scripts/gpu_profiles.sh) for cfg2, cfg3 and batched cfg5, then the default bench line
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_final; mkdir -p $O
export TMPDIR=/tmp
CONFIGS="${CONFIGS:-cfg2 cfg3 cfg5::_batch}" BENCH_STEPS=200 INSTS=1 bash scripts/gpu_profiles.sh > $O/profiles.log 2>&1 || { tail -30 $O/profiles.log; exit 1; }
grep -E "^== |rc=" $O/profiles.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); r=d['roofline']
print('default', d['value'], d['ms_per_step'], r['frac'], r.get('frac_of_ceiling'), d.get('lnl_rel_err_vs_cpu'))"
