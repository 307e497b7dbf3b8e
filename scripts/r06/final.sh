# r06 final evidence, one call: GPU suite, smoke, then per config a kernel trace + PMC passes +
# bench line (scripts/gpu_profiles.sh), the edges and patterns lines
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR" $O/pytest_gpu.log | head -20; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
CONFIGS="${CONFIGS:-cfg2 cfg3 cfg5::_batch}" BENCH_STEPS=200 INSTS=1 bash scripts/gpu_profiles.sh > $O/profiles.log 2>&1 || { tail -30 $O/profiles.log; exit 1; }
grep -E "^== |rc=" $O/profiles.log
for w in edges patterns; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
done
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); r=d['roofline']
print('default', d['value'], d['ms_per_step'], r['frac'], r.get('frac_of_ceiling'), d.get('lnl_rel_err_vs_cpu'))"
