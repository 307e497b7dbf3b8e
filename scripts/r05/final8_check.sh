# r05 final, call 8 (after the protein chunk-rule fix): GPU suite,
# smoke, default bench line, cfg5 and cfg3 bench lines
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/final_r05
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu8.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu8.log | tail -2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke8.log 2>&1 || { cat $O/smoke8.log; exit 1; }
tail -1 $O/smoke8.log
for c in default cfg5 cfg3; do
  a=""; [ $c != default ] && a="--config $c"
  timeout -k 10 600 python -u bench.py $a > $O/bench_${c}8.json 2> $O/bench_${c}8.err || { tail -20 $O/bench_${c}8.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/bench_${c}8.json').read().splitlines() if l.startswith('{')][-1])
print('$c', 'value %.1f' % d['value'], 'step %.4f ms' % d['ms_per_step'], 'frac', d['roofline']['frac'])"
done
