# r06 call 21: pattern compression with the one-workgroup tail (k_tail) after k_settle: pattern GPU
# tests (bit-exact against np.unique), the patterns bench line, A/B against PU_PAT_NO_TAIL,
# kernel stats
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call21; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_patterns.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR|Error" $O/pytest_gpu.log | head -30; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for v in 0 1; do
  if [ $v = 1 ]; then export PU_PAT_NO_TAIL=1; else unset PU_PAT_NO_TAIL; fi
  timeout -k 10 300 python -u bench.py --workload patterns > $O/bench_patterns_ns$v.json 2> $O/bench_patterns_ns$v.err || { tail -20 $O/bench_patterns_ns$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_patterns_ns$v.json').read().strip().splitlines()[-1])
print('no_tail=$v', d['value'], d['ms_per_step'], d.get('config',{}).get('rounds'))"
done
done
unset PU_PAT_NO_TAIL
