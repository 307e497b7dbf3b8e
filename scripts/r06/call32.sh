# r06 call 32: non-temporal stores in the pattern compression (PU_PAT_NT: 1 the pack's packed
# words, 2 the unpack's rows, 3 both) against the default: pattern GPU tests, bench lines
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call32; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_patterns.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR|Error" $O/pytest_gpu.log | head -30; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for v in 0 1 2 3; do
  PU_PAT_NT=$v timeout -k 10 300 python -u bench.py --workload patterns > $O/p_$v.json 2> $O/p_$v.err || { tail -20 $O/p_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/p_$v.json').read().strip().splitlines()[-1])
print('nt=$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
done
