# r06 call 23: pattern compression with its flags and counts in mapped host memory (no copy
# launches), k_tail's word scan in 8-word steps: pattern GPU tests, three bench lines, a trace
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call23; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_patterns.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR|Error" $O/pytest_gpu.log | head -30; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload patterns > $O/bench_patterns_$r.json 2> $O/bench_patterns_$r.err || { tail -20 $O/bench_patterns_$r.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_patterns_$r.json').read().strip().splitlines()[-1])
print('patterns', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
rm -rf $O/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
