# r06 call 22: pattern compression without the U / bad-code round trips (unpack grid over S,
# U from the device); k_pack A/B: 128 threads x 4 columns (default) vs 256 x 2 vs 512 x 1
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call22; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_patterns.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR|Error" $O/pytest_gpu.log | head -30; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for v in 4 2 1; do
  PU_PACK_V=$v timeout -k 10 300 python -u bench.py --workload patterns > $O/bench_patterns_v$v.json 2> $O/bench_patterns_v$v.err || { tail -20 $O/bench_patterns_v$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_patterns_v$v.json').read().strip().splitlines()[-1])
print('pack V=$v', d['value'], d['ms_per_step'])"
done
done
