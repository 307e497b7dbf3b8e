# r06 call 31: k_unpack_lds with the next slice's words in registers while the rows go out (PF)
# against loads after each barrier (PU_UNPACK_PF=0): pattern GPU tests, bench lines
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call31; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_patterns.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR|Error" $O/pytest_gpu.log | head -30; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for v in 1 0; do
  PU_UNPACK_PF=$v timeout -k 10 300 python -u bench.py --workload patterns > $O/p_$v.json 2> $O/p_$v.err || { tail -20 $O/p_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/p_$v.json').read().strip().splitlines()[-1])
print('upf=$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
done
rm -rf $O/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
