# r06 call 16: device Newton with per-site weights and pattern weights in LDS (no exp, no global
# read per evaluation), state in LDS, one xor tree per sum; +I test case
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call16; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_edges_golden.py tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR|Error" $O/pytest_gpu.log | head -30; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/r06/newton_probe.py > $O/newton_probe.log 2>&1 || { tail -30 $O/newton_probe.log; exit 1; }
grep -v amdgpu.ids $O/newton_probe.log
timeout -k 10 300 python -u bench.py --workload edges > $O/bench_edges.json 2> $O/bench_edges.err || { tail -20 $O/bench_edges.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_edges.json').read().strip().splitlines()[-1])
print(json.dumps({k: d[k] for k in ('value','ms_per_step','device_newton','single_call','sweep')}))"
