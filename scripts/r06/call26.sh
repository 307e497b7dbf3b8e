# r06 call 26: the reference's brent / dbrent in one persistent launch (pu_minimise_edge):
# edge GPU tests (the host driver bit-equal to the Python restatement, the device driver to
# tolerance), the edges line with the minimisers block
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call26; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_edges_golden.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR|Error|assert" $O/pytest_gpu.log | head -40; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload edges > $O/bench_edges.json 2> $O/bench_edges.err || { tail -20 $O/bench_edges.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_edges.json').read().strip().splitlines()[-1])
print(json.dumps({k: d[k] for k in ('value','device_newton','minimisers','sweep')}))"
