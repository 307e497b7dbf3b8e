# r06 call 42: the engine-mode parity tests with the ambiguity-coded DNA case added (the tip
# products of all 16 codes from the per-row P kernel), plus the batch and parity files
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call42; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR" $O/pytest_gpu.log | head -20; tail -2 $O/pytest_gpu.log; exit $rc
