#!/bin/bash
# GPU tests only (optionally a subset: TESTS="tests/test_gpu_edges.py").  Time-limited; a
# crash / abort / timeout stops the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "[gpu_tests] pytest rc=$rc"
tail -25 gpurun_out/pytest_gpu.log
exit $rc
