cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/dbg
PU_DEBUG_PLAN=1 PU_DEBUG_PTRS=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 60 --timeout-method thread -p no:cacheprovider -k "test_worker_lists_bitwise and 50-100000-4-env0" > gpurun_out/dbg/dbg.log 2>&1
grep -E "pu plan|pu ptrs\] K|FAIL|passed|failed|Error" gpurun_out/dbg/dbg.log | head -20
