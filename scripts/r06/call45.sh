# r06 call 45: batch groups of 56 as the default -- the batch and parity GPU tests, then cfg5's
# trace, PMC passes and bench line (scripts/gpu_profiles.sh)
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call45; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR" $O/pytest_gpu.log | head -20; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
CONFIGS="cfg5::_batch" BENCH_STEPS=200 INSTS=1 bash scripts/gpu_profiles.sh > $O/profiles.log 2>&1 || { tail -30 $O/profiles.log; exit 1; }
grep -E "^== |rc=" $O/profiles.log
