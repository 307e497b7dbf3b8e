# r06 call 8: the protein tip-code look-ahead: parity suite, then the cfg3 A/B against the
# build without it (libphylo_hip_old.so, -DPU_AB_NO_CODE_AHEAD)
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call8; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges_golden.py tests/test_kernel_isa.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR" $O/pytest_gpu.log | head -20; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
TAG=cfg3_code_ahead LIBS="new old" ROUNDS=3 bash scripts/r06/ab_libs.sh
