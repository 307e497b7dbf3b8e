# r06 call 2: protein parity on the ballot / descriptor-prefetch build, then the cfg3 A/B
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
TAG=cfg3_ballot LIBS="new old nob nod" ROUNDS=3 bash scripts/r06/ab_libs.sh
