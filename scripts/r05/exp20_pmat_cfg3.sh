# r05 exp20: the per-side protein P kernel with seven chains per thread -- protein GPU tests,
# then the cfg3 profile (kernel trace, traffic, bench)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "protein or cfg3 or pmat or all_partials or P_" > gpurun_out/pytest_protein.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_protein.log; [ $rc -ne 0 ] && exit $rc
CONFIGS="cfg3" BENCH_STEPS=200 bash scripts/gpu_profiles.sh
