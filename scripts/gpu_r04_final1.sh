# r04 final, call 1: GPU tests + smoke on the installed build, then per config the rocprofv3
# kernel trace, the PMC FETCH / WRITE passes and the instruction-mix pass (no bench lines:
# those are taken once these profiles are committed, so their roofline reads them)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
INSTS=1 BENCH=0 CONFIGS="cfg2 cfg3 cfg4 cfg5:--lnl-only:_lnl" bash scripts/gpu_profiles.sh
