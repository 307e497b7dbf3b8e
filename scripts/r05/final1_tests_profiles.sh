# r05 final, call 1: the GPU suite and smoke on the shipped library, then kernel trace + PMC
# traffic + bench line for cfg2 and cfg3 (scripts/gpu_profiles.sh); a failure or timeout ends
# the call
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/final_r05
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/final_r05/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/final_r05/pytest_gpu.log | tail -2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_r05/smoke.log 2>&1 || { cat gpurun_out/final_r05/smoke.log; exit 1; }
cat gpurun_out/final_r05/smoke.log
CONFIGS="cfg2 cfg3" BENCH_STEPS=200 bash scripts/gpu_profiles.sh > gpurun_out/final_r05/profiles1.log 2>&1 || { tail -30 gpurun_out/final_r05/profiles1.log; exit 1; }
grep -E "^== |rc=" gpurun_out/final_r05/profiles1.log
