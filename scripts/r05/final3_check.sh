# r05 final, call 3 (after the batch's grid order): GPU suite, smoke, default bench lines of
# cfg2 and cfg5
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/final_r05
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/final_r05/pytest_gpu3.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/final_r05/pytest_gpu3.log | tail -2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_r05/smoke3.log 2>&1 || { cat gpurun_out/final_r05/smoke3.log; exit 1; }
tail -1 gpurun_out/final_r05/smoke3.log
timeout -k 10 600 python -u bench.py > gpurun_out/final_r05/bench_default.json 2> gpurun_out/final_r05/bench_default.err || { tail -20 gpurun_out/final_r05/bench_default.err; exit 1; }
tail -1 gpurun_out/final_r05/bench_default.json | cut -c1-400
timeout -k 10 600 python -u bench.py --config cfg5 > gpurun_out/final_r05/bench_cfg5.json 2> gpurun_out/final_r05/bench_cfg5.err || { tail -20 gpurun_out/final_r05/bench_cfg5.err; exit 1; }
tail -1 gpurun_out/final_r05/bench_cfg5.json | cut -c1-400
