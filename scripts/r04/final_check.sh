# r04 end: GPU tests, smoke and the default bench line on the library built from the
# committed source (after the late experiments were reverted)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_end.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_end.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_end.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_end.log
timeout -k 10 600 python bench.py > gpurun_out/bench_end.json 2> gpurun_out/bench_end.err || exit $?
tail -c 600 gpurun_out/bench_end.json
