# r04 final sanity on the library built by __graft_entry__.build() from the committed source:
# GPU tests, smoke, the default bench line
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_n.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_n.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_n.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_n.log
timeout -k 10 600 python bench.py > gpurun_out/bench_n.json 2> gpurun_out/bench_n.err || exit $?
tail -c 400 gpurun_out/bench_n.json
