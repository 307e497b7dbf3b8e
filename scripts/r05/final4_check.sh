# r05 final, call 4 (after the pattern-compression rework): GPU suite, smoke, default bench
# line, the patterns bench line and its kernel trace
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/final_r05
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu4.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu4.log | tail -2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke4.log 2>&1 || { cat $O/smoke4.log; exit 1; }
tail -1 $O/smoke4.log
timeout -k 10 600 python -u bench.py > $O/bench_default4.json 2> $O/bench_default4.err || { tail -20 $O/bench_default4.err; exit 1; }
tail -1 $O/bench_default4.json | cut -c1-300
timeout -k 10 600 python -u bench.py --workload patterns > $O/bench_patterns4.json 2> $O/bench_patterns4.err || { tail -20 $O/bench_patterns4.err; exit 1; }
tail -1 $O/bench_patterns4.json | cut -c1-300
rm -rf $O/patterns_trace4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/patterns_trace4 -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $O/patterns_trace4.log 2>&1 || { tail -20 $O/patterns_trace4.log; exit 1; }
echo done
