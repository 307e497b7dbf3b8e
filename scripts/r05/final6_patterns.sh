# r05 final, call 6: the pattern-compression line on the final code (16-word unpack slices):
# bench line, kernel trace, FETCH_SIZE / WRITE_SIZE passes
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/final_r05
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --workload patterns > $O/bench_patterns6.json 2> $O/bench_patterns6.err || { tail -20 $O/bench_patterns6.err; exit 1; }
tail -1 $O/bench_patterns6.json | cut -c1-200
rm -rf $O/patterns_trace6 $O/pfetch6 $O/pwrite6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/patterns_trace6 -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $O/patterns_trace6.log 2>&1 || { tail -20 $O/patterns_trace6.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pfetch6 -- python bench.py --workload patterns --steps 3 --warmup 5 --no-cpu-baseline > $O/pfetch6.log 2>&1 || { tail -20 $O/pfetch6.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pwrite6 -- python bench.py --workload patterns --steps 3 --warmup 5 --no-cpu-baseline > $O/pwrite6.log 2>&1 || { tail -20 $O/pwrite6.log; exit 1; }
echo done
