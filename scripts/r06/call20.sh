# r06 call 20: pattern compression after k_settle: kernel trace (csv) and the FETCH / WRITE passes
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call20; mkdir -p $O
export TMPDIR=/tmp
rm -rf $O/trace $O/pfetch $O/pwrite
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pfetch -- python bench.py --workload patterns --steps 3 --warmup 5 --no-cpu-baseline > $O/pfetch.log 2>&1 || { tail -20 $O/pfetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pwrite -- python bench.py --workload patterns --steps 3 --warmup 5 --no-cpu-baseline > $O/pwrite.log 2>&1 || { tail -20 $O/pwrite.log; exit 1; }
python scripts/r05/patterns_traffic.py $O/pfetch $O/pwrite $O/traffic.json && cat $O/traffic.json
