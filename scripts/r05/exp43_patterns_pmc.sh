# r05 exp43: HBM bytes of one pattern compression -- FETCH_SIZE and WRITE_SIZE, each its own
# rocprofv3 --pmc pass over a short patterns bench
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp43
rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -- python bench.py --workload patterns --steps 3 --warmup 5 --no-cpu-baseline > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -- python bench.py --workload patterns --steps 3 --warmup 5 --no-cpu-baseline > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
echo ok
