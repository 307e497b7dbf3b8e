# r04: the secondary-path bench lines on the final library (N1 edge evaluations, N2 pattern
# compression)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --workload edges > gpurun_out/bench_edges.json 2> gpurun_out/bench_edges.err || exit $?
tail -c 600 gpurun_out/bench_edges.json
timeout -k 10 600 python bench.py --workload patterns > gpurun_out/bench_patterns.json 2> gpurun_out/bench_patterns.err || exit $?
tail -c 600 gpurun_out/bench_patterns.json
