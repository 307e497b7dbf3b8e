# r05 final, call 2: cfg4, cfg5 (lnL only, per-tree launches over 4 streams) and the N2 / N1
# secondary lines, then the strong-scaling shard sizes of the 1M-site cfg4 alignment
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/final_r05
export TMPDIR=/tmp
CONFIGS="cfg4 cfg5:--lnl-only:_lnl" BENCH_STEPS=100 INSTS=1 bash scripts/gpu_profiles.sh > gpurun_out/final_r05/profiles2.log 2>&1 || { tail -30 gpurun_out/final_r05/profiles2.log; exit 1; }
grep -E "^== |rc=" gpurun_out/final_r05/profiles2.log
timeout -k 10 300 python -u bench.py --workload patterns > gpurun_out/final_r05/bench_patterns.json 2> gpurun_out/final_r05/bench_patterns.err || { tail -20 gpurun_out/final_r05/bench_patterns.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload edges > gpurun_out/final_r05/bench_edges.json 2> gpurun_out/final_r05/bench_edges.err || { tail -20 gpurun_out/final_r05/bench_edges.err; exit 1; }
export PU_BENCH_CACHE=/tmp/pu_bench_sim
timeout -k 10 300 python -u scripts/presim.py --config cfg4 --total-sites 1000000 --workers 8 > gpurun_out/final_r05/presim.log 2>&1 || { tail -20 gpurun_out/final_r05/presim.log; exit 1; }
for T in 1000000 500000 250000; do
  CFG=cfg4 BENCH_ARGS="--total-sites $T" TAGSUFFIX="_s$T" RUN_TESTS=0 PROFILE=1 BENCH=1 BENCH_STEPS=20 \
      bash scripts/gpu_round.sh > gpurun_out/final_r05/strong_$T.log 2>&1 || { tail -20 gpurun_out/final_r05/strong_$T.log; exit 1; }
  grep -E "rc=" gpurun_out/final_r05/strong_$T.log
done
