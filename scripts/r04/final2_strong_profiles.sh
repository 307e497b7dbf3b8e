# r04 final, call 2: strong-scaling shards of one 1M-site cfg4 alignment (bench.py
# --total-sites 1000000 at the N = 1, 2, 4 per-rank sizes; N = 8's 125k shard is cfg4 itself):
# kernel trace + PMC traffic per size, keyed cfg4_s<sites> (bench.pmc_tag)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu2.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu2.log; [ $rc -ne 0 ] && exit $rc
set -e
export PU_BENCH_CACHE=/tmp/pu_bench_sim
timeout -k 10 300 python -u scripts/presim.py --config cfg4 --total-sites 1000000 --workers 8
for T in ${SIZES:-1000000 500000 250000}; do
  echo "== strong $T"
  CFG=cfg4 BENCH_ARGS="--total-sites $T" TAGSUFFIX="_s$T" RUN_TESTS=0 PROFILE=1 BENCH=0 \
      bash scripts/gpu_round.sh
done
set +e
bash scripts/r04/protein_diagnostics.sh
