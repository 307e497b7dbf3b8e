# r05 exp19: the GPU suite on the per-side protein P kernel, then the cfg3 profile (kernel
# trace, traffic, bench) and the 1M-site strong-scaling shard profile
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu_r05.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_r05.log; [ $rc -ne 0 ] && exit $rc
CONFIGS="cfg3" BENCH_STEPS=200 bash scripts/gpu_profiles.sh || exit 1
export PU_BENCH_CACHE=/tmp/pu_bench_sim
timeout -k 10 300 python -u scripts/presim.py --config cfg4 --total-sites 1000000 --workers 8 || exit 1
CFG=cfg4 BENCH_ARGS="--total-sites 1000000" TAGSUFFIX="_s1000000" RUN_TESTS=0 PROFILE=1 BENCH=1 BENCH_STEPS=20 \
    bash scripts/gpu_round.sh
