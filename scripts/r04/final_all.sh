# r04 final evidence in one call on the installed library: GPU tests + smoke; kernel traces and
# PMC passes for cfg2 / cfg3 / cfg4 / cfg5 lnL-only and the strong-scaling shards; the profiles
# collected on the box (so the bench lines read them) and copied to gpurun_out/final_profiles;
# then the bench lines
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/final_profiles
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_final.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_final.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_final.log
rm -rf gpurun_out/prof_*
INSTS=1 BENCH=0 CONFIGS="cfg2 cfg3 cfg4 cfg5:--lnl-only:_lnl" bash scripts/gpu_profiles.sh || exit $?
export PU_BENCH_CACHE=/tmp/pu_bench_sim
timeout -k 10 300 python -u scripts/presim.py --config cfg4 --total-sites 1000000 --workers 8 > /dev/null || exit $?
for T in 1000000 500000 250000; do
  CFG=cfg4 BENCH_ARGS="--total-sites $T" TAGSUFFIX="_s$T" RUN_TESTS=0 PROFILE=1 BENCH=0 \
      bash scripts/gpu_round.sh > /dev/null || exit $?
done
for c in cfg2 cfg3 cfg4; do
  python scripts/collect_profiles.py --round r04 --config $c --src gpurun_out/prof_$c > /dev/null || exit $?
done
python scripts/collect_profiles.py --round r04 --config cfg5 --suffix _lnl --src gpurun_out/prof_cfg5_lnl > /dev/null || exit $?
for T in 1000000 500000 250000; do
  python scripts/collect_profiles.py --round r04 --config cfg4 --suffix _s$T --src gpurun_out/prof_cfg4_s$T > /dev/null || exit $?
done
cp profiles/r04_*kernel_stats.csv profiles/r04_traffic_*.json profiles/r04_pmc_cfg2.json \
   profiles/r04_pmc_cfg3.json profiles/r04_pmc_cfg4.json profiles/r04_pmc_cfg5_lnl.json gpurun_out/final_profiles/
b() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
  local rc=$?; echo "[final] $tag rc=$rc $(tail -c 200 gpurun_out/bench_$tag.json | tr -d '\n' | cut -c1-120)"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
b cfg2
b cfg3 --config cfg3
b cfg4 --config cfg4 --steps 60
b cfg5_lnl --config cfg5 --lnl-only
for T in 1000000 500000 250000 125000; do
  b cfg4_strong_s$T --config cfg4 --total-sites $T --steps 30 --no-cpu-baseline
done
