# r04 final, call 3: bench lines on the committed r04 profiles -- the four configs, then the
# strong-scaling runs of one 1M-site alignment at the N = 1, 2, 4 and 8 per-rank sizes
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PU_BENCH_CACHE=/tmp/pu_bench_sim
b() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
  local rc=$?; echo "[final3] $tag rc=$rc"; tail -c 400 gpurun_out/bench_$tag.json; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
b cfg2 --config cfg2
b cfg3 --config cfg3
b cfg4 --config cfg4 --steps 60
b cfg5_lnl --config cfg5 --lnl-only
timeout -k 10 300 python -u scripts/presim.py --config cfg4 --total-sites 1000000 --workers 8 || exit $?
for T in 1000000 500000 250000 125000; do
  b cfg4_strong_s$T --config cfg4 --total-sites $T --steps 30
done
