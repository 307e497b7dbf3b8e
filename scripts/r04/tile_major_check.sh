# r04 late: the adopted tile-major DNA layout -- GPU tests, smoke, default bench line and the
# default-plan sweep (50 taxa) with its neighbour check
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/tmc
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/tmc/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/tmc/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/tmc/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/tmc/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/tmc/bench.json 2> gpurun_out/tmc/bench.err || exit $?
timeout -k 10 600 python -u scripts/sweep.py --config cfg2 \
  --sites 50000,62500,75000,87500,100000,112500,125000,131072,137500,150000,175000,200000,250000,300000 \
  --steps 100 --rounds 3 --json gpurun_out/tmc/sweep_sites.json > gpurun_out/tmc/sweep_sites.txt 2>&1 || exit $?
timeout -k 10 600 python -u scripts/sweep.py --config cfg2 --taxa 500,1000 --steps 30 --rounds 3 \
  --sites 100000,131072,200000 --json gpurun_out/tmc/sweep_taxa.json > gpurun_out/tmc/sweep_taxa.txt 2>&1 || exit $?
grep "neighbour" gpurun_out/tmc/sweep_sites.txt gpurun_out/tmc/sweep_taxa.txt
