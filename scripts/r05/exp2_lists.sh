# r05 exp2: worker lists (TV_LIST).  Parity tests first (a fault or hang ends the call), then
# the timeline of the stamps build, a same-box sweep r04 library vs this one, a bench line
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "worker_lists or keep_occupancy or register_stash or kernel_builds_and_plans" > $O/pytest_lists.log 2>&1 || { tail -30 $O/pytest_lists.log; exit 1; }
tail -3 $O/pytest_lists.log
PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_stamps.so timeout -k 10 200 python -u scripts/wg_timeline.py --sites 100000 --taxa 50 --launches 2 --out $O/tl > $O/tl.log 2>&1 || exit 1
grep -A4 "launch 1" $O/tl.log; grep "end perc\|hand-off\|total bytes" $O/tl.log
for r in 1 2; do
for lib in libphylo_hip_r04.so libphylo_hip.so; do
  PHYLO_HIP_LIB=phylo_utils_amd/$lib timeout -k 10 300 python -u scripts/sweep.py --config cfg2 --sites 62500,87500,100000,112500,131072,150000 --steps 200 --rounds 3 --json $O/sweep_${lib}_$r.json > $O/sweep_${lib}_$r.txt 2>&1 || exit 1
done
done
grep traverse $O/sweep_*.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit 1
tail -c 600 $O/bench_cfg2.json
