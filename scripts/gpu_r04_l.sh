# r04 final build (row-pair protein stores + padded layout pitch): GPU tests + smoke, the cfg3
# profile (its kernel changed), the profiles collected on the box so the bench lines read
# them, then the cfg3 and default (cfg2) bench lines
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/final_profiles
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_final.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_final.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_final.log
CFG=cfg3 RUN_TESTS=0 PROFILE=1 INSTS=1 BENCH=0 bash scripts/gpu_round.sh || exit $?
python scripts/collect_profiles.py --round r04 --config cfg3 --src gpurun_out/prof_cfg3 || exit $?
cp profiles/r04_cfg3_kernel_stats.csv profiles/r04_traffic_cfg3.json profiles/r04_pmc_cfg3.json \
   gpurun_out/final_profiles/
timeout -k 10 600 python bench.py --config cfg3 > gpurun_out/bench_cfg3_final.json 2> gpurun_out/bench_cfg3_final.err || exit $?
tail -c 300 gpurun_out/bench_cfg3_final.json
timeout -k 10 600 python bench.py > gpurun_out/bench_cfg2_final.json 2> gpurun_out/bench_cfg2_final.err || exit $?
tail -c 300 gpurun_out/bench_cfg2_final.json
