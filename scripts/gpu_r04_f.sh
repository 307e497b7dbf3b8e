# r04: GPU tests on the current build, the layout probe (write_pattern10) for the cfg2 and cfg4
# shapes, and the PU_PA_EARLY A/B (libphylo_hip_paearly.so) on cfg5 and cfg2
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 scripts/probes/_write_pattern10 49 1563 4 > gpurun_out/r04_wp10_cfg2.txt 2>&1 || exit $?
timeout -k 10 300 scripts/probes/_write_pattern10 999 1954 4 > gpurun_out/r04_wp10_cfg4.txt 2>&1 || exit $?
cat gpurun_out/r04_wp10_cfg2.txt gpurun_out/r04_wp10_cfg4.txt
B=paearly CFG=cfg5 ROUNDS=2 STEPS=100 bash scripts/ab_bench.sh || exit $?
B=paearly CFG=cfg2 ROUNDS=3 bash scripts/ab_bench.sh || exit $?
