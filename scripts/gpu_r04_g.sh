# r04: register stash slots (TV_RSLOTS, libphylo_hip_rslots.so) -- GPU tests on that build,
# then same-box A/B on cfg4 (read-backs 11 -> 0) and cfg2 (unchanged plan)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PHYLO_HIP_LIB=$PWD/phylo_utils_amd/libphylo_hip_rslots.so timeout -k 10 600 python -u -m pytest \
  tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_rslots.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_rslots.log; [ $rc -ne 0 ] && exit $rc
B=rslots CFG=cfg4 ROUNDS=3 STEPS=60 bash scripts/ab_bench.sh || exit $?
B=rslots CFG=cfg2 ROUNDS=2 bash scripts/ab_bench.sh || exit $?
