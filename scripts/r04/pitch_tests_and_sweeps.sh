# r04: pitch = layout rows padded by one tile when the tile count is a multiple of 256
# (pu_internal.h tile_pitch): GPU tests on that build, then the power-of-two probe and the
# default-plan sweep on it
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PHYLO_HIP_LIB=$PWD/phylo_utils_amd/libphylo_hip_pitch.so
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_pitch.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_pitch.log; [ $rc -ne 0 ] && exit $rc
PU_DEBUG_PLAN=1 timeout -k 10 600 python -u scripts/sweep.py --config cfg2 --steps 100 --rounds 3 \
  --sites 65472,65536,65600,130944,131008,131072,131136,131200,262080,262144,262208 \
  --json gpurun_out/sweep_pow2_pitch.json > gpurun_out/sweep_pow2_pitch.txt 2>&1 || exit $?
grep -E "traverse" gpurun_out/sweep_pow2_pitch.txt
S=$(python -c "print(','.join(str(s) for s in sorted(set(list(range(50000, 300001, 12500)) + [131072]))))")
timeout -k 10 900 python -u scripts/sweep.py --config cfg2 --sites "$S" --steps 100 --rounds 3 \
  --json gpurun_out/sweep_cfg2_sites_pitch.json > gpurun_out/sweep_cfg2_sites_pitch.txt 2>&1 || exit $?
tail -8 gpurun_out/sweep_cfg2_sites_pitch.txt
timeout -k 10 900 python -u scripts/sweep.py --config cfg2 --taxa 500,1000 \
  --sites 50000,100000,131072,200000,300000 --steps 50 --rounds 3 \
  --json gpurun_out/sweep_cfg2_taxa_pitch.json > gpurun_out/sweep_cfg2_taxa_pitch.txt 2>&1 || exit $?
tail -6 gpurun_out/sweep_cfg2_taxa_pitch.txt
