# r04: GPU tests on the new planner + k_prune dispatch, then the occupancy sweep
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
export PU_DEBUG_PLAN=1
timeout -k 10 500 python -u scripts/sweep.py --config cfg4 --steps 40 --rounds 3 \
  --grid 'PU_KEEP_OCC=,3,4,5,6,7,8' > gpurun_out/r04_occ_cfg4.txt 2>&1 || exit $?
timeout -k 10 500 python -u scripts/sweep.py --config cfg2 --steps 100 --rounds 3 \
  --sites 50000,75000,90000,100000,115000,131072,150000,200000,300000 \
  --grid 'PU_KEEP_OCC=,4,5,6,7,8' > gpurun_out/r04_occ_cfg2.txt 2>&1 || exit $?
timeout -k 10 500 python -u scripts/sweep.py --config cfg4 --steps 40 --rounds 3 \
  --taxa 200,500 --sites 100000,125000 \
  --grid 'PU_KEEP_OCC=,4,5,6' > gpurun_out/r04_occ_taxa.txt 2>&1 || exit $?
grep -v "^\[pu plan\]" gpurun_out/r04_occ_cfg4.txt gpurun_out/r04_occ_cfg2.txt gpurun_out/r04_occ_taxa.txt
