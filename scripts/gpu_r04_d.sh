# r04: pair kernel parity + cfg5, then the occupancy data the planner is fitted to:
# split vs occupancy plans for cfg4 on one box, and a dense 50 / 100-taxon size sweep
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_r04_c.sh || exit $?
timeout -k 10 400 python -u scripts/sweep.py --config cfg4 --steps 30 --rounds 3 \
  --grid 'PU_KEEP_OCC:PU_SPLIT:PU_LDS_SLOTS=:,4::,:9:2,:9:3' > gpurun_out/r04_cfg4_split_vs_occ.txt 2>&1 || exit $?
grep -v "^\[pu plan\]" gpurun_out/r04_cfg4_split_vs_occ.txt
timeout -k 10 500 python -u scripts/sweep.py --config cfg2 --steps 60 --rounds 2 \
  --sites 40000,57344,65536,73728,81920,98304,106496,122880,139264,163840,180224,196608,229376,262144 \
  --grid 'PU_KEEP_OCC=4,5,6,7,8' > gpurun_out/r04_occ_dense50.txt 2>&1 || exit $?
timeout -k 10 500 python -u scripts/sweep.py --config cfg2 --steps 40 --rounds 2 --taxa 100 \
  --sites 50000,75000,90000,100000,131072,200000 \
  --grid 'PU_KEEP_OCC=4,5,6,7,8' > gpurun_out/r04_occ_dense100.txt 2>&1 || exit $?
grep -v "^\[pu plan\]\|amdgpu.ids" gpurun_out/r04_occ_dense50.txt gpurun_out/r04_occ_dense100.txt | head -150
