# r04: cfg4 shard plan sweep (split vs unsplit, stash slots, occupancy)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/sweep.py --config cfg4 --steps 40 --rounds 3 \
  --grid 'PU_SPLIT:PU_LDS_SLOTS:PU_WAVES:PU_LDS_PAD=::,0:3:1:,0:4:1:,0:5:1:,9:3:1:,9:3:1:3968,0:3:1:3968,0:2:1:' \
  > gpurun_out/r04_cfg4_sweep_a.txt 2>&1
rc=$?
cat gpurun_out/r04_cfg4_sweep_a.txt
exit $rc
