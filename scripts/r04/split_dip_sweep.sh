# r04: do chain tasks (PU_SPLIT=n, a finer work granule than one tile's whole tree) lift the
# sizes the default-plan sweep flags (a partly empty last round of workgroups)?  cfg2, 50 taxa
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/sweep.py --config cfg2 --grid 'PU_SPLIT=,2,3,4,6' \
  --sites 50000,62500,75000,87500,100000,112500,125000,137500,150000 --steps 100 --rounds 3 \
  --json gpurun_out/split_dip.json > gpurun_out/split_dip.txt 2>&1
