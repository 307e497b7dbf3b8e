# r04: does the layout row pitch (tiles per (slot, category) row) explain the sizes the
# default-plan sweep flags?  PU_PITCH_EXTRA=e (experiment build) adds e unused tiles per row;
# one process per e (the pitch is read once per process).  cfg2, 50 taxa
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/pitch_probe
export TMPDIR=/tmp
for e in 0 1 2 3 4 5 6 7 8 12 16; do
  PU_PITCH_EXTRA=$e timeout -k 10 300 python -u scripts/sweep.py --config cfg2 \
    --sites 50000,62500,75000,87500,100000,112500,125000,137500 --steps 100 --rounds 3 \
    --json gpurun_out/pitch_probe/e$e.json > gpurun_out/pitch_probe/e$e.txt 2>&1 || exit $?
  echo "e=$e done"
done
