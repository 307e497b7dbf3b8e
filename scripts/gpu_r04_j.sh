# r04: the 131072-site dip of the sweep -- power-of-two tile counts against their neighbours
# (one tile fewer / more), with the plan printed (PU_DEBUG_PLAN), 50 taxa
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PU_DEBUG_PLAN=1 timeout -k 10 600 python -u scripts/sweep.py --config cfg2 --steps 100 --rounds 3 \
  --sites 65472,65536,65600,130944,131008,131072,131136,131200,262080,262144,262208 \
  --json gpurun_out/sweep_pow2.json > gpurun_out/sweep_pow2.txt 2>&1 || exit $?
grep -E "traverse|pu plan" gpurun_out/sweep_pow2.txt | sort -u | head -40
