#!/bin/bash
# Same-box A/B/C... timing: scripts/sweep.py alternately on libphylo_hip.so (A) and each
# phylo_utils_amd/libphylo_hip_<name>.so of LIBS="name1 name2", ROUNDS times each.
# CFG, SWEEP_ARGS select the workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  out=$(timeout -k 10 150 python scripts/sweep.py --config ${CFG:-cfg2} --rounds 3 $SWEEP_ARGS 2>/dev/null)
  rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "A rc=$rc"; exit $rc; }
  echo "$out" | tail -1 | sed "s/^/A       /"
  for b in $LIBS; do
    out=$(PHYLO_HIP_LIB=$PWD/phylo_utils_amd/libphylo_hip_$b.so timeout -k 10 150 python scripts/sweep.py --config ${CFG:-cfg2} --rounds 3 $SWEEP_ARGS 2>/dev/null)
    rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "$b rc=$rc"; exit $rc; }
    echo "$out" | tail -1 | sed "s/^/$b   /"
  done
done
