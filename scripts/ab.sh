#!/bin/bash
# Same-box A/B timing: scripts/sweep.py alternately on libphylo_hip.so (A) and
# libphylo_hip_$B.so (B), ROUNDS times each.  CFG, SWEEP_ARGS select the workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=${B:-old}
for i in $(seq 1 ${ROUNDS:-3}); do
  timeout -k 10 120 python scripts/sweep.py --config ${CFG:-cfg2} --rounds 3 $SWEEP_ARGS 2>/dev/null | tail -1 | sed "s/^/A   /" || exit $?
  PHYLO_HIP_LIB=$PWD/phylo_utils_amd/libphylo_hip_$B.so timeout -k 10 120 python scripts/sweep.py --config ${CFG:-cfg2} --rounds 3 $SWEEP_ARGS 2>/dev/null | tail -1 | sed "s/^/B   /" || exit $?
done
