#!/bin/bash
# PMC passes of one sweep.py workload on the current library and on each
# phylo_utils_amd/libphylo_hip_<name>.so of LIBS: one rocprofv3 --pmc run per counter set.
#   PMC_SETS="A B C|D E"  CFG=cfg5  SWEEP_ARGS=--lnl-only  LIBS="old"  KERNEL=k_prune
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcab
export TMPDIR=/tmp
IFS='|' read -ra SETS <<< "$PMC_SETS"
for lib in cur $LIBS; do
  if [ "$lib" = cur ]; then unset PHYLO_HIP_LIB; else export PHYLO_HIP_LIB=$PWD/phylo_utils_amd/libphylo_hip_$lib.so; fi
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    d=gpurun_out/pmcab/${lib}_set$i
    rm -rf $d
    timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d $d \
        -- python scripts/sweep.py --config ${CFG:-cfg2} --rounds 1 --steps 20 --warm-seconds 0.5 $SWEEP_ARGS > $d.log 2>&1
    rc=$?
    echo "[pmc_ab] $lib set$i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
    python scripts/pmc_summary.py $d ${KERNEL:-k_prune}
  done
done
