#!/bin/bash
# PMC passes over one kernel variant (sweep.py with a single setting).  Usage:
#   PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES ...|TCC_HIT_sum TCC_MISS_sum" bash scripts/pmc.sh <sweep args>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/${PMC_DIR:-pmc}
mkdir -p $D
export TMPDIR=/tmp
i=0
IFS='|' read -ra SETS <<< "$PMC_SETS"
for set in "${SETS[@]}"; do
  i=$((i+1))
  rm -rf $D/set$i
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $D/set$i \
      -- python scripts/sweep.py --rounds 1 --steps 20 --warm-seconds 0.5 "$@" > $D/set$i.log 2>&1
  rc=$?
  echo "[pmc] set$i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $D/set$i.log; exit $rc; fi
done
