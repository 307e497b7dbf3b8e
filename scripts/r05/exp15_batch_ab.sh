# r05 exp15: batched launch order / waves / stash slots (scripts/r05/batch_probe.py)
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp15
mkdir -p $O
for v in "PU_BATCH_ORDER=tree" "PU_BATCH_ORDER=tile" "PU_BATCH_WAVES=7" "PU_BATCH_ORDER=tile PU_BATCH_WAVES=7" "PU_LDS_SLOTS=1 PU_BATCH_WAVES=7" "PU_LDS_SLOTS=1 PU_BATCH_ORDER=tile PU_BATCH_WAVES=7" "PU_LDS_SLOTS=3"; do
  echo "== $v"
  env $v PU_DEBUG_PLAN=1 timeout -k 10 300 python -u scripts/r05/batch_probe.py --trees 1,32 > $O/p.txt 2>&1 || { tail -20 $O/p.txt; exit 1; }
  grep -E "batch|own launch" $O/p.txt | grep -v "^\[pu plan\]" | head -8
done
