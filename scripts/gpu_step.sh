#!/bin/bash
# One gpurun call of the build -> measure loop: optional GPU tests, then sweep.py runs.
#   TESTS="tests/test_gpu_tiles.py ..."   pytest files (-m gpu), skipped when empty
#   SWEEPS="cfg2|--grid PU_TILES=1,2#cfg5|--lnl-only --grid ..."   '#'-separated runs
# Every GPU step has its own time limit; a crash, abort or time-out ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on() {  # rc name
  local rc=$1 name=$2
  echo "[gpu_step] $name rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[gpu_step] stopping after $name"; exit "$rc"; fi
}
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_step.log 2>&1
  rc=$?
  tail -15 gpurun_out/pytest_step.log
  stop_on $rc pytest
fi
i=0
IFS='#' read -ra RUNS <<< "$SWEEPS"
for run in "${RUNS[@]}"; do
  [ -z "$run" ] && continue
  i=$((i+1))
  cfg=${run%%|*}
  args=${run#*|}
  timeout -k 10 ${SWEEP_TIMEOUT:-400} python -u scripts/sweep.py --config $cfg $args \
      > gpurun_out/sweep_$i.txt 2>&1
  rc=$?
  cat gpurun_out/sweep_$i.txt | grep -v "^\[" | tail -40
  stop_on $rc "sweep $i ($cfg $args)"
done
