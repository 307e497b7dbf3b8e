#!/bin/bash
# cfg3 A/B of the P kernel and lnL-sum launch forms (each in its own process: the switches
# are read once per process), after the GPU tests.  Stops at the first failing GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
mkdir -p gpurun_out/ab3
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab3/gputest.log 2>&1
tail -2 gpurun_out/ab3/gputest.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --config cfg3 --no-cpu-baseline > gpurun_out/ab3/new_$i.json 2>>gpurun_out/ab3/err.log
  PU_LSE_TWO_LAUNCH=1 timeout -k 10 120 python bench.py --config cfg3 --no-cpu-baseline > gpurun_out/ab3/lse2_$i.json 2>>gpurun_out/ab3/err.log
  PU_PMAT_AA_SIDE=1 timeout -k 10 120 python bench.py --config cfg3 --no-cpu-baseline > gpurun_out/ab3/side_$i.json 2>>gpurun_out/ab3/err.log
  PU_PMAT_BLOCK=1 PU_LSE_TWO_LAUNCH=1 timeout -k 10 120 python bench.py --config cfg3 --no-cpu-baseline > gpurun_out/ab3/old_$i.json 2>>gpurun_out/ab3/err.log
done
