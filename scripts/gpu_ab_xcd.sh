#!/bin/bash
# A/B: XCD-contiguous workgroup->tile mapping (PU_STORE_MODE=64) against the default, cfg2
# and cfg4, alternating in processes of their own.  Stops at the first failing GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
mkdir -p gpurun_out/abx
for i in 1 2 3; do
  for cfg in cfg2 cfg4; do
    timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/abx/${cfg}_def_$i.json 2>>gpurun_out/abx/err.log
    PU_STORE_MODE=64 timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/abx/${cfg}_xcd_$i.json 2>>gpurun_out/abx/err.log
  done
done
