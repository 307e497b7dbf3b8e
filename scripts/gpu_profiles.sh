#!/bin/bash
# All bench configs in one gpurun call: kernel trace + PMC passes + bench line per config
# (scripts/gpu_round.sh with RUN_TESTS=0), then scripts/collect_profiles.py turns
# gpurun_out/prof_<tag>/ into profiles/<round>_*.  A crash or timeout stops the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
for spec in ${CONFIGS:-cfg2 cfg3 cfg4 cfg5:--lnl-only:_lnl}; do
  IFS=: read -r cfg args suffix <<< "$spec"
  echo "== $cfg $args"
  CFG=$cfg BENCH_ARGS="$args" TAGSUFFIX="$suffix" RUN_TESTS=0 PROFILE=1 BENCH_STEPS=${BENCH_STEPS:-200} \
      bash scripts/gpu_round.sh
done
