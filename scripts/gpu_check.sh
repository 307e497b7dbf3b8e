#!/bin/bash
# One gpurun call: smoke, GPU parity tests, a short bench.  Every GPU step has its own
# time limit; a crash/abort/timeout (exit >= 124 or signal) stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok_or_stop() {  # rc 0/1 (test failures) continue; anything else ends the call
  local rc=$1 what=$2
  echo "[gpu_check] $what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[gpu_check] stopping after $what"; exit "$rc"; fi
}
rocm-smi --showproductname > gpurun_out/rocm_smi.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
ok_or_stop $? smoke
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
ok_or_stop $? pytest
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-100} --warmup 10 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
ok_or_stop $? bench
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/bench.json
