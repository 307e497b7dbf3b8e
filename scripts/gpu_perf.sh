#!/bin/bash
# Correctness + performance evidence in one gpurun call.  Every GPU step is time-limited;
# a crash/abort/timeout stops the script (test failures, rc=1, do not).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@"
  local rc=$?
  echo "[gpu_perf] $name rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[gpu_perf] stopping after $name"; exit "$rc"; fi
}
RUN_TESTS=${RUN_TESTS:-1}
CFG=${CFG:-cfg2}
if [ "$RUN_TESTS" = 1 ]; then
  step pytest 900 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider -o log_cli=false \
       > gpurun_out/pytest_gpu.log 2>&1
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ -n "$SWEEP" ]; then
  eval "step sweep 600 python scripts/sweep.py --config $CFG $SWEEP" > gpurun_out/sweep_$CFG.txt 2>&1
  cat gpurun_out/sweep_$CFG.txt
fi
if [ -n "$PROFILE" ]; then
  rm -rf gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write
  step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace \
       -- python bench.py --config $CFG --steps 100 --warmup 10 --warm-seconds 1 --no-cpu-baseline $PROFILE_ARGS \
       > gpurun_out/bench_trace_$CFG.json 2> gpurun_out/bench_trace_$CFG.err
  step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch \
       -- python bench.py --config $CFG --steps 20 --warmup 2 --warm-seconds 0 --no-cpu-baseline $PROFILE_ARGS \
       > /dev/null 2> gpurun_out/pmc_fetch.err
  step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write \
       -- python bench.py --config $CFG --steps 20 --warmup 2 --warm-seconds 0 --no-cpu-baseline $PROFILE_ARGS \
       > /dev/null 2> gpurun_out/pmc_write.err
fi
if [ "${BENCH:-1}" = 1 ]; then
  step bench 900 python bench.py --config $CFG --steps ${BENCH_STEPS:-200} --warmup 20 ${BENCH_ARGS} \
       > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err
  cat gpurun_out/bench_$CFG.json
fi
