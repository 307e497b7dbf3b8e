#!/bin/bash
# One gpurun call: GPU tests, then (PROFILE=1) kernel trace + the two PMC passes of bench.py
# for $CFG, then the bench line.  Every GPU step has its own time limit; a crash, abort or
# timeout ends the call (test failures, rc=1, do not).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@"
  local rc=$?
  echo "[gpu_round] $name rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[gpu_round] stopping after $name"; exit "$rc"; fi
}
CFG=${CFG:-cfg2}
if [ "${RUN_TESTS:-1}" = 1 ]; then
  step pytest ${TEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 120 \
       --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -15
fi
TAG=${CFG}${TAGSUFFIX}
if [ -n "$PROFILE" ]; then
  P=gpurun_out/prof_$TAG
  rm -rf $P
  step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/prof_trace \
       -- python bench.py --config $CFG --steps 100 --warmup 10 --warm-seconds 1 --no-cpu-baseline $BENCH_ARGS \
       > gpurun_out/bench_trace_$TAG.json 2> gpurun_out/bench_trace_$TAG.err
  step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/prof_fetch \
       -- python bench.py --config $CFG --steps 20 --warmup 2 --warm-seconds 0 --no-cpu-baseline $BENCH_ARGS \
       > /dev/null 2> gpurun_out/pmc_fetch.err
  step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/prof_write \
       -- python bench.py --config $CFG --steps 20 --warmup 2 --warm-seconds 0 --no-cpu-baseline $BENCH_ARGS \
       > /dev/null 2> gpurun_out/pmc_write.err
  if [ -n "$INSTS" ]; then  # instruction mix + busy cycles of the traversal (one pass, 6 SQ counters)
    step pmc_insts 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CU_CYCLES \
         --output-format csv -d $P/prof_insts \
         -- python bench.py --config $CFG --steps 20 --warmup 2 --warm-seconds 0 --no-cpu-baseline $BENCH_ARGS \
         > /dev/null 2> gpurun_out/pmc_insts.err
  fi
fi
if [ "${BENCH:-1}" = 1 ]; then
  step bench 600 python bench.py --config $CFG --steps ${BENCH_STEPS:-200} --warmup 20 $BENCH_ARGS \
       > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  cat gpurun_out/bench_$TAG.json; tail -4 gpurun_out/bench_$TAG.err
fi
