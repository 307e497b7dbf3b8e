#!/bin/bash
# r05: stall attribution of the traversal kernel per config (three SQ passes, 8 counters each,
# one rocprofv3 run per pass; MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY
# ~ WAVE_CYCLES, all in quad-cycles).  scripts/r05/stall_collect.py writes profiles/r05_stall_<tag>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
PASS1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_WAVES"
PASS2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_BUSY_CYCLES"
PASS3="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM_WR"
for spec in ${CONFIGS:-cfg5::_batch: cfg5::_streams:PU_BENCH_BATCH=0 cfg2 cfg3}; do
  IFS=: read -r cfg args suffix envs <<< "$spec"
  D=gpurun_out/stall_${cfg}${suffix}
  rm -rf $D; mkdir -p $D
  i=0
  for set in "$PASS1" "$PASS2" "$PASS3"; do
    i=$((i+1))
    env $envs timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $D/pass$i \
        -- python bench.py --config $cfg --steps 20 --warmup 2 --warm-seconds 0 --no-cpu-baseline $args \
        > $D/pass$i.log 2>&1
    rc=$?
    echo "[stall] $cfg$suffix pass$i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $D/pass$i.log; exit $rc; fi
  done
done
