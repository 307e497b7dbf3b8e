#!/bin/bash
# r06: matrix-pipe attribution of the protein traversal: is the 55 %
# issue stall the MFMA pipe being busy, or MFMA RAW dependency?  One rocprofv3 --pmc pass
# per counter set (MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts cycles, SQ_WAVE_CYCLES
# counts quad-cycles).  scripts/r06/mfma_collect.py writes profiles/r06_mfma_<tag>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_mfma
mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1
grep -oE "SQ_[A-Z0-9_]*MFMA[A-Z0-9_]*|SQ_[A-Z0-9_]*VALU[A-Z0-9_]*|SQ_[A-Z0-9_]*SALU[A-Z0-9_]*" $O/list_avail.txt | sort -u > $O/mfma_counters.txt
cat $O/mfma_counters.txt | tr '\n' ' '; echo
PASSA="${PASSA:-SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT}"
PASSB="${PASSB:-SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64}"
for cfg in ${CONFIGS:-cfg3}; do
  i=0
  for set in "$PASSA" "$PASSB"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/${cfg}_pass$i \
        -- python bench.py --config $cfg --steps 20 --warmup 2 --warm-seconds 0 --no-cpu-baseline \
        > $O/${cfg}_pass$i.log 2>&1
    echo "[mfma] $cfg pass$i rc=$?"
  done
done
