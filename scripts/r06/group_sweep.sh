#!/bin/bash
# r06: cfg5 batch grid group size with the shared alignment (PU_BATCH_GROUP), same box,
# alternating rounds -> gpurun_out/r06_ab/cfg5_groups.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_ab; mkdir -p $O
for i in $(seq 1 ${ROUNDS:-2}); do
  for g in ${GROUPS_:-16 24 32 40 48 64}; do
    PU_BATCH_GROUP=$g timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 \
        --no-cpu-baseline > $O/line.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    python -c "
import json; d = json.loads(open('$O/line.json').read().strip().splitlines()[-1])
print('g %-3s value %.1f step %.4f ms kernel %.4f ms' % ('$g', d['value'], d['ms_per_step'], d['roofline']['kernel_ms']))" | tee -a $O/cfg5_groups.txt
  done
done
