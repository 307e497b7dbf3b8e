# r06 call 33: cfg5 launch shape re-check: one batch of 125 trees (default) vs 2 / 3 batches on
# their own streams (PU_BENCH_BATCH), and the tree-group size (PU_BATCH_GROUP 40 default / 56)
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call33; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for v in b1 b2 b3 g56; do
  unset PU_BENCH_BATCH PU_BATCH_GROUP
  case $v in b*) export PU_BENCH_BATCH=${v#b};; g*) export PU_BATCH_GROUP=${v#g};; esac
  timeout -k 10 300 python -u bench.py --config cfg5 --steps 100 --warmup 10 --no-cpu-baseline > $O/c5_$v.json 2> $O/c5_$v.err || { tail -20 $O/c5_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'))"
done
done
