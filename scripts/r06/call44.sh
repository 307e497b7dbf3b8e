# r06 call 44: cfg5 batch group size re-checked without the root-partial stores (56 against 48-64)
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call44; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for g in 56 48 64 52 60; do
  PU_BATCH_GROUP=$g timeout -k 10 300 python -u bench.py --config cfg5 --steps 100 --warmup 10 --no-cpu-baseline --no-rank-check > $O/cfg5_g$g.json 2> $O/cfg5_g$g.err || { tail -20 $O/cfg5_g$g.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/cfg5_g$g.json').read().strip().splitlines()[-1])
print('cfg5 group=$g', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'))"
done
done
