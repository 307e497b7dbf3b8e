# r06 call 41: cfg2, fused lnL sum (default) against the k_reduce launch (PU_RED_FUSED=0), four
# alternating rounds on one box: value, step, traversal event median, roofline fraction
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call41; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3 4; do
for v in 1 0; do
  PU_RED_FUSED=$v timeout -k 10 300 python -u bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-rank-check > $O/cfg2_r$v.json 2> $O/cfg2_r$v.err || { tail -20 $O/cfg2_r$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/cfg2_r$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('cfg2 fused=$v', d['value'], d['ms_per_step'], r.get('kernel_ms'), r['frac'], r.get('frac_of_ceiling'))"
done
done
