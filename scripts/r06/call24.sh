# r06 call 24: cfg5 (batched, lnL-only) against the LDS stash slot count (fewer read-backs vs
# occupancy): PU_LDS_SLOTS unset (2) / 3 / 4 / 1, two rounds
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call24; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for L in def 3 4 1; do
  if [ $L = def ]; then unset PU_LDS_SLOTS; else export PU_LDS_SLOTS=$L; fi
  timeout -k 10 300 python -u bench.py --config cfg5 --steps 100 --warmup 10 --no-cpu-baseline > $O/cfg5_L$L.json 2> $O/cfg5_L$L.err || { tail -20 $O/cfg5_L$L.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/cfg5_L$L.json').read().strip().splitlines()[-1])
print('L=$L', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'))"
done
done
