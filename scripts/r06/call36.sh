# r06 call 36: k_pmatrix_lane as one lane per P row (tip products from the row it holds) --
# the whole GPU suite, a cfg5 kernel trace, then cfg5 batch / cfg2 bench lines
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call36; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR" $O/pytest_gpu.log | head -20; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
PU_BENCH_BATCH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg5 -o run -- python3 -u bench.py --config cfg5 --steps 50 --warmup 10 --no-cpu-baseline --no-rank-check > $O/cfg5_prof.json 2> $O/cfg5_prof.err || { tail -20 $O/cfg5_prof.err; exit 1; }
f=$(find $O/prof_cfg5 -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -8
for r in 1 2; do
  PU_BENCH_BATCH=1 timeout -k 10 300 python -u bench.py --config cfg5 --steps 100 --warmup 10 --no-cpu-baseline --no-rank-check > $O/cfg5_$r.json 2> $O/cfg5_$r.err || { tail -20 $O/cfg5_$r.err; exit 1; }
  timeout -k 10 300 python -u bench.py --config cfg2 --steps 400 --warmup 20 --no-cpu-baseline --no-rank-check > $O/cfg2_$r.json 2> $O/cfg2_$r.err || { tail -20 $O/cfg2_$r.err; exit 1; }
  for c in cfg5 cfg2; do python -c "
import json; d=json.loads(open('$O/${c}_$r.json').read().strip().splitlines()[-1])
print('$c', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'))"; done
done
