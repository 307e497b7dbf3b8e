# r06 call 40: the batch without root-partial stores (default) against PU_BATCH_ROOT=1: the
# whole GPU suite, cfg5 bench lines alternating, then cfg5's trace + PMC passes
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call40; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR" $O/pytest_gpu.log | head -20; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for v in 0 1; do
  PU_BATCH_ROOT=$v timeout -k 10 300 python -u bench.py --config cfg5 --steps 100 --warmup 10 --no-cpu-baseline --no-rank-check > $O/cfg5_root$v.json 2> $O/cfg5_root$v.err || { tail -20 $O/cfg5_root$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/cfg5_root$v.json').read().strip().splitlines()[-1])
print('cfg5 root=$v', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'))"
done
done
CONFIGS="cfg5::_batch" BENCH_STEPS=100 bash scripts/gpu_profiles.sh > $O/profiles.log 2>&1 || { tail -30 $O/profiles.log; exit 1; }
grep -E "^== |rc=" $O/profiles.log
