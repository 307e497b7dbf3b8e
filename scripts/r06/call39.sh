# r06 call 39: the fused lnL sum polling 4 slots per thread at once (TraverseArgs::red_slots, DNA) against
# the k_reduce launch (PU_RED_FUSED=0; r06 final: the default is the launch, 1 opts in): the whole GPU suite, then cfg2 bench lines
# alternating
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call39; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR" $O/pytest_gpu.log | head -20; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
for cfg in cfg2; do
for v in 1 0; do
  PU_RED_FUSED=$v timeout -k 10 300 python -u bench.py --config $cfg --steps 400 --warmup 20 --no-cpu-baseline --no-rank-check > $O/${cfg}_r$v.json 2> $O/${cfg}_r$v.err || { tail -20 $O/${cfg}_r$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/${cfg}_r$v.json').read().strip().splitlines()[-1])
print('$cfg fused=$v', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'))"
done
done
done
