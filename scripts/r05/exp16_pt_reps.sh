# r05 exp16: tip-product replicas (PU_PT_REPS) on one tree's launch, the batched launch (tree /
# tile order, 1 / 7 waves) and the cfg5 bench over streams
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp16
mkdir -p $O
for v in "PU_PT_REPS=1" "PU_PT_REPS=8" "PU_PT_REPS=32" "PU_PT_REPS=8 PU_BATCH_ORDER=tile" "PU_PT_REPS=8 PU_BATCH_WAVES=7" "PU_PT_REPS=8 PU_BATCH_ORDER=tile PU_BATCH_WAVES=7" "PU_PT_REPS=1 PU_BATCH_ORDER=tile PU_BATCH_WAVES=7"; do
  echo "== $v"
  env $v PU_DEBUG_PLAN=1 timeout -k 10 300 python -u scripts/r05/batch_probe.py --trees 1,32,125 > $O/p.txt 2>&1 || { tail -20 $O/p.txt; exit 1; }
  grep -E "^batch|own launch" $O/p.txt | head -8
done
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], 'value %.0f step %.4f kernel %.4f' % (d['value'], d['ms_per_step'], r['kernel_ms']))" "$1" "$2"; }
for v in "PU_BENCH_BATCH=0 PU_PT_REPS=1" "PU_BENCH_BATCH=0 PU_PT_REPS=8" "PU_BENCH_BATCH=1 PU_PT_REPS=8 PU_BATCH_ORDER=tile PU_BATCH_WAVES=7"; do
  env $v timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  line $O/b.json "$v"
done
