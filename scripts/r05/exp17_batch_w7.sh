# r05 exp17: the batch with its 7-wave rule -- GPU tests, then cfg5 batched vs streams, alternating
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp17
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_batch.py > $O/batch_tests.txt 2>&1 || { tail -40 $O/batch_tests.txt; exit 1; }
grep -E "passed|failed" $O/batch_tests.txt | tail -2
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], 'value %.0f step %.4f kernel %.4f' % (d['value'], d['ms_per_step'], r['kernel_ms']), 'maxrel', d.get('lnl_max_rel_diff_vs_sync_runs'))" "$1" "$2"; }
for i in 1 2; do
  for v in "PU_BENCH_BATCH=1" "PU_BENCH_BATCH=0"; do
    env $v PU_DEBUG_PLAN=1 timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"; grep "pu batch" $O/b.err | head -1
  done
done
