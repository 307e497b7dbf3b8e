# r05 exp26: the batch's grouped order as default -- batch GPU tests, then cfg5 bench lines
# (batched default vs per-tree streams) and a group / waves sweep of the bench
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp26
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_parity.py -k "batch or cfg5" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
grep -E "passed|failed" $O/tests.txt | tail -1
line() { python -c "
import json,sys; t=open(sys.argv[1]).read(); d=json.loads([l for l in t.splitlines() if l.startswith('{')][-1])
print(sys.argv[2], 'value %.0f step %.4f kernel %s maxrel %s' % (d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'), d.get('lnl_max_rel_diff_vs_sync_runs')))" "$1" "$2"; }
for i in 1 2; do
  for v in "PU_BENCH_BATCH=1" "PU_BENCH_BATCH=0" "PU_BATCH_GROUP=8" "PU_BATCH_GROUP=8 PU_BATCH_WAVES=1" "PU_BATCH_GROUP=24" "PU_BATCH_GROUP=16 PU_BATCH_WAVES=1"; do
    env $v timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"
  done
done
