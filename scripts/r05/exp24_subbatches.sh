# r05 exp24: cfg5 as k batches of 125 / k trees on k streams (PU_BENCH_BATCH=k), 7-wave rule
# and the default build, against the per-tree launches over 4 streams
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp24
rm -rf $O; mkdir -p $O
line() { python -c "
import json,sys; t=open(sys.argv[1]).read(); d=json.loads([l for l in t.splitlines() if l.startswith('{')][-1])
print(sys.argv[2], 'value %.0f step %.4f maxrel %s' % (d['value'], d['ms_per_step'], d.get('lnl_max_rel_diff_vs_sync_runs')))" "$1" "$2"; }
for i in 1 2; do
  for v in "PU_BENCH_BATCH=0" "PU_BENCH_BATCH=2" "PU_BENCH_BATCH=4" "PU_BENCH_BATCH=4 PU_BATCH_WAVES=1" "PU_BENCH_BATCH=8" "PU_BENCH_BATCH=8 PU_BATCH_WAVES=1"; do
    env $v timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"
  done
done
