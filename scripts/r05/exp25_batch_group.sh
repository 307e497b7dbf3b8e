# r05 exp25: the batch's grouped tile order (PU_BATCH_GROUP = trees per group) x waves, 125 trees
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp25
rm -rf $O; mkdir -p $O
for v in "PU_BATCH_GROUP=0" "PU_BATCH_GROUP=8" "PU_BATCH_GROUP=16" "PU_BATCH_GROUP=32" "PU_BATCH_GROUP=64" "PU_BATCH_GROUP=16 PU_BATCH_WAVES=1" "PU_BATCH_GROUP=32 PU_BATCH_WAVES=1"; do
  env $v timeout -k 10 300 python -u scripts/r05/batch_probe.py --trees 125 > $O/p.txt 2>&1 || { tail -20 $O/p.txt; exit 1; }
  echo "$v: $(grep '^batch' $O/p.txt)"
done
line() { python -c "
import json,sys; t=open(sys.argv[1]).read(); d=json.loads([l for l in t.splitlines() if l.startswith('{')][-1])
print(sys.argv[2], 'value %.0f step %.4f maxrel %s' % (d['value'], d['ms_per_step'], d.get('lnl_max_rel_diff_vs_sync_runs')))" "$1" "$2"; }
for i in 1 2; do
  for v in "PU_BENCH_BATCH=0" "PU_BENCH_BATCH=1 PU_BATCH_GROUP=16" "PU_BENCH_BATCH=1 PU_BATCH_GROUP=32"; do
    env $v timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"
  done
done
