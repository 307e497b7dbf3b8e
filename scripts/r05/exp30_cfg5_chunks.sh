# r05 exp30: cfg5 batched -- staging chunk size (PU_CHUNK_USES) and group 24 vs 40
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp30
rm -rf $O; mkdir -p $O
line() { python -c "
import json,sys; t=open(sys.argv[1]).read(); d=json.loads([l for l in t.splitlines() if l.startswith('{')][-1])
print(sys.argv[2], 'value %.0f step %.4f maxrel %s' % (d['value'], d['ms_per_step'], d.get('lnl_max_rel_diff_vs_sync_runs')))" "$1" "$2"; }
for i in 1 2; do
  for v in "PU_DUMMY=1" "PU_CHUNK_USES=16" "PU_CHUNK_USES=48" "PU_CHUNK_USES=100" "PU_BATCH_GROUP=40" "PU_BATCH_GROUP=56"; do
    env $v timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"
  done
done
