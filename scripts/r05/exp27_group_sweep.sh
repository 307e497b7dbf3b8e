# r05 exp27: batch group size sweep on the cfg5 bench (W7 rule), two rounds
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp27
rm -rf $O; mkdir -p $O
line() { python -c "
import json,sys; t=open(sys.argv[1]).read(); d=json.loads([l for l in t.splitlines() if l.startswith('{')][-1])
print(sys.argv[2], 'value %.0f step %.4f maxrel %s' % (d['value'], d['ms_per_step'], d.get('lnl_max_rel_diff_vs_sync_runs')))" "$1" "$2"; }
for i in 1 2; do
  for g in 16 20 24 28 40 48; do
    PU_BATCH_GROUP=$g timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "group $g"
  done
done
