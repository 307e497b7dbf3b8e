# r05 exp41: cfg3 split targets (PU_SPLIT = n: chains of about n_ops / n ops) with the
# 4-per-CU chunk rule, alternating
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp41
rm -rf $O; mkdir -p $O
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); t=d.get('timing',{})
print(sys.argv[2], 'step %.4f ms  kernel median %s' % (d['ms_per_step'], t.get('kernel_ms_median')))" "$1" "$2"; }
for i in 1 2; do
  for v in "PU_DUMMY=1" "PU_SPLIT=2" "PU_SPLIT=4" "PU_SPLIT=5" "PU_LDS_SLOTS=2"; do
    env $v timeout -k 10 300 python -u bench.py --config cfg3 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"
  done
done
