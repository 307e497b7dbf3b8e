# r05 exp32: per-kernel times of the pattern-compression variants (16-word column pitch):
# default (k_pack_B<4,16> + k_unpack_w<16>), PU_PATTERNS_R05 (k_pack_T + k_unpack_lds),
# PU_PACK_PW=8, PU_UNPACK_US8 -- one kernel trace each
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp32
rm -rf $O; mkdir -p $O
for r in 1 2; do
for v in "PU_DUMMY=1" "PU_PATTERNS_R05=1" "PU_PACK_PW=8" "PU_UNPACK_US8=1"; do
  d=$O/${v%%=*}_$r
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python -c "
import csv,glob,sys
f=glob.glob('$d/**/*kernel_stats.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
tot=sum(float(r['TotalDurationNs']) for r in rows)/24e3
out=['$v', 'all %.1f us/step' % tot]
for r in rows:
    if 'pack' in r['Name']: out.append('%s %.1f' % (r['Name'].split('(')[0].split('::')[-1], float(r['AverageNs'])/1e3))
print('  '.join(out))
"
done
done
