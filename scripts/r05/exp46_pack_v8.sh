# r05 exp46: k_pack<8> (1024 columns per workgroup, 8-byte loads, 1 KB per row and workgroup;
# 74 KB tile: 2 workgroups per CU; PU_PACK_V8) against k_pack<4>: tests on it, kernel times
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp46
rm -rf $O; mkdir -p $O
PU_PACK_V8=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_patterns.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
for v in "PU_DUMMY=1" "PU_PACK_V8=1"; do
  d=$O/trace_${v%%=*}_$i
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python -c "
import csv,glob
f=glob.glob('$d/**/*kernel_stats.csv', recursive=True)[0]
print('$v', '  '.join('%s %.1f us' % (r['Name'].split('(')[0].split('::')[-1][:24], float(r['AverageNs'])/1e3) for r in csv.DictReader(open(f)) if 'k_pack' in r['Name']))
"
done
done
