# r05 exp44: the unpack's gather reads each 128-byte line twice (8-word slices, the line's
# other half a slice later, after the L2 has dropped it: PMC 1.95 GB for 1.45 GB
# algorithmic).  k_unpack_lds<16> (whole-line slices, 128 patterns, 2-byte stores;
# PU_UNPACK_LDS16) against k_unpack_w: tests, kernel times, FETCH_SIZE
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp44
rm -rf $O; mkdir -p $O
PU_UNPACK_LDS16=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_patterns.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
for v in "PU_DUMMY=1" "PU_UNPACK_LDS16=1"; do
  d=$O/trace_${v%%=*}_$i
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python -c "
import csv,glob
f=glob.glob('$d/**/*kernel_stats.csv', recursive=True)[0]
print('$v', '  '.join('%s %.1f us' % (r['Name'].split('(')[0].split('::')[-1][:24], float(r['AverageNs'])/1e3) for r in csv.DictReader(open(f)) if 'unpack' in r['Name']))
"
done
done
for v in "PU_DUMMY=1" "PU_UNPACK_LDS16=1"; do
  env $v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_${v%%=*} -- python bench.py --workload patterns --steps 3 --warmup 5 --no-cpu-baseline > $O/fetch_${v%%=*}.log 2>&1 || { tail -20 $O/fetch_${v%%=*}.log; exit 1; }
done
echo ok
