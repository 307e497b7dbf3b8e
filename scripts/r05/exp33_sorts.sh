# r05 exp33: Onesweep radix sorts from 64k items (default) against rocPRIM's merge path
# (PU_SORT_MERGE=1), with the k_pack_B<4,8> / k_unpack_w<8> defaults: pattern GPU tests,
# alternating bench lines, a kernel trace of each
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp33
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_patterns.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
PU_SORT_MERGE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_patterns.py > $O/tests_merge.txt 2>&1 || { tail -30 $O/tests_merge.txt; exit 1; }
tail -1 $O/tests_merge.txt
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'kernel %.4f ms  step %.4f ms  %.1f M columns/s' % (d['roofline']['kernel_ms'], d['ms_per_step'], d['value']))" "$1" "$2"; }
for i in 1 2 3; do
  for v in "PU_DUMMY=1" "PU_SORT_MERGE=1"; do
    env $v timeout -k 10 300 python -u bench.py --workload patterns --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"
  done
done
for v in "PU_DUMMY=1" "PU_SORT_MERGE=1"; do
  d=$O/trace_${v%%=*}
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python -c "
import csv,glob
f=glob.glob('$d/**/*kernel_stats.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
tot=sum(float(r['TotalDurationNs']) for r in rows)/24e3
print('$v', 'kernel sum %.1f us/step' % tot)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:6]:
    print('   %-60s %5s %8.1f us/step' % (r['Name'][:60], r['Calls'], float(r['TotalDurationNs'])/24e3))
"
done
