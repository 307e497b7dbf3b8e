# r05 exp37: one composite (rank, class) sort instead of two 32-bit sorts, against a10b06d
# (
# pattern code (libphylo_hip_prevpat2.so: same other objects): pattern GPU tests, alternating
# bench lines, a kernel trace
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp37
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_patterns.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'kernel %.4f ms  step %.4f ms  %.1f M columns/s  U %d' % (d['roofline']['kernel_ms'], d['ms_per_step'], d['value'], d['config']['patterns']))" "$1" "$2"; }
for i in 1 2 3; do
  for v in "PU_DUMMY=1" "PHYLO_HIP_LIB=$PWD/phylo_utils_amd/libphylo_hip_prevpat2.so"; do
    env $v timeout -k 10 300 python -u bench.py --workload patterns --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "${v:0:40}"
  done
done
d=$O/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
python -c "
import csv,glob
f=glob.glob('$d/**/*kernel_stats.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
tot=sum(float(r['TotalDurationNs']) for r in rows)/24e3
print('kernel sum %.1f us/step' % tot)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:10]:
    print('   %-60s %5s %8.1f us/step' % (r['Name'][:60], r['Calls'], float(r['TotalDurationNs'])/24e3))
"
