# r05 exp31 (third run: 16-word column pitch; pack slices 16 / 32, unpack slices 16 / 8): batched-load pack (k_pack_B) and 4-byte unpack (k_unpack_w) against the r05
# kernels (PU_PATTERNS_R05=1): pattern GPU tests, alternating bench lines, a kernel trace
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp31
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_patterns.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4f ms  %.1f M columns/s' % (d['roofline']['kernel_ms'], d['value']))" "$1" "$2"; }
for i in 1 2; do
  for v in "PU_DUMMY=1" "PU_PACK_PW=32" "PU_UNPACK_US8=1" "PU_PATTERNS_R05=1"; do
    env $v timeout -k 10 300 python -u bench.py --workload patterns --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python -c "
import csv,glob
f=glob.glob('$O/trace/**/*kernel_stats.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print('%-60s %5s avg %8.1f us  %5.1f%%' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, 100*float(r['TotalDurationNs'])/tot))
"
