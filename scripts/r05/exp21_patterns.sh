# r05 exp21: fused pack / transpose / hash for pattern compression -- its GPU tests (bit-exact
# against np.unique), the N2 bench line and a kernel trace
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp21
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_patterns.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python -u bench.py --workload patterns > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('patterns: %.3f ms, %.1f M columns/s, frac %.4f' % (d['ms_per_step'], d['value'], d['roofline']['frac']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python -c "
import csv,glob
f=glob.glob('$O/trace/**/*kernel_stats.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print('%-70s %5s avg %8.1f us  %5.1f%%' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3, 100*float(r['TotalDurationNs'])/tot))
"
