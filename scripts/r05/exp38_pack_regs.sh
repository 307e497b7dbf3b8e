# r05 exp38: the LDS-free pack (k_pack_r: 32-row batches, each lane stores its columns' words
# directly) against the LDS-tile pack (PU_PACK_LDS=1): pattern GPU tests, alternating bench
# lines, per-kernel times of both
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp38
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_patterns.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'kernel %.4f ms  step %.4f ms  %.1f M columns/s' % (d['roofline']['kernel_ms'], d['ms_per_step'], d['value']))" "$1" "$2"; }
for i in 1 2 3; do
  for v in "PU_DUMMY=1" "PU_PACK_LDS=1"; do
    env $v timeout -k 10 300 python -u bench.py --workload patterns --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"
  done
done
for v in "PU_DUMMY=1" "PU_PACK_LDS=1"; do
  d=$O/trace_${v%%=*}
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -- python bench.py --workload patterns --steps 20 --no-cpu-baseline > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python -c "
import csv,glob
f=glob.glob('$d/**/*kernel_stats.csv', recursive=True)[0]
rows=list(csv.DictReader(open(f)))
print('$v', '  '.join('%s %.1f' % (r['Name'].split('(')[0].split('::')[-1], float(r['AverageNs'])/1e3) for r in rows if 'pack' in r['Name']))
"
done
