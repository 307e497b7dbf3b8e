# r06 final evidence, call A: the whole GPU suite, smoke, then the edges and patterns lines with
# their kernel traces (and the patterns FETCH / WRITE passes)
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_final2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR" $O/pytest_gpu.log | head -20; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for w in edges patterns; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  rm -rf $O/trace_$w
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$w -- python bench.py --workload $w --steps 20 --no-cpu-baseline > $O/trace_$w.log 2>&1 || { tail -20 $O/trace_$w.log; exit 1; }
done
rm -rf $O/pfetch $O/pwrite
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pfetch -- python bench.py --workload patterns --steps 3 --warmup 5 --no-cpu-baseline > $O/pfetch.log 2>&1 || { tail -20 $O/pfetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pwrite -- python bench.py --workload patterns --steps 3 --warmup 5 --no-cpu-baseline > $O/pwrite.log 2>&1 || { tail -20 $O/pwrite.log; exit 1; }
python scripts/r05/patterns_traffic.py $O/pfetch $O/pwrite $O/traffic_patterns.json > /dev/null
python -c "
import json
for w in ('edges', 'patterns'):
    d = json.loads(open('$O/bench_%s.json' % w).read().strip().splitlines()[-1])
    print(w, d['value'], d['ms_per_step'], d.get('roofline', {}).get('frac'))
print('patterns PMC', json.load(open('$O/traffic_patterns.json'))['hbm_bytes_per_call'])"
