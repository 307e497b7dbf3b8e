# r06 call 46: the cfg5 bench line again, reading the committed groups-of-56 trace and PMC files
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call46; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config cfg5 > $O/bench_cfg5_batch.json 2> $O/bench_cfg5_batch.err || { tail -20 $O/bench_cfg5_batch.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_cfg5_batch.json').read().strip().splitlines()[-1]); r=d['roofline']
print('cfg5', d['value'], d['ms_per_step'], r['kernel_ms'], r['traffic'], r.get('rocprof_check'), d.get('cpu_baseline', {}).get('value'))"
