# r05 exp10: why the bench's k_prune events read ~5 % above the sweep's on one box
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp10
mkdir -p $O
timeout -k 10 300 python -u scripts/sweep.py --config cfg2 --grid 'PU_DUMMY=1,2' --sites 100000 --steps 200 --rounds 4 > $O/sweep1.txt 2>&1 || exit 1
grep -h "traverse" $O/sweep1.txt
run() { timeout -k 10 300 python -u bench.py "$@" > $O/b.txt 2>&1 || { tail -20 $O/b.txt; exit 1; }; python -c "
import json,sys; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); r=d['roofline']; t=d['timing']
print(sys.argv[1:], 'value %.0f step %.4f kernel med %.4f mean %.4f frac %.4f' % (d['value'], d['ms_per_step'], t['kernel_ms_median'], t['kernel_ms_mean'], r['frac']))" "$@" "$PU_BENCH_STREAM"; }
run
run --events timed
export PU_BENCH_STREAM=side
run
run --events timed
unset PU_BENCH_STREAM
timeout -k 10 300 python -u scripts/sweep.py --config cfg2 --grid 'PU_DUMMY=1,2' --sites 100000 --steps 200 --rounds 4 > $O/sweep2.txt 2>&1 || exit 1
grep -h "traverse" $O/sweep2.txt
