# r05 exp11: layout trial over (allocation, pitch) vs pitch only vs off, three models each
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp11
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pitch" > $O/pitch_test.txt 2>&1 || { tail -30 $O/pitch_test.txt; exit 1; }
tail -1 $O/pitch_test.txt
PU_DEBUG_PLAN=1 timeout -k 10 500 python -u scripts/sweep.py --config cfg2 --grid 'PU_PITCH_TRIAL:PU_ALLOC_TRIAL=0:1,1:1,1:3;PU_DUMMY=1,2,3' --sites 100000 --steps 200 --rounds 4 > $O/sweep.txt 2>&1 || { tail -30 $O/sweep.txt; exit 1; }
grep -h "traverse\|layout trial" $O/sweep.txt
for i in 1 2; do timeout -k 10 300 python -u bench.py > $O/b.txt 2>&1 || { tail -20 $O/b.txt; exit 1; }; python -c "
import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); r=d['roofline']; t=d['timing']
print('value %.0f step %.4f kernel med %.4f mean %.4f frac %.4f' % (d['value'], d['ms_per_step'], t['kernel_ms_median'], t['kernel_ms_mean'], r['frac']))"; done
