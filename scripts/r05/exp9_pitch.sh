# r05 exp9: the plan-time layout pitch trial -- bitwise test, GPU suite, then cfg2 with the
# trial on / off on several allocations (PU_DUMMY only labels them), and two bench lines
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp9
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pitch" > $O/pitch_test.txt 2>&1 || { tail -30 $O/pitch_test.txt; exit 1; }
tail -3 $O/pitch_test.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_suite.txt 2>&1 || { tail -30 $O/gpu_suite.txt; exit 1; }
tail -3 $O/gpu_suite.txt
PU_DEBUG_PLAN=1 timeout -k 10 400 python -u scripts/sweep.py --config cfg2 --grid 'PU_PITCH_TRIAL=0,1;PU_DUMMY=1,2,3' --sites 100000 --steps 200 --rounds 4 > $O/sweep.txt 2>&1 || { tail -30 $O/sweep.txt; exit 1; }
grep -h "traverse\|pitch trial" $O/sweep.txt
for i in 1 2; do timeout -k 10 300 python -u bench.py > $O/bench$i.txt 2>&1 || { tail -30 $O/bench$i.txt; exit 1; }; tail -1 $O/bench$i.txt; done
