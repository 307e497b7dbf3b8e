# r05 exp7: how much does one allocation of the same plan differ from another?  Five models
# of cfg2 with identical settings (PU_DUMMY only labels them), interleaved rounds
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp7
mkdir -p $O
timeout -k 10 400 python -u scripts/sweep.py --config cfg2 --grid 'PU_DUMMY=1,2,3,4,5' --sites 100000 --steps 200 --rounds 4 > $O/alloc.txt 2>&1 || exit 1
timeout -k 10 400 python -u scripts/sweep.py --config cfg2 --grid 'PU_DUMMY=1,2,3,4,5' --sites 98304 --steps 200 --rounds 4 >> $O/alloc.txt 2>&1 || exit 1
grep -h "traverse\|^config" $O/alloc.txt
