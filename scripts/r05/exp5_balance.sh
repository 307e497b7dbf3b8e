# r05 exp5: is the cfg2 kernel set by the most-loaded CU?  1536 blocks (6 per CU exactly),
# 1537 (one CU gets 7), 1563 (cfg2), 1600; and the per-CU end times of the first two
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp5
mkdir -p $O
for r in 1 2; do
timeout -k 10 300 python -u scripts/sweep.py --config cfg2 --sites 98304,98368,100000,102400,106496 --steps 200 --rounds 3 > $O/sweep_$r.txt 2>&1 || exit 1
done
grep -h "traverse\|^config" $O/sweep_*.txt
PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_stamps.so timeout -k 10 200 python -u scripts/wg_timeline.py --sites 98304,98368 --taxa 50 --launches 2 --out $O/tl > $O/tl.log 2>&1 || exit 1
grep "span\|end perc" $O/tl.log
