# r05 exp6 (timing only): does a narrower tile width balance the grid?  PU_HACK_W=56 build:
# lanes 56..63 store nothing, so 1792 tiles of 64 lanes move the bytes of 100352 sites in 1792
# blocks (7 per CU).  Against the normal build at 98304 / 100000 / 114688 sites
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp6
mkdir -p $O
for r in 1 2; do
PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_w56.so timeout -k 10 300 python -u scripts/sweep.py --config cfg2 --sites 114688 --steps 200 --rounds 3 > $O/w56_$r.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/sweep.py --config cfg2 --sites 98304,100000,114688 --steps 200 --rounds 3 > $O/base_$r.txt 2>&1 || exit 1
done
grep -h "traverse\|^config" $O/*.txt
