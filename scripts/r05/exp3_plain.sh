# r05 exp3: the plain grid with the pattern weight preloaded, one staging chunk or two, worker
# lists, against the r04 library: same-box sweep, alternating libraries and settings
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp3
mkdir -p $O
PU_LIST=0 PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_stamps.so timeout -k 10 200 python -u scripts/wg_timeline.py --sites 100000 --taxa 50 --launches 2 --out $O/tl_plain > $O/tl_plain.log 2>&1 || exit 1
PU_LIST=0 PU_CHUNK_USES=64 PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_stamps.so timeout -k 10 200 python -u scripts/wg_timeline.py --sites 100000 --taxa 50 --launches 2 --out $O/tl_plain_c64 > $O/tl_plain_c64.log 2>&1 || exit 1
for r in 1 2; do
  PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_r04.so timeout -k 10 300 python -u scripts/sweep.py --config cfg2 --grid 'PU_CHUNK_USES=,64' --sites 62500,87500,100000,112500,131072 --steps 200 --rounds 3 > $O/sweep_r04_$r.txt 2>&1 || exit 1
  timeout -k 10 300 python -u scripts/sweep.py --config cfg2 --grid 'PU_LIST=0,1;PU_CHUNK_USES=,64' --sites 62500,87500,100000,112500,131072 --steps 200 --rounds 3 > $O/sweep_new_$r.txt 2>&1 || exit 1
done
grep -h "traverse\|^config" $O/sweep_*.txt
