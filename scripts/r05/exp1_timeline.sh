# r05 exp1: per-workgroup timeline with the pattern weight preloaded, default chunking vs one
# chunk (PU_CHUNK_USES=64); then k_prune timing r04 build vs this build, both chunkings
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp1
mkdir -p $O
L=phylo_utils_amd/libphylo_hip_stamps.so
PHYLO_HIP_LIB=$L timeout -k 10 200 python -u scripts/wg_timeline.py --sites 100000 --taxa 50 --launches 2 --out $O/tl_def > $O/tl_def.log 2>&1 || exit $?
PU_CHUNK_USES=64 PHYLO_HIP_LIB=$L timeout -k 10 200 python -u scripts/wg_timeline.py --sites 100000 --taxa 50 --launches 2 --out $O/tl_c64 > $O/tl_c64.log 2>&1 || exit $?
for r in 1 2; do
for lib in libphylo_hip_r04.so libphylo_hip.so; do
  PHYLO_HIP_LIB=phylo_utils_amd/$lib timeout -k 10 200 python -u scripts/sweep.py --config cfg2 --grid 'PU_CHUNK_USES=,64' --steps 200 --rounds 3 >> $O/sweep_$lib.txt 2>&1 || exit $?
done
done
echo done
