# r04: the default plan over 50k-300k DNA sites (12.5k apart, plus
# 131072) on the cfg2 tree, then 500- and 1000-taxon trees; per-update rate and the 5 %
# neighbour check into gpurun_out/sweep_*.json
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=$(python -c "print(','.join(str(s) for s in sorted(set(list(range(50000, 300001, 12500)) + [131072]))))")
timeout -k 10 900 python -u scripts/sweep.py --config cfg2 --sites "$S" --steps 100 --rounds 3 \
  --json gpurun_out/sweep_cfg2_sites.json > gpurun_out/sweep_cfg2_sites.txt 2>&1 || exit $?
tail -3 gpurun_out/sweep_cfg2_sites.txt
timeout -k 10 900 python -u scripts/sweep.py --config cfg2 --taxa 500,1000 \
  --sites 50000,100000,131072,200000,300000 --steps 50 --rounds 3 \
  --json gpurun_out/sweep_cfg2_taxa.json > gpurun_out/sweep_cfg2_taxa.txt 2>&1 || exit $?
tail -3 gpurun_out/sweep_cfg2_taxa.txt
