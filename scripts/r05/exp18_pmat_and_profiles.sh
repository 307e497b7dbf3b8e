# r05 exp18: the protein P-kernel probe, then the r05 profiles of cfg4 and cfg2 (kernel trace,
# FETCH / WRITE PMC passes, bench line) via scripts/gpu_profiles.sh
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/exp18
timeout -k 10 120 scripts/probes/pmat_aa_probe > gpurun_out/exp18/pmat_probe.txt 2>&1 || { cat gpurun_out/exp18/pmat_probe.txt; exit 1; }
cat gpurun_out/exp18/pmat_probe.txt
CONFIGS="cfg4 cfg2" BENCH_STEPS=100 bash scripts/gpu_profiles.sh
