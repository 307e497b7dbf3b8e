# r05 exp28: the cfg5 batched default -- kernel trace, FETCH / WRITE / instruction-mix PMC and
# the bench line (tag cfg5_batch), then its stall attribution passes
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
CONFIGS="cfg5::_batch" BENCH_STEPS=100 INSTS=1 bash scripts/gpu_profiles.sh > gpurun_out/exp28_profiles.log 2>&1 || { tail -30 gpurun_out/exp28_profiles.log; exit 1; }
grep -E "^== |rc=" gpurun_out/exp28_profiles.log
CONFIGS="cfg5::_batch:" bash scripts/r05/stall_pmc.sh
