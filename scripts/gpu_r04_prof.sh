# r04: committed evidence -- per config: rocprofv3 kernel trace, PMC FETCH/WRITE passes, the
# instruction-mix pass, and the bench line (scripts/gpu_round.sh PROFILE=1 INSTS=1)
cd "${GRAFT_REPO_ROOT}"
export INSTS=1
CONFIGS="${CONFIGS:-cfg2 cfg3 cfg4 cfg5:--lnl-only:_lnl}" bash scripts/gpu_profiles.sh
