# r05 exp13: exp12 (multi-tree launch tests, cfg5 batched vs streams, refactor A/B), then the
# stall-attribution PMC passes (cfg5 batched / streams, cfg2, cfg3)
cd "${GRAFT_REPO_ROOT}"
bash scripts/r05/exp12_batch.sh && bash scripts/r05/stall_pmc.sh
