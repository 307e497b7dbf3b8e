# r06 call 9 = calls 7 + 8 (the pool was full for an hour): device Newton tests, stamps and the
# edges line; the cfg5 group sweep; the protein tip-code look-ahead parity and cfg3 A/B
cd "${GRAFT_REPO_ROOT}"
bash scripts/r06/call8.sh || exit $?
bash scripts/r06/call7.sh || exit $?
