# r06 call 17: device Newton phase stamps inside the tile phase (factors + barrier, sites + wave
# sums, barrier)
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call17; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/r06/newton_probe.py > $O/newton_probe.log 2>&1 || { tail -30 $O/newton_probe.log; exit 1; }
grep -v amdgpu.ids $O/newton_probe.log
