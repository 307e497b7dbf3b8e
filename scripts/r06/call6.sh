# r06 call 6: device Newton phase stamps (debug), then the profiles of call 5
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call6; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/r06/newton_probe.py > $O/newton_probe.log 2>&1 || { tail -30 $O/newton_probe.log; exit 1; }
cat $O/newton_probe.log | grep -v amdgpu.ids
bash scripts/r06/call5.sh
