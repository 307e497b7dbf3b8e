# r05 exp29: protein chain tasks interleaved in the grid (consecutive workgroups run different
# chain tasks) against the task-major grid, cfg3 KEEP and lnL-only, alternating
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp29
rm -rf $O; mkdir -p $O
PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_inter.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "protein or cfg3 or all_partials or split" > $O/tests.txt 2>&1
rc=$?; tail -1 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
line() { python -c "
import json,sys; t=open(sys.argv[1]).read(); d=json.loads([l for l in t.splitlines() if l.startswith('{')][-1])
print(sys.argv[2], 'value %.0f step %.5f kernel %.5f lnl %.10f' % (d['value'], d['ms_per_step'], d['timing']['kernel_ms_median'], d['lnl']))" "$1" "$2"; }
for i in 1 2 3; do
  for lib in libphylo_hip.so libphylo_hip_inter.so; do
    for cfg in cfg3 "cfg3 --lnl-only"; do
      PHYLO_HIP_LIB=phylo_utils_amd/$lib timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 200 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      line $O/b.json "$lib $cfg"
    done
  done
done
