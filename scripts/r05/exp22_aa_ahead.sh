# r05 exp22: protein children one op ahead (PU_AA_AHEAD) -- protein GPU tests on the new
# build, then cfg3 bench lines alternating with the -DPU_AA_AHEAD=0 build (lnL must match)
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp22
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "protein or cfg3 or pmat or all_partials or split or kernel_builds or repeated" > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/tests.txt | head; exit $rc; }
line() { python -c "
import json,sys; t=open(sys.argv[1]).read(); d=json.loads([l for l in t.splitlines() if l.startswith('{')][-1])
print(sys.argv[2], 'value %.0f step %.5f kernel %.5f lnl %.10f' % (d['value'], d['ms_per_step'], d['timing']['kernel_ms_median'], d['lnl']))" "$1" "$2"; }
for i in 1 2 3; do
  for lib in libphylo_hip.so libphylo_hip_noahead.so; do
    for cfg in cfg3 "cfg3 --lnl-only"; do
      PHYLO_HIP_LIB=phylo_utils_amd/$lib timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 200 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      line $O/b.json "$lib $cfg"
    done
  done
done
