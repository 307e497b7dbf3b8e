# r05 exp23: protein CLV store policy sc1 nt (PU_AA_POL=3) and scaler stores from one lane
# group (PU_AA_SCALE16=1) against the default build, cfg3 bench lines alternating
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp23
rm -rf $O; mkdir -p $O
for lib in libphylo_hip_pol3.so libphylo_hip_s16.so; do
  PHYLO_HIP_LIB=phylo_utils_amd/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "protein or cfg3 or all_partials or split" > $O/tests_$lib.txt 2>&1
  rc=$?; echo "$lib: $(tail -1 $O/tests_$lib.txt)"; [ $rc -ne 0 ] && exit $rc
done
line() { python -c "
import json,sys; t=open(sys.argv[1]).read(); d=json.loads([l for l in t.splitlines() if l.startswith('{')][-1])
print(sys.argv[2], 'value %.0f step %.5f kernel %.5f lnl %.10f' % (d['value'], d['ms_per_step'], d['timing']['kernel_ms_median'], d['lnl']))" "$1" "$2"; }
for i in 1 2 3; do
  for lib in libphylo_hip.so libphylo_hip_pol3.so libphylo_hip_s16.so; do
    PHYLO_HIP_LIB=phylo_utils_amd/$lib timeout -k 10 300 python -u bench.py --config cfg3 --no-cpu-baseline --steps 200 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$lib"
  done
done
