# r05 exp42: k_pmatrix_aa with one wave per (side, category) (PU_PMAT_AA64) against the
# 4-wave form: protein GPU tests on it, then kernel traces of cfg3 for both, alternating
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp42
rm -rf $O; mkdir -p $O
PU_PMAT_AA64=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "protein or cfg3 or aa or pmatri" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
for v in "PU_DUMMY=1" "PU_PMAT_AA64=1"; do
  d=$O/trace_${v%%=*}_$i
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -- python bench.py --config cfg3 --steps 200 --no-cpu-baseline > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python -c "
import csv,glob
f=glob.glob('$d/**/*kernel_stats.csv', recursive=True)[0]
print('$v', '  '.join('%s %.2f us' % (r['Name'].split('(')[0].split('::')[-1][:24], float(r['AverageNs'])/1e3) for r in csv.DictReader(open(f)) if 'pmatrix' in r['Name'] or 'mfma' in r['Name']))
"
done
done
