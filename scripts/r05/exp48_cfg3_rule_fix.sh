# r05 exp48: the chunk rule with the LDS margin (exp47 showed the first rule left cfg3 at 3
# workgroups per CU): resident waves, protein GPU tests, cfg3 lines against PU_CHUNK_USES=32
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp48
rm -rf $O; mkdir -p $O
d=$O/occ
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES --output-format csv -d $d -- python bench.py --config cfg3 --steps 10 --warmup 2 --warm-seconds 0 --no-cpu-baseline > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
python -c "
import csv,glob
vals={}
for f in glob.glob('$d/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_prune_mfma' in r['Kernel_Name']:
            vals.setdefault(r['Counter_Name'],[]).append(float(r['Counter_Value']))
print('default: resident waves per busy CU %.2f' % (4*sum(vals['SQ_WAVE_CYCLES'])/sum(vals['SQ_BUSY_CU_CYCLES'])))
"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_edges.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); t=d.get('timing',{})
print(sys.argv[2], 'step %.4f ms  kernel median %s' % (d['ms_per_step'], t.get('kernel_ms_median')))" "$1" "$2"; }
for i in 1 2 3; do
  for v in "PU_DUMMY=1" "PU_CHUNK_USES=32"; do
    env $v timeout -k 10 300 python -u bench.py --config cfg3 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"
  done
done
