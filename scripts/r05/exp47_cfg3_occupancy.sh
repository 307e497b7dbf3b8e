# r05 exp47: does a shorter tip-code chunk give cfg3 a fourth workgroup per CU?  Resident
# waves per CU = 4 * SQ_WAVE_CYCLES (quad-cycles) / SQ_BUSY_CU_CYCLES, one --pmc pass per
# chunk target
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp47
rm -rf $O; mkdir -p $O
for v in "PU_DUMMY=1" "PU_CHUNK_USES=4" "PU_CHUNK_USES=8" "PU_CHUNK_USES=32"; do
  d=$O/${v//=/_}
  env $v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES --output-format csv -d $d -- python bench.py --config cfg3 --steps 10 --warmup 2 --warm-seconds 0 --no-cpu-baseline > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python -c "
import csv,glob
vals={}
for f in glob.glob('$d/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_prune_mfma' in r['Kernel_Name']:
            vals.setdefault(r['Counter_Name'],[]).append(float(r['Counter_Value']))
w=sum(vals['SQ_WAVE_CYCLES']); b=sum(vals['SQ_BUSY_CU_CYCLES'])
print('$v', 'resident waves per busy CU %.2f' % (4*w/b), 'waves', sum(vals['SQ_WAVES'])/len(vals['SQ_WAVES']))
"
done
