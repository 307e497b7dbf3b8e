# r05 exp39: cfg3 with smaller tip-code staging chunks (PU_CHUNK_USES), so that 3 stash slots
# fit 4 protein workgroups per CU (LDS: the code table + the chunk's codes + 36 KB of stash
# must stay under 40 KB) -- bench lines alternating with the default, and the LDS size of
# each from a kernel trace
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp39
rm -rf $O; mkdir -p $O
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); t=d.get('timing',{})
print(sys.argv[2], 'step %.4f ms  kernel median %s  value %.2f' % (d['ms_per_step'], t.get('kernel_ms_median'), d['value']/1e3))" "$1" "$2"; }
for i in 1 2; do
  for v in "PU_DUMMY=1" "PU_CHUNK_USES=8" "PU_CHUNK_USES=4" "PU_CHUNK_USES=12"; do
    env $v timeout -k 10 300 python -u bench.py --config cfg3 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"
  done
done
for v in "PU_DUMMY=1" "PU_CHUNK_USES=8"; do
  d=$O/trace_${v%%=*}
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -- python bench.py --config cfg3 --steps 5 --warmup 2 --no-cpu-baseline > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python -c "
import csv,glob
f=glob.glob('$d/**/*kernel_trace.csv', recursive=True)[0]
rows=[r for r in csv.DictReader(open(f)) if 'k_prune_mfma' in r['Kernel_Name']]
r=rows[-1]; print('$v', 'LDS', r['LDS_Block_Size'], 'VGPR', r['VGPR_Count'], 'grid', r['Grid_Size_X'], 'ms', (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6)
"
done
