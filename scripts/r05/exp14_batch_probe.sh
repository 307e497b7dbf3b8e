# r05 exp14: batched vs own launches (scripts/r05/batch_probe.py), plus the streams bench with
# the generic build forced and without tip products (latency hypotheses for cfg5)
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp14
mkdir -p $O
timeout -k 10 300 python -u scripts/r05/batch_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
PU_FORCE_GENERIC=1 timeout -k 10 300 python -u scripts/r05/batch_probe.py --trees 1,8 > $O/probe_generic.txt 2>&1 || { tail -20 $O/probe_generic.txt; exit 1; }
cat $O/probe_generic.txt
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], 'value %.0f step %.4f kernel %.4f' % (d['value'], d['ms_per_step'], r['kernel_ms']))" "$1" "$2"; }
for v in "PU_BENCH_BATCH=0" "PU_BENCH_BATCH=0 PU_NO_PTIP=1" "PU_BENCH_BATCH=0 PU_FORCE_GENERIC=1"; do
  env $v timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  line $O/b.json "$v"
done
