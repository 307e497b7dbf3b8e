# r05 exp12: the multi-tree launch (pu_batch) -- its GPU tests, cfg5 batched vs per-tree
# streams, and an A/B of the prune_tree refactor (HEAD build vs this build) on cfg2 / cfg5
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp12
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_batch.py > $O/batch_tests.txt 2>&1 || { tail -40 $O/batch_tests.txt; exit 1; }
grep -E "passed|failed" $O/batch_tests.txt | tail -3
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[2], 'value %.0f step %.4f kernel %.4f' % (d['value'], d['ms_per_step'], r['kernel_ms']), d['config'].get('launch',''), 'maxrel', d.get('lnl_max_rel_diff_vs_sync_runs'))" "$1" "$2"; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $O/cfg5_batch_$i.json 2> $O/cfg5_batch_$i.err || { tail -20 $O/cfg5_batch_$i.err; exit 1; }
  line $O/cfg5_batch_$i.json "cfg5 batch"
  PU_BENCH_BATCH=0 timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $O/cfg5_streams_$i.json 2> $O/cfg5_streams_$i.err || { tail -20 $O/cfg5_streams_$i.err; exit 1; }
  line $O/cfg5_streams_$i.json "cfg5 streams"
  PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_head.so PU_BENCH_BATCH=0 timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > $O/cfg5_head_$i.json 2> $O/cfg5_head_$i.err || { tail -20 $O/cfg5_head_$i.err; exit 1; }
  line $O/cfg5_head_$i.json "cfg5 HEAD streams"
  timeout -k 10 300 python -u bench.py --config cfg2 --no-cpu-baseline > $O/cfg2_new_$i.json 2> $O/cfg2_new_$i.err || { tail -20 $O/cfg2_new_$i.err; exit 1; }
  line $O/cfg2_new_$i.json "cfg2 new"
  PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_head.so timeout -k 10 300 python -u bench.py --config cfg2 --no-cpu-baseline > $O/cfg2_head_$i.json 2> $O/cfg2_head_$i.err || { tail -20 $O/cfg2_head_$i.err; exit 1; }
  line $O/cfg2_head_$i.json "cfg2 HEAD"
done
