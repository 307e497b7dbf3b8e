# r04: per-op phase cycles of one protein wave (timing build, s_memtime; the unsplit plan, whose
# workgroup 0 runs the whole post-order), cfg3 KEEP and lnL-only, plus the same plans untimed
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/phylo_utils_amd
for args in "" "--lnl-only"; do
  PHYLO_HIP_LIB=$L/libphylo_hip_timing.so PU_TIMING=1 PU_SPLIT=1 timeout -k 10 300 \
    python bench.py --config cfg3 --steps 50 --warmup 5 --no-cpu-baseline $args \
    > gpurun_out/timing.json 2> gpurun_out/timing.txt || exit $?
  echo "cfg3 $args: $(grep 'pu timing' gpurun_out/timing.txt | tail -1)" | tee -a gpurun_out/protein_timing.txt
  PU_SPLIT=1 timeout -k 10 300 python bench.py --config cfg3 --steps 200 --warmup 20 --no-cpu-baseline $args \
    > gpurun_out/ab_line.json 2> /dev/null || exit $?
  python -c "
import json; d = json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1])
print('cfg3 $args unsplit, untimed build: kernel %s ms' % d.get('timing', {}).get('kernel_ms_median'))" | tee -a gpurun_out/protein_timing.txt
done
