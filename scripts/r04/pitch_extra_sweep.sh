# r04: one extra unused tile per layout row (libphylo_hip_p1.so, -DPU_PITCH_EXTRA=1) against
# the installed build over the default-plan sweep, the taxa sweep, cfg3 and cfg5
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/phylo_utils_amd
S=$(python -c "print(','.join(str(s) for s in sorted(set(list(range(50000, 300001, 12500)) + [131072]))))")
for lib in libphylo_hip.so libphylo_hip_p1.so; do
  PHYLO_HIP_LIB=$L/$lib timeout -k 10 900 python -u scripts/sweep.py --config cfg2 --sites "$S" \
    --steps 100 --rounds 3 --json gpurun_out/sweep_sites_$lib.json > gpurun_out/sweep_sites_$lib.txt 2>&1 || exit $?
  PHYLO_HIP_LIB=$L/$lib timeout -k 10 900 python -u scripts/sweep.py --config cfg2 --taxa 500,1000 \
    --sites 50000,100000,131072,200000,300000 --steps 50 --rounds 3 \
    --json gpurun_out/sweep_taxa_$lib.json > gpurun_out/sweep_taxa_$lib.txt 2>&1 || exit $?
done
for i in 1 2; do
  for lib in libphylo_hip.so libphylo_hip_p1.so; do
    for cfg in cfg3 cfg5; do
      PHYLO_HIP_LIB=$L/$lib timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 10 \
        --no-cpu-baseline > gpurun_out/ab_line.json 2> gpurun_out/ab_err.txt || exit $?
      python -c "
import json; d = json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1])
t = d.get('timing', {})
print('%-5s %-20s step %.5f ms  kernel %s  value %.1f' % ('$cfg', '$lib', d['ms_per_step'], t.get('kernel_ms_median'), d['value']))" | tee -a gpurun_out/ab_pitch2.txt
    done
  done
done
