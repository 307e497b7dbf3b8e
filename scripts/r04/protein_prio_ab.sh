# r04: static wave priority for every other protein workgroup (-DPU_AA_PRIO), cfg3 A/B
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/phylo_utils_amd
PHYLO_HIP_LIB=$L/libphylo_hip_prio.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "protein or cfg3" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_prio.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_prio.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for lib in libphylo_hip.so libphylo_hip_prio.so; do
    PHYLO_HIP_LIB=$L/$lib timeout -k 10 300 python bench.py --config cfg3 --steps 200 --warmup 20 \
      --no-cpu-baseline > gpurun_out/ab_line.json 2> /dev/null || exit $?
    python -c "
import json; d = json.loads(open('gpurun_out/ab_line.json').read().strip().splitlines()[-1])
t = d.get('timing', {})
print('cfg3 %-22s step %.5f ms  kernel %.5f ms  lnl %r' % ('$lib', d['ms_per_step'], t.get('kernel_ms_median'), d.get('lnl')))" | tee -a gpurun_out/ab_prio.txt
  done
done
