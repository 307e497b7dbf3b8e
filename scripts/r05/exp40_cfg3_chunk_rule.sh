# r05 exp40: the protein chunk rule (largest tip-use target >= 8 that fits 4 workgroups per
# CU) -- the GPU suite, then cfg3 bench lines alternating with the old 32-use target
# (PU_CHUNK_USES=32) and a kernel trace of the default
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp40
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
line() { python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); t=d.get('timing',{})
print(sys.argv[2], 'step %.4f ms  kernel median %s  value %.2f  frac %s' % (d['ms_per_step'], t.get('kernel_ms_median'), d['value']/1e3, d['roofline']['frac']))" "$1" "$2"; }
for i in 1 2 3; do
  for v in "PU_DUMMY=1" "PU_CHUNK_USES=32"; do
    env $v timeout -k 10 300 python -u bench.py --config cfg3 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    line $O/b.json "$v"
  done
done
