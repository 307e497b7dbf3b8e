# r05 exp45: the unpack with 16-word slices as the only unpack path -- pattern tests and
# three bench lines
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp45
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_patterns.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload patterns --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('kernel %.4f ms  step %.4f ms  %.1f M columns/s' % (d['roofline']['kernel_ms'], d['ms_per_step'], d['value']))"
done
