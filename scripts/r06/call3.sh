# r06 call 3: GPU suite on the DNA ballot-gated rescale build, DNA A/B (cfg2, cfg5), the
# default bench line with the write-ceiling probe
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
TAG=cfg2_dna_ballot CFG=cfg2 LIBS="new old" ROUNDS=3 bash scripts/r06/ab_libs.sh || exit 1
TAG=cfg5_dna_ballot CFG=cfg5 STEPS=20 LIBS="new old" ROUNDS=3 bash scripts/r06/ab_libs.sh || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); r=d['roofline']
print('default', d['value'], r['frac'], r.get('ceiling_GBps'), r.get('frac_of_ceiling'))"
