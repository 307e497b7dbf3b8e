# r06 call 1: GPU suite on the round-5 head, then the protein matrix-pipe counters
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
bash scripts/r06/mfma_pmc.sh
for c in cfg5 default; do
  a=""; [ $c != default ] && a="--config $c"
  timeout -k 10 600 python -u bench.py $a > $O/bench_${c}.json 2> $O/bench_${c}.err || { tail -20 $O/bench_${c}.err; exit 1; }
  tail -c 600 $O/bench_${c}.json
done
