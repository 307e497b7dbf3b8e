# r04: the pair kernel (lnL-only DNA) -- parity, then cfg5 single tree and bench (pair / split)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pair.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_pair.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/sweep.py --config cfg5 --lnl-only --steps 200 --rounds 3 \
  --grid 'PU_NO_PAIR:PU_SPLIT=1:,:,1:3,:3,:2,:4' > gpurun_out/r04_cfg5_split.txt 2>&1 || exit $?
cat gpurun_out/r04_cfg5_split.txt
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline \
  > gpurun_out/r04_cfg5_bench.json 2> gpurun_out/r04_cfg5_bench.err || exit $?
PU_NO_PAIR=1 timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline \
  > gpurun_out/r04_cfg5_bench_nopair.json 2> gpurun_out/r04_cfg5_bench_nopair.err || exit $?
PU_SPLIT=3 timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline \
  > gpurun_out/r04_cfg5_bench_split3.json 2> gpurun_out/r04_cfg5_bench_split3.err || exit $?
python - <<'PY'
import json
for s in ("", "_nopair", "_split3"):
    d = json.load(open("gpurun_out/r04_cfg5_bench%s.json" % s))
    print("cfg5 bench%-8s" % s, d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"],
          d["lnl_max_rel_diff_vs_sync_runs"])
PY
