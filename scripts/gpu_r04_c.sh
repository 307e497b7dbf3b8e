# r04: lnL-only split plans for under-filled grids (cfg5), single tree and the 125-tree bench
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/sweep.py --config cfg5 --lnl-only --steps 200 --rounds 3 \
  --grid 'PU_SPLIT=,2,3,4,6' > gpurun_out/r04_cfg5_split.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline \
  > gpurun_out/r04_cfg5_bench_split.json 2> gpurun_out/r04_cfg5_bench_split.err || exit $?
PU_SPLIT=3 timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline \
  > gpurun_out/r04_cfg5_bench_split3.json 2> gpurun_out/r04_cfg5_bench_split3.err || exit $?
cat gpurun_out/r04_cfg5_split.txt
python - <<'PY'
import json
for s in ("", "3"):
    d = json.load(open("gpurun_out/r04_cfg5_bench_split%s.json" % s))
    print("split", s or "-", d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])
PY
