# r05 exp4: GPU suite on the build (pattern weight preloaded, register stash in registers, pair
# kernel gone), then a same-box sweep against the r04 library and a cfg2 bench line
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp4
mkdir -p $O
bash scripts/gpu_tests.sh > $O/tests.txt 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 $O/tests.txt
for r in 1 2; do
  PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_r04.so timeout -k 10 300 python -u scripts/sweep.py --config cfg2 --sites 75000,87500,100000,112500 --steps 200 --rounds 3 > $O/sweep_r04_$r.txt 2>&1 || exit 1
  timeout -k 10 300 python -u scripts/sweep.py --config cfg2 --sites 75000,87500,100000,112500 --steps 200 --rounds 3 > $O/sweep_new_$r.txt 2>&1 || exit 1
done
grep -h "traverse" $O/sweep_*.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit 1
python -c "import json;d=json.loads(open('$O/bench_cfg2.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['kernel_ms'])"
