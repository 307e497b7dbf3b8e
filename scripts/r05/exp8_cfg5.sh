# r05 exp8: counter names; cfg5 bench with the default build vs the 7-wave lnL-only build
# (alternating); the single-tree k_pmatrix A/B for cfg3 (PU_PMAT_AA_WAVE)
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/exp8
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config cfg5 --steps 10 --warmup 3 > $O/cfg5_def_$r.json 2> $O/cfg5_def_$r.err || exit 1
  PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_w7.so timeout -k 10 300 python -u bench.py --config cfg5 --steps 10 --warmup 3 > $O/cfg5_w7_$r.json 2> $O/cfg5_w7_$r.err || exit 1
done
for f in $O/cfg5_*.json; do python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'])"; done
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config cfg3 --steps 20 --warmup 5 > $O/cfg3_def_$r.json 2> $O/cfg3_def_$r.err || exit 1
  PU_PMAT_AA_WAVE=1 timeout -k 10 300 python -u bench.py --config cfg3 --steps 20 --warmup 5 > $O/cfg3_wave_$r.json 2> $O/cfg3_wave_$r.err || exit 1
done
for f in $O/cfg3_*.json; do python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);t=d['timing'];print('$f',d['value'],d['ms_per_step'],t['step_ms_median'],t['kernel_ms_median'],d['lnl'])"; done
grep -o "SQ_[A-Z0-9_]*" $O/counters.txt | sort -u | tr '\n' ' ' | head -c 5000
# one lnL-only tree over more sites fills the GPU in one launch: the throughput a batched
# multi-tree launch could reach (default build and the 7-wave build)
timeout -k 10 300 python -u scripts/sweep.py --config cfg5 --lnl-only --sites 50000,100000,200000,400000 --steps 50 --rounds 2 > $O/cfg5_sites.txt 2>&1 || exit 1
PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_w7.so timeout -k 10 300 python -u scripts/sweep.py --config cfg5 --lnl-only --sites 50000,100000,200000,400000 --steps 50 --rounds 2 > $O/cfg5_sites_w7.txt 2>&1 || exit 1
grep -h "traverse\|^config" $O/cfg5_sites*.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "deviation_is_the_pmatrix or padded_tile_pitch" -s > $O/deviation.log 2>&1 || { tail -30 $O/deviation.log; exit 1; }
grep "partials vs\|passed\|failed" $O/deviation.log
