set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
for i in 1 2; do
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/b_cfg2_new_$i.json 2>gpurun_out/b_err.log
PU_PMAT_BLOCK=1 timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/b_cfg2_old_$i.json 2>>gpurun_out/b_err.log
timeout -k 10 120 python bench.py --config cfg3 --no-cpu-baseline > gpurun_out/b_cfg3_new_$i.json 2>>gpurun_out/b_err.log
PU_PMAT_BLOCK=1 timeout -k 10 120 python bench.py --config cfg3 --no-cpu-baseline > gpurun_out/b_cfg3_old_$i.json 2>>gpurun_out/b_err.log
done
