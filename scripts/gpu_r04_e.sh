# r04: GPU tests, protein chunk size / stash slots, then the committed profiles of every config
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/sweep.py --config cfg3 --steps 100 --rounds 3 \
  --grid 'PU_CHUNK_USES:PU_LDS_SLOTS=:,16:,64:,128:,:2,:4' > gpurun_out/r04_cfg3_chunks.txt 2>&1 || exit $?
grep -v "amdgpu.ids" gpurun_out/r04_cfg3_chunks.txt
bash scripts/gpu_r04_prof.sh
