# r05: list the SQ / TCC / TA counters of this gfx950 rocprofv3 (names for the stall passes)
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/exp8
timeout -k 10 120 rocprofv3 -L > gpurun_out/exp8/counters.txt 2>&1 || timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/exp8/counters.txt 2>&1
grep -o "SQ_[A-Z0-9_]*" gpurun_out/exp8/counters.txt | sort -u | tr '\n' ' ' | head -c 6000
