# r06 call 13: where the host-to-host time of pu_optimise_edge goes (entry/launch/result/drain
# stamps, raw back-to-back calls), cooperative vs ordinary launch of the co-resident grid
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call13; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/r06/newton_probe.py > $O/newton_probe.log 2>&1 || { tail -30 $O/newton_probe.log; exit 1; }
grep -v amdgpu.ids $O/newton_probe.log
for p in 0 1; do
PU_NT_PLAIN=$p timeout -k 10 300 python -u bench.py --workload edges > $O/bench_edges_plain$p.json 2> $O/bench_edges_plain$p.err || { tail -20 $O/bench_edges_plain$p.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_edges_plain$p.json').read().strip().splitlines()[-1])
print('plain $p', json.dumps({k: d[k] for k in ('value','device_newton','sweep')}))"
done
