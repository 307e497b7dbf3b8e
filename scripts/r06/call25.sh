# r06 call 25: device Newton with 2 tiles per wave (half the workgroups, half the slots to
# gather) against 1 (PU_NT_TPW), edges bench lines alternating, stamps from the probe
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call25; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for t in 1 2; do
  PU_NT_TPW=$t timeout -k 10 300 python -u bench.py --workload edges > $O/edges_t$t.json 2> $O/edges_t$t.err || { tail -20 $O/edges_t$t.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/edges_t$t.json').read().strip().splitlines()[-1])
print('tpw=$t', d['device_newton']['us_per_evaluation'], d['device_newton']['us_per_optimisation'], d['sweep']['ms'])"
done
done
PU_NT_TPW=2 timeout -k 10 300 python -u scripts/r06/newton_probe.py > $O/probe_t2.log 2>&1 || { tail -30 $O/probe_t2.log; exit 1; }
grep "ev 1\|grid" $O/probe_t2.log | head -4
