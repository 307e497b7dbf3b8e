# r06 call 27: cfg3 plan re-check on the final r06 kernel: split target n_ops / PU_SPLIT
# (default 3) and stash slots (PU_LDS_SLOTS, default 3), two rounds
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r06_call27; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for v in def s2 s4 s5 s6 l2; do
  unset PU_SPLIT PU_LDS_SLOTS
  case $v in s*) export PU_SPLIT=${v#s};; l*) export PU_LDS_SLOTS=${v#l};; esac
  timeout -k 10 300 python -u bench.py --config cfg3 --steps 200 --warmup 20 --no-cpu-baseline > $O/cfg3_$v.json 2> $O/cfg3_$v.err || { tail -20 $O/cfg3_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/cfg3_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'))"
done
done
