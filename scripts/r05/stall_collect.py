#!/usr/bin/env python
"""gpurun_out/stall_<tag>/pass*/ (scripts/r05/stall_pmc.sh) -> profiles/<round>_stall_<tag>.json:
per-launch means of each SQ counter for the traversal kernel and the wave-cycle attribution
(MI355X_MICROARCH.md, rocprofv3 PMC slots: SQ_WAIT_ANY = parked on s_waitcnt / barrier,
SQ_WAIT_INST_ANY = ready but not issued, SQ_ACTIVE_INST_ANY = issuing; disjoint, summing to
about SQ_WAVE_CYCLES; all in quad-cycles).

    python scripts/r05/stall_collect.py --round r05 --tag cfg5_lnl
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from collect_profiles import per_dispatch  # noqa: E402

COUNTERS = ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_WAIT_INST_LDS", "SQ_INSTS_SMEM", "SQ_INST_LEVEL_SMEM", "SQ_WAVES",
            "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM",
            "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM",
            "SQ_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
            "SQ_INST_CYCLES_SMEM", "SQ_INST_CYCLES_VMEM_WR", "SQ_INST_CYCLES_VMEM_RD",
            "SQ_BUSY_CU_CYCLES", "SQ_INSTS_VMEM_WR"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r05")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kernel", default="k_prune")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    a = ap.parse_args()
    src = os.path.join(a.src, "stall_" + a.tag)
    v, n = {}, {}
    for c in COUNTERS:
        d = per_dispatch(src, c, a.kernel)
        if d:
            v[c] = sum(d) / len(d)
            n[c] = len(d)
    wc = v.get("SQ_WAVE_CYCLES", 0.0)
    out = {"kernel": a.kernel, "tag": a.tag, "per_launch": v, "dispatches": n,
           "units": "SQ_*_CYCLES, SQ_WAIT_*, SQ_ACTIVE_* in quad-cycles summed over waves; "
                    "SQ_INSTS_* wave-instructions; SQ_INST_LEVEL_* summed in-flight count"}
    if wc:
        parts = {k: v.get(k, 0.0) / wc for k in
                 ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
        out["wave_cycle_fractions"] = parts
        out["attributed"] = sum(parts.values())
        out["active_breakdown_of_wave_cycles"] = {
            k: v.get(k, 0.0) / wc for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
                                            "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS",
                                            "SQ_ACTIVE_INST_MISC")}
        out["wait_inst_lds_of_wave_cycles"] = v.get("SQ_WAIT_INST_LDS", 0.0) / wc
        if v.get("SQ_WAVES"):
            out["quad_cycles_per_wave"] = wc / v["SQ_WAVES"]
    if v.get("SQ_INSTS_SMEM"):
        out["smem_level_per_inst"] = v.get("SQ_INST_LEVEL_SMEM", 0.0) / v["SQ_INSTS_SMEM"]
    if v.get("SQ_INSTS_VMEM"):
        out["vmem_level_per_inst"] = v.get("SQ_INST_LEVEL_VMEM", 0.0) / v["SQ_INSTS_VMEM"]
    dst = os.path.join(ROOT, "profiles", "%s_stall_%s.json" % (a.round, a.tag))
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: out[k] for k in out if k not in ("per_launch", "dispatches")}, indent=1))
    print("wrote", dst)


if __name__ == "__main__":
    main()
