#!/usr/bin/env python
"""gpurun_out/r06_mfma/<cfg>_pass*/ (scripts/r06/mfma_pmc.sh) -> profiles/r06_mfma_<cfg>.json:
per-launch means of the matrix-pipe counters of the protein traversal and the derived
fractions (MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES in cycles summed over SIMDs,
GRBM_GUI_ACTIVE in cycles summed over the 8 XCDs, SQ_WAVE_CYCLES in quad-cycles).

    python scripts/r06/mfma_collect.py --cfg cfg3 [--tag cfg3_ballot]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
N_SIMD, N_XCD = 1024, 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="cfg3")
    ap.add_argument("--tag", default=None)
    ap.add_argument("--kernel", default="k_prune_mfma")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "r06_mfma"))
    a = ap.parse_args()
    v = defaultdict(list)
    for p in sorted(glob.glob(os.path.join(a.src, a.cfg + "_pass*", "*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(p)):
            if a.kernel in r["Kernel_Name"]:
                v[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(x) / len(x) for k, x in v.items()}
    out = {"kernel": a.kernel, "config": a.cfg, "per_launch": m,
           "dispatches": {k: len(x) for k, x in v.items()}}
    xcd = m.get("GRBM_GUI_ACTIVE", 0.0) / N_XCD
    if xcd and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        busy = m["SQ_VALU_MFMA_BUSY_CYCLES"] / N_SIMD
        out["mfma_busy_cycles_per_simd"] = busy
        out["kernel_cycles_per_xcd"] = xcd
        out["mfma_pipe_busy_frac"] = busy / xcd
    if m.get("SQ_INSTS_VALU_MFMA_F64"):
        out["busy_cycles_per_mfma"] = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / m["SQ_INSTS_VALU_MFMA_F64"]
        out["wave_ops"] = m["SQ_INSTS_VALU_MFMA_F64"] / 20
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU"):
            if k in m:
                out[k.lower() + "_per_wave_op"] = m[k] / out["wave_ops"]
    if xcd and "SQ_WAVE_CYCLES" in m:
        out["resident_waves_per_simd"] = 4 * m["SQ_WAVE_CYCLES"] / (N_SIMD * xcd)
    out["units"] = ("SQ_VALU_MFMA_BUSY_CYCLES cycles summed over SIMDs; GRBM_GUI_ACTIVE cycles "
                    "summed over 8 XCDs; SQ_WAVE_CYCLES quad-cycles summed over waves")
    dst = os.path.join(ROOT, "profiles", "r06_mfma_%s.json" % (a.tag or a.cfg))
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: out[k] for k in out if k not in ("per_launch", "dispatches", "units")}))


if __name__ == "__main__":
    main()
