#!/usr/bin/env python
"""Turn a scripts/gpu_round.sh PROFILE=1 run (gpurun_out/prof_trace, prof_fetch, prof_write)
into the committed evidence under profiles/:

  profiles/<round>_<cfg>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<round>_traffic_<cfg>.json       HBM bytes per k_prune launch from the PMC passes

    python scripts/collect_profiles.py --round r01 --config cfg2

HBM bytes follow the guide's gfx950 rules: FETCH_SIZE and WRITE_SIZE are in KiB,
FETCH_SIZE counts half the bytes of wide streaming reads (doubled here), WRITE_SIZE is exact
for 16-byte-per-lane stores (the CLV stores are dbl2 per lane).
"""
import argparse
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(root, counter, kernel):
    """Counter per traversal: the mean over dispatches of each kernel whose name contains
    `kernel`, summed over those kernels (a split protein traversal is two launches, the chain
    tasks and the top task, named apart by their template arguments).  Returned as a list of
    per-dispatch-set values (one entry per dispatch of the most frequent kernel) so that the
    callers' len() still counts dispatches."""
    vals = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if kernel in name and row["Counter_Name"] == counter:
                key = (name, f, row["Dispatch_Id"])
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    by_name = {}
    for (name, _, _), v in vals.items():
        by_name.setdefault(name, []).append(v)
    if not by_name:
        return []
    total = sum(sum(v) / len(v) for v in by_name.values())
    n = max(len(v) for v in by_name.values())
    return [total] * n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r01")
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--suffix", default="", help="e.g. _lnl for a PU_LNL_ONLY profile")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--kernel", default="k_prune")
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    tag = "%s%s" % (a.config, a.suffix)
    stats = glob.glob(os.path.join(a.src, "prof_trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        dst = os.path.join(ROOT, "profiles", "%s_%s_kernel_stats.csv" % (a.round, tag))
        shutil.copy(stats[0], dst)
        print("wrote", dst)
        for row in csv.DictReader(open(stats[0])):
            if a.kernel in row["Name"]:
                print("  %s calls %s avg %.1f us" % (row["Name"][:60], row["Calls"],
                                                    float(row["AverageNs"]) / 1e3))
    fetch = per_dispatch(os.path.join(a.src, "prof_fetch"), "FETCH_SIZE", a.kernel)
    write = per_dispatch(os.path.join(a.src, "prof_write"), "WRITE_SIZE", a.kernel)
    if fetch and write:
        f_kb = sum(fetch) / len(fetch)
        w_kb = sum(write) / len(write)
        out = {"kernel": a.kernel, "config": a.config, "mode": a.suffix.strip("_") or "keep",
               "dispatches": [len(fetch), len(write)],
               "fetch_size_kib": f_kb, "write_size_kib": w_kb,
               "fetch_bytes": 2 * f_kb * 1024, "write_bytes": w_kb * 1024,
               "hbm_bytes_per_launch": 2 * f_kb * 1024 + w_kb * 1024,
               "rule": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM)"}
        dst = os.path.join(ROOT, "profiles", "%s_traffic_%s.json" % (a.round, tag))
        json.dump(out, open(dst, "w"), indent=1)
        print("wrote", dst, "hbm bytes/launch %.1f MB" % (out["hbm_bytes_per_launch"] / 1e6))
    ins = {c: per_dispatch(os.path.join(a.src, "prof_insts"), c, a.kernel)
           for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS",
                     "SQ_WAVES", "SQ_BUSY_CU_CYCLES")}
    if all(ins.values()):
        # per launch (mean over dispatches); bench.py's latest_pmc reads this file
        out = {c: sum(v) / len(v) for c, v in ins.items()}
        out.update({"kernel": a.kernel, "config": a.config, "dispatches": len(ins["SQ_WAVES"]),
                    "unit": "wave-instructions per launch; SQ_BUSY_CU_CYCLES summed over CUs"})
        dst = os.path.join(ROOT, "profiles", "%s_pmc_%s.json" % (a.round, tag))
        json.dump(out, open(dst, "w"), indent=1)
        print("wrote", dst)


if __name__ == "__main__":
    main()
