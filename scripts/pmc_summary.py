#!/usr/bin/env python
"""Summarise rocprofv3 --pmc CSVs for the traversal kernel: mean counter value per launch.

    python scripts/pmc_summary.py gpurun_out/pmc_keep [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "k_traverse"
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(float)
        for row in csv.DictReader(open(f)):
            if pat not in row.get("Kernel_Name", ""):
                continue
            per[(row["Counter_Name"], row["Dispatch_Id"])] += float(row["Counter_Value"])
        for (name, _), v in per.items():
            vals[name].append(v)
    for name in sorted(vals):
        v = vals[name]
        print("%-28s %16.1f  (n=%d)" % (name, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main()
