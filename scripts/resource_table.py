#!/usr/bin/env python
"""Per-kernel register / spill table from `make -C phylo_utils_amd/csrc asm` remarks.

    python scripts/resource_table.py [filter]
"""
import re
import subprocess
import sys

path = "phylo_utils_amd/csrc/_obj/resource.txt"
flt = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = {}, None
for line in open(path):
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([^:]+): (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
names = list(rows)
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                     text=True).stdout.split("\n")
keys = ["TotalSGPRs", "VGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
        "SGPRs Spill", "VGPRs Spill"]
print("%-44s %5s %5s %7s %4s %6s %6s" % ("kernel", "SGPR", "VGPR", "scratch", "occ",
                                         "Sspill", "Vspill"))
for n, d in zip(names, dem):
    d = d.replace("(anonymous namespace)::", "").replace("pu::", "")
    d = d.replace("(TraverseArgs)", "").replace("void ", "")
    if flt not in d:
        continue
    r = rows[n]
    print("%-44s %5s %5s %7s %4s %6s %6s" % ((d[:44],) + tuple(r.get(k, "-") for k in keys)))
