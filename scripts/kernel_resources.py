#!/usr/bin/env python
"""Per-kernel resources from a gfx950 assembly listing (hipcc --offload-device-only -S):
private segment bytes, VGPRs, SGPRs and scratch / flat instruction counts.

    python scripts/kernel_resources.py phylo_utils_amd/csrc/_obj/pu_kernels.s [name-filter]
"""
import re
import sys


def kernels(text):
    out = {}
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", text, re.S):
        name, body = m.group(1), m.group(2)

        def get(k):
            r = re.search(r"\.amdhsa_%s (\d+)" % k, body)
            return int(r.group(1)) if r else -1
        out[name] = {"private": get("private_segment_fixed_size"),
                     "vgpr": get("next_free_vgpr"), "sgpr": get("next_free_sgpr")}
    for name in out:
        m = re.search(r"^%s:.*?\n(.*?)s_endpgm" % re.escape(name), text, re.S | re.M)
        body = m.group(1) if m else ""
        out[name]["scratch_insts"] = len(re.findall(r"^\s*scratch_", body, re.M))
        out[name]["flat_insts"] = len(re.findall(r"^\s*flat_", body, re.M))
    return out


def main():
    text = open(sys.argv[1]).read()
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, r in sorted(kernels(text).items()):
        if filt in name:
            print("%4d %4d %4d %4d %4d %s" % (r["private"], r["vgpr"], r["sgpr"],
                                               r["scratch_insts"], r["flat_insts"], name))


if __name__ == "__main__":
    main()
