#!/usr/bin/env python
"""Instruction mix of one kernel in a `make asm` listing (static counts, whole kernel).

    python scripts/isa_mix.py <file.s> <mangled-name-substring> [...]
"""
import sys
from collections import Counter


def kernel_text(path, name):
    s = open(path).read()
    for line in s.split("\n"):
        head = line.split(";")[0].strip()
        if head.endswith(":") and name in head and not head.startswith("."):
            lab = line
            break
    else:
        raise SystemExit("no kernel matching %s in %s" % (name, path))
    i = s.index("\n" + lab + "\n")
    j = s.index(".Lfunc_end", i)
    return lab, s[i:j]


def classify(op):
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op in ("v_readlane_b32", "v_writelane_b32"):
        return "lane_spill"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return op


for name in sys.argv[2:]:
    lab, text = kernel_text(sys.argv[1], name)
    ops = [l.split()[0] for l in (x.strip() for x in text.split("\n"))
           if l and not l.startswith((".", ";", "_")) and not l.endswith(":")]
    c = Counter(classify(o) for o in ops)
    print("%s  total %d  %s" % (lab[:70], len(ops), dict(c.most_common())))
