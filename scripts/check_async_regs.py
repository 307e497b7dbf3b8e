#!/usr/bin/env python3
"""Check that no instruction touches the destination VGPRs of an in-flight vector load.

The protein kernel (k_prune_mfma, pu_kernels.hip) issues its P prefetches as inline-asm
global loads and waits for them with counted `s_waitcnt vmcnt(N)`: the compiler does not
know the registers are written asynchronously, so a register copy it schedules between a
load and its wait (e.g. a phi copy at the top of the next loop iteration) would copy stale
data.

This is a forward dataflow analysis over the kernel's control-flow graph.  For every
inline-asm load still possibly outstanding it keeps the MINIMUM, over all paths, of the
number of vector-memory operations (loads and stores, the compiler's and the asm's) issued
after it; vector-memory operations retire in issue order on gfx950, so `s_waitcnt vmcnt(N)`
retires exactly the loads with at least N younger operations.  Merges take the union of
pending loads with the smaller count; the analysis iterates to a fixed point and then
reports every instruction that reads or writes a register of a possibly pending asm load.
(The compiler waits for its own loads itself; they only count as younger operations.)

  hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -simplifycfg-sink-common=false \\
        -S --cuda-device-only phylo_utils_amd/csrc/pu_kernels.hip -o /tmp/k.s
  python scripts/check_async_regs.py /tmp/k.s k_prune_mfma
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
CAP = 256  # younger-operation counts saturate here (any real wait count is smaller)


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return frozenset(out)


def functions(lines, name):
    cur, body = None, []
    for ln in lines:
        if re.match(r"^_Z\S*:\s*(;.*)?$", ln):
            cur, body = ln.split(":")[0], []
        elif cur is not None:
            body.append(ln)
            if "s_endpgm" in ln:
                if name in cur:
                    yield cur, body
                cur = None


def parse(body):
    """Instructions [(kind, text, regs, extra)] and basic blocks with successors."""
    insts, labels, starts = [], {}, {0}
    in_asm = False
    for raw in body:
        s = raw.strip()
        if "#ASMSTART" in s or "#ASMEND" in s:
            in_asm = "#ASMSTART" in s
            continue
        m = re.match(r"^(\.LBB\w+):", s)
        if m:
            labels[m.group(1)] = len(insts)
            starts.add(len(insts))
            continue
        ln = s.split(";")[0].strip()
        if not ln or ln.startswith("."):
            continue
        op = ln.split()[0]
        operands = ln[len(op):]
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", ln)
            insts.append(("wait", ln, frozenset(), int(m.group(1)) if m else None))
        elif op.startswith(("global_load", "buffer_load", "flat_load")):
            parts = operands.split(",")
            insts.append(("load", ln, regs(operands), (regs(parts[0]), in_asm)))
        elif op.startswith(("global_store", "buffer_store", "flat_store", "global_atomic")):
            insts.append(("store", ln, regs(operands), None))
        elif op == "s_branch" or op.startswith("s_cbranch"):
            insts.append(("branch", ln, frozenset(), (op, operands.strip())))
            starts.add(len(insts))
        elif op == "s_endpgm":
            insts.append(("end", ln, frozenset(), None))
            starts.add(len(insts))
        else:
            insts.append(("inst", ln, regs(operands), None))
    starts = sorted(s for s in starts if s < len(insts))
    blocks = [(a, b) for a, b in zip(starts, starts[1:] + [len(insts)]) if a < b]
    block_of = {a: k for k, (a, b) in enumerate(blocks)}
    succ = []
    for k, (a, b) in enumerate(blocks):
        kind, _, _, extra = insts[b - 1]
        nxt = [k + 1] if k + 1 < len(blocks) else []
        if kind == "branch":
            op, target = extra
            t = block_of.get(labels.get(target, -1))
            tgt = [t] if t is not None else []
            succ.append(tgt if op == "s_branch" else tgt + nxt)
        elif kind == "end":
            succ.append([])
        else:
            succ.append(nxt)
    return insts, blocks, succ


def step(state, inst, idx, dst, problems=None):
    """state: {asm load index: min younger operations}; the state after inst."""
    kind, text, rs, extra = inst
    if problems is not None and kind != "wait":
        pending = set()
        for li in state:
            pending |= dst[li]
        bad = rs & pending
        if bad:
            srcs = [li for li in state if dst[li] & bad]
            problems.append((text, sorted(bad), idx, srcs))
    if kind == "wait":
        if extra is None:
            return state
        return {li: c for li, c in state.items() if c < extra}
    if kind in ("load", "store"):
        st = {li: min(c + 1, CAP) for li, c in state.items()}
        if kind == "load" and extra[1]:  # inline-asm load: tracked
            dst[idx] = extra[0]
            st[idx] = 0
        return st
    return state


def merge(a, b):
    out = dict(a)
    for li, c in b.items():
        out[li] = min(c, out.get(li, CAP))
    return out


def check(body):
    insts, blocks, succ = parse(body)
    dst = {}
    entry = [None] * len(blocks)
    entry[0] = {}
    work = [0]
    while work:
        k = work.pop()
        st = entry[k]
        a, b = blocks[k]
        for i in range(a, b):
            st = step(st, insts[i], i, dst)
        for s in succ[k]:
            m = st if entry[s] is None else merge(entry[s], st)
            if m != entry[s]:
                entry[s] = m
                work.append(s)
    problems = []
    for k, (a, b) in enumerate(blocks):
        if entry[k] is None:
            continue
        st = entry[k]
        for i in range(a, b):
            st = step(st, insts[i], i, dst, problems)
    return problems


def main():
    path, name = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_prune_mfma"
    lines = open(path).read().splitlines()
    n_bad, n_fn = 0, 0
    for fn, body in functions(lines, name):
        probs = check(body)
        n_fn += 1
        print(f"{fn}: {len(probs)} hazard(s)")
        for txt, r, idx, srcs in probs[:12]:
            print(f"   {txt}   (in-flight v{r}; inst {idx}, loads {srcs})")
        n_bad += len(probs)
    sys.exit(1 if n_bad or not n_fn else 0)


if __name__ == "__main__":
    main()
