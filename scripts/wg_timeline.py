#!/usr/bin/env python
"""Per-workgroup timeline of k_prune (diagnostic build, r05).

    make -C phylo_utils_amd/csrc ab VARIANT=stamps FLAGS=-DPU_WG_STAMPS
    PHYLO_HIP_LIB=phylo_utils_amd/libphylo_hip_stamps.so \
        python scripts/wg_timeline.py --sites 62500,100000,131072 --taxa 50 --out gpurun_out/tl

The stamps build records, per workgroup, s_memrealtime (100 MHz) at entry, at the start of
its first op, after its op loop and at exit, plus HW_ID / XCC_ID.  This script runs a few
warm traversals, then `--launches` stamped ones per size, and prints for each launch: the
span, the workgroup lifetimes of the first dispatch round and of the rest, how many
workgroups are resident over time and the CLV bytes written per microsecond of that
occupancy (a workgroup writes its (n_ops + 1) x 8 KB evenly over its op loop).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import CONFIGS, make_model  # noqa: E402


def load(path):
    raw = np.fromfile(path, dtype=np.uint64)
    out, i = [], 0
    while i < raw.size:
        grid, n_tiles, n_ops, S = (int(x) for x in raw[i:i + 4])
        w = raw[i + 4:i + 4 + 8 * grid].reshape(grid, 8).astype(np.int64)
        out.append(dict(grid=grid, n_tiles=n_tiles, n_ops=n_ops, S=S, w=w))
        i += 4 + 8 * grid
    return out


def analyse(L, bytes_per_wg):
    w = L["w"]
    t0 = w[:, 0].min()
    beg, ops, loop, end = ((w[:, k] - t0) / 100.0 for k in range(4))  # microseconds
    hw, xcc = w[:, 4], w[:, 5]
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    cu_key = (xcc & 0xF) * 1000 + se * 100 + sh * 50 + cu
    n_cu = len(np.unique(cu_key))
    span = end.max()
    life = end - beg
    grid = L["grid"]
    order = np.argsort(beg, kind="stable")
    # first dispatch round: workgroups that started before the first one ended
    first_end = end.min()
    r1 = beg < first_end
    lines = []
    lines.append("grid %d  n_ops %d  S %d  CUs seen %d  span %.2f us" %
                 (grid, L["n_ops"], L["S"], n_cu, span))
    per_cu = np.bincount(np.unique(cu_key, return_inverse=True)[1])
    lines.append("  workgroups per CU: min %d max %d mean %.2f" %
                 (per_cu.min(), per_cu.max(), per_cu.mean()))
    lines.append("  first round: %d workgroups (%.2f per CU), lifetime %.2f..%.2f us "
                 "(median %.2f), staging %.2f us median, epilogue %.2f us median" %
                 (r1.sum(), r1.sum() / max(n_cu, 1), life[r1].min(), life[r1].max(),
                  np.median(life[r1]), np.median((ops - beg)[r1]), np.median((end - loop)[r1])))
    if (~r1).any():
        lines.append("  later: %d workgroups, start %.2f..%.2f us, lifetime %.2f..%.2f "
                     "(median %.2f)" % ((~r1).sum(), beg[~r1].min(), beg[~r1].max(),
                                        life[~r1].min(), life[~r1].max(),
                                        np.median(life[~r1])))
    # resident workgroups and the write rate over time (1 us bins)
    nb = int(np.ceil(span)) + 1
    res = np.zeros(nb)
    wr = np.zeros(nb)
    for b_, o_, l_, e_ in zip(beg, ops, loop, end):
        i0, i1 = int(b_), int(e_)
        res[i0:i1 + 1] += 1
        if l_ > o_:
            rate = bytes_per_wg / (l_ - o_)
            j0, j1 = int(o_), int(l_)
            wr[j0:j1 + 1] += rate
    lines.append("  time(us)  resident  est.write TB/s")
    step = max(1, nb // 24)
    for i in range(0, nb, step):
        lines.append("  %7.1f  %8.0f  %6.2f" % (i, res[i:i + step].mean(),
                                             wr[i:i + step].mean() / 1e6))
    lines.append("  total bytes %.1f MB over span -> %.2f TB/s" %
                 (bytes_per_wg * grid / 1e6, bytes_per_wg * grid / span / 1e6))
    # when does the grid drain: time from the 90th percentile end to the last end
    q = np.percentile(end, [50, 90, 99, 100])
    lines.append("  end percentiles 50/90/99/100: %.1f %.1f %.1f %.1f us" % tuple(q))
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--sites", default="100000")
    ap.add_argument("--taxa", default="50")
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/wg_timeline")
    args = ap.parse_args()
    from phylo_utils_amd import TreeModel
    from phylo_utils_amd import _native as N
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import random_tree, simulate_states
    os.makedirs(args.out, exist_ok=True)
    for n in (int(x) for x in args.taxa.split(",")):
        for m in (int(x) for x in args.sites.split(",")):
            cfg = dict(CONFIGS[args.config], ntax=n, sites=m)
            model = make_model(cfg)
            K = len(model.freqs)
            rm = GammaRateModel(cfg["ncat"], cfg["alpha"])
            tree = random_tree(np.random.default_rng(1234), n)
            st = simulate_states(np.random.default_rng(1000), tree, model, rm.rates, m)
            names = sorted(st, key=lambda s: int(s[1:]))
            codes = np.stack([st[x] for x in names]).astype(np.uint8)
            tm = TreeModel(keep_partials=True)
            tm.set_alignment_codes(codes, np.eye(K), names)
            tm.set_substitution_model(model)
            tm.set_rate_model(rm)
            tm.set_tree(tree)
            tm.initialise()
            ctx = tm._ctx
            for _ in range(400):
                N.check(N.lib().pu_enqueue(ctx), ctx)
            N.check(N.lib().pu_synchronize(ctx, None), ctx)
            path = os.path.join(args.out, "n%d_s%d.bin" % (n, m))
            if os.path.exists(path):
                os.remove(path)
            os.environ["PU_STAMPS_FILE"] = path
            for _ in range(args.launches):
                N.check(N.lib().pu_enqueue(ctx), ctx)
            N.check(N.lib().pu_synchronize(ctx, None), ctx)
            os.environ.pop("PU_STAMPS_FILE")
            # (n_ops + 1) parents x 4 categories x 64 sites x 32 B per block
            plan = N.ctx_plan(ctx)
            bytes_per_wg = n * 8192 * plan["blocks"] / plan["grid"]
            print("plan", plan, flush=True)
            txt = []
            for i, L in enumerate(load(path)):
                txt.append("== taxa %d sites %d launch %d\n%s" % (n, m, i,
                                                                 analyse(L, bytes_per_wg)))
            txt = "\n".join(txt)
            print(txt, flush=True)
            with open(os.path.join(args.out, "n%d_s%d.txt" % (n, m)), "w") as f:
                f.write(txt + "\n")
            del tm


if __name__ == "__main__":
    main()
