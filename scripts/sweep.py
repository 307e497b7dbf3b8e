#!/usr/bin/env python
"""Kernel-variant sweep on one GPU (interleaved rounds in one process).

    python scripts/sweep.py --config cfg2 --regs 0,2,4,6 --budgets 16384,32768 --rounds 3

Each variant re-plans the schedule (PU_REGS / PU_LDS_BUDGET are read by
pu_set_schedule) and times `--steps` traversal kernels with HIP events.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import CONFIGS, make_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--regs", default="")
    ap.add_argument("--budgets", default="")
    ap.add_argument("--grid", default="",
                    help="extra env axes, e.g. 'PU_VARIANT=0,8,12;PU_PERSIST=,4' (empty = unset)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lnl-only", action="store_true")
    ap.add_argument("--warm-seconds", type=float, default=2.0)
    ap.add_argument("--sites", default="", help="comma list: sweep the alignment length")
    ap.add_argument("--taxa", default="", help="comma list: sweep the tree size")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.taxa:
        for n in args.taxa.split(","):
            c2 = dict(cfg, ntax=int(n))
            if args.sites:
                for m in args.sites.split(","):
                    run_one(args, dict(c2, sites=int(m)))
            else:
                run_one(args, c2)
        return
    if args.sites:
        for n in args.sites.split(","):
            c2 = dict(cfg, sites=int(n))
            run_one(args, c2)
        return
    run_one(args, cfg)


def run_one(args, cfg):
    from phylo_utils_amd import TreeModel
    from phylo_utils_amd import _native as N
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import random_tree, simulate_states
    model = make_model(cfg)
    K = len(model.freqs)
    rm = GammaRateModel(cfg["ncat"], cfg["alpha"])
    tree = random_tree(np.random.default_rng(1234), cfg["ntax"])
    st = simulate_states(np.random.default_rng(1000), tree, model, rm.rates, cfg["sites"])
    names = sorted(st, key=lambda s: int(s[1:]))
    codes = np.stack([st[n] for n in names]).astype(np.uint8)
    import itertools
    axes = []
    if args.regs:
        axes.append(("PU_REGS", args.regs.split(",")))
    if args.budgets:
        axes.append(("PU_LDS_BUDGET", args.budgets.split(",")))
    for item in filter(None, args.grid.split(";")):
        k, vals = item.split("=", 1)
        axes.append((k.strip(), vals.split(",")))  # "A:B=1:2,3:4" sets A and B together
    names_ax = [a[0] for a in axes]
    variants = list(itertools.product(*[a[1] for a in axes])) or [()]
    models = {}
    for var in variants:
        for k, v in zip(names_ax, var):
            for kk, vv in zip(k.split(":"), v.split(":")):
                if vv == "":
                    os.environ.pop(kk, None)
                else:
                    os.environ[kk] = vv
        tm = TreeModel(keep_partials=not args.lnl_only)
        tm.set_alignment_codes(codes, np.eye(K), names)
        tm.set_substitution_model(model)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        models[var] = tm
    ref = models[variants[0]].likelihood()
    import time
    ctx0 = models[variants[0]]._ctx
    tw = time.perf_counter()
    while time.perf_counter() - tw < args.warm_seconds:  # clocks up before timing
        for _ in range(50):
            N.check(N.lib().pu_enqueue(ctx0), ctx0)
        N.check(N.lib().pu_synchronize(ctx0, None), ctx0)
    U = (cfg["ntax"] - 1) * cfg["sites"] * rm.ncat
    res = {v: [] for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            ctx = models[v]._ctx
            N.check(N.lib().pu_ctx_profile(ctx, 1), ctx)
            for _ in range(args.steps):
                N.check(N.lib().pu_enqueue(ctx), ctx)
            t, a, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
            N.check(N.lib().pu_ctx_kernel_ms(ctx, ctypes.byref(t), ctypes.byref(a),
                                             ctypes.byref(n)), ctx)
            N.check(N.lib().pu_ctx_profile(ctx, 0), ctx)
            res[v].append((t.value, a.value))
    print("config %s sites %d U=%d lnl=%.10f" % (args.config, cfg["sites"], U, ref))
    for v in variants:
        tm = models[v]
        lnl = tm.likelihood()
        tr = min(x[0] for x in res[v])
        al = min(x[1] for x in res[v])
        label = " ".join("%s=%s" % (k, x) for k, x in zip(names_ax, v))
        print("%-45s traverse %.4f ms (%.0f M upd/s)  step %.4f ms  dlnl=%.1e" %
              (label, tr, U / tr / 1e3, al, abs(lnl - ref)))


if __name__ == "__main__":
    main()
