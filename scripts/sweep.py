#!/usr/bin/env python
"""Plan / size sweep on one GPU (interleaved rounds in one process).

    python scripts/sweep.py --config cfg2 --grid 'PU_KEEP_OCC=,4,7' --sites 65536,100000
    python scripts/sweep.py --config cfg2 --sites 50000,...,300000 --json out.json

Each variant (the `--grid` env axes, empty = unset) re-plans the schedule and times
`--steps` traversal kernels with HIP events; the best of `--rounds` is reported.  With
`--json`, the default plan's per-update rate of every size is written with the
neighbour check of DESIGN 4.1: a point is flagged when its rate is more than 5 % below the
better of the sizes either side of it (per tree size).
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
    ap.add_argument("--grid", default="",
                    help="extra env axes, e.g. 'PU_VARIANT=0,8,12;PU_PERSIST=,4' (empty = unset)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lnl-only", action="store_true")
    ap.add_argument("--warm-seconds", type=float, default=2.0)
    ap.add_argument("--sites", default="", help="comma list: sweep the alignment length")
    ap.add_argument("--taxa", default="", help="comma list: sweep the tree size")
    ap.add_argument("--json", default="", help="write the per-size results and neighbour check")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    taxa = [int(n) for n in args.taxa.split(",")] if args.taxa else [cfg["ntax"]]
    sites = [int(m) for m in args.sites.split(",")] if args.sites else [cfg["sites"]]
    rows = []
    for n in taxa:
        for m in sites:
            rows += run_one(args, dict(cfg, ntax=n, sites=m))
    if args.json:
        import json
        out = {"config": args.config, "steps": args.steps, "rounds": args.rounds,
               "rows": rows, "neighbour_check": neighbour_check(rows)}
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
        for r in out["neighbour_check"]:
            print("neighbour check: %s" % r)


def neighbour_check(rows, tol=0.05):
    """Per (variant, taxa): flag sizes whose M updates/s is > tol below the better neighbour."""
    flags = []
    keys = sorted({(r["variant"], r["taxa"]) for r in rows})
    for var, n in keys:
        pts = sorted((r["sites"], r["mups"]) for r in rows
                     if r["variant"] == var and r["taxa"] == n)
        bad = 0
        for i, (m, v) in enumerate(pts):
            nb = [pts[j][1] for j in (i - 1, i + 1) if 0 <= j < len(pts)]
            if nb and v < (1 - tol) * max(nb):
                flags.append({"variant": var, "taxa": n, "sites": m, "mups": round(v),
                              "best_neighbour": round(max(nb)),
                              "below": round(1 - v / max(nb), 4)})
                bad += 1
        if not bad:
            flags.append({"variant": var, "taxa": n, "ok": True, "points": len(pts)})
    return flags


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
    print("config %s taxa %d sites %d U=%d lnl=%.10f" % (args.config, cfg["ntax"], cfg["sites"],
                                                         U, ref))
    rows = []
    for v in variants:
        tm = models[v]
        lnl = tm.likelihood()
        tr = min(x[0] for x in res[v])
        al = min(x[1] for x in res[v])
        label = " ".join("%s=%s" % (k, x) for k, x in zip(names_ax, v))
        print("%-45s traverse %.4f ms (%.0f M upd/s)  step %.4f ms  dlnl=%.1e" %
              (label, tr, U / tr / 1e3, al, abs(lnl - ref)))
        rows.append({"variant": label or "default", "taxa": cfg["ntax"], "sites": cfg["sites"],
                     "traverse_ms": tr, "step_ms": al, "mups": U / tr / 1e3,
                     "dlnl": abs(lnl - ref)})
    return rows


if __name__ == "__main__":
    main()
