#!/usr/bin/env python
"""r05: where does the batched traversal (k_prune_trees) lose against k_prune?  cfg5 trees
(100 taxa, 50k sites, lnL-only): traversal time of one tree's own launch, of a batch of that
one tree, of batches of 8 / 32 trees (per tree), each the median of --reps launches."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import CONFIGS, make_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trees", default="1,8,32")
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    from phylo_utils_amd import TreeModel
    from phylo_utils_amd import _native as N
    from phylo_utils_amd.batch import TreeBatch
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import random_tree, simulate_states
    cfg = CONFIGS["cfg5"]
    model = make_model(cfg)
    rm = GammaRateModel(cfg["ncat"], cfg["alpha"])
    true = random_tree(np.random.default_rng(1234), cfg["ntax"])
    st = simulate_states(np.random.default_rng(999), true, model, rm.rates, cfg["sites"])
    names = sorted(st, key=lambda s: int(s[1:]))
    codes = np.stack([st[n] for n in names]).astype(np.uint8)
    T = max(int(x) for x in args.trees.split(","))
    tms = []
    for i in range(T):
        tm = TreeModel(keep_partials=False)
        tm.set_alignment_codes(codes, np.eye(4), names)
        tm.set_substitution_model(model)
        tm.set_rate_model(rm)
        tm.set_tree(random_tree(np.random.default_rng(10_000 + i), cfg["ntax"]))
        tm.initialise()
        tm.likelihood()
        tms.append(tm)
    lib = N.lib()
    upd = (cfg["ntax"] - 1) * cfg["sites"] * cfg["ncat"]

    def single(tm):
        ctx = tm._ctx
        for _ in range(10):
            lib.pu_enqueue(ctx)
        N.check(lib.pu_ctx_profile(ctx, 1), ctx)
        for _ in range(args.reps):
            N.check(lib.pu_enqueue(ctx), ctx)
        tr, tot = np.zeros(args.reps), np.zeros(args.reps)
        n = ctypes.c_int()
        N.check(lib.pu_ctx_kernel_times(ctx, N.ptr(tr), N.ptr(tot), args.reps, ctypes.byref(n)), ctx)
        N.check(lib.pu_ctx_profile(ctx, 0), ctx)
        return float(np.median(tr[:n.value]))

    def batched(models):
        b = TreeBatch(models)
        for _ in range(5):
            b.enqueue()
        b._check(lib.pu_batch_profile(b._b, 1), "profile")
        for _ in range(args.reps):
            b.enqueue()
        tr, tot = np.zeros(args.reps), np.zeros(args.reps)
        n = ctypes.c_int()
        b._check(lib.pu_batch_kernel_times(b._b, N.ptr(tr), N.ptr(tot), args.reps,
                                           ctypes.byref(n)), "times")
        b.close()
        return float(np.median(tr[:n.value]))

    plan = N.ctx_plan(tms[0]._ctx)
    print("tree 0 plan", plan, flush=True)
    for i in range(min(4, T)):
        print("tree %d own launch: %.4f ms (%.0f G upd/s)  variant %d" % (
            i, single(tms[i]), upd / single(tms[i]) / 1e6, N.ctx_plan(tms[i]._ctx)["variant"]),
            flush=True)
    for n in (int(x) for x in args.trees.split(",")):
        ms = batched(tms[:n])
        print("batch of %3d: %.4f ms, %.4f ms per tree (%.0f G upd/s)" % (
            n, ms, ms / n, n * upd / ms / 1e6), flush=True)


if __name__ == "__main__":
    main()
