#!/usr/bin/env python
"""Fill PU_BENCH_CACHE with the blocks of bench.py's strong-scaling alignment, in parallel,
before any GPU work: every later `bench.py --total-sites T` process of the same call loads the
blocks instead of simulating them (bench.strong_block).

    PU_BENCH_CACHE=/tmp/pu_sim python scripts/presim.py --config cfg4 --total-sites 1000000
"""
import argparse
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def one(args):
    config, b, n = args
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import random_tree
    cfg = bench.CONFIGS[config]
    model = bench.make_model(cfg)
    rm = GammaRateModel(cfg["ncat"], cfg["alpha"])
    tree = random_tree(np.random.default_rng(1234), cfg["ntax"])  # bench.py's tree
    bench.strong_block(tree, model, rm.rates, b, n)
    return b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--total-sites", type=int, default=1_000_000)
    ap.add_argument("--workers", type=int, default=8)
    a = ap.parse_args()
    if not os.environ.get("PU_BENCH_CACHE"):
        sys.exit("presim.py: set PU_BENCH_CACHE")
    blk = bench.STRONG_BLOCK
    jobs = [(a.config, b, min(blk, a.total_sites - b * blk))
            for b in range((a.total_sites + blk - 1) // blk)]
    with ProcessPoolExecutor(max_workers=min(a.workers, len(jobs))) as ex:
        for b in ex.map(one, jobs):
            print("[presim] block %d" % b, flush=True)


if __name__ == "__main__":
    main()
