#!/usr/bin/env python
"""Debug: the bench's LnlRing over gloo with two ranks on one GPU, the slot filled by
pu_enqueue (strong-scaling slices of a 5000-site alignment).  Prints every rank's slot
before and after each all-reduce.  Launch: python scripts/debug_ring_gpu.py (spawns 2)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    if "WORLD_SIZE" not in os.environ:
        sys.exit(bench.spawn_ranks(2, [os.path.abspath(__file__)]))
    import numpy as np
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo")
    from phylo_utils_amd import TreeModel
    from phylo_utils_amd import _native as N
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import random_tree
    cfg = bench.CONFIGS["cfg2"]
    model = bench.make_model(cfg)
    rm = GammaRateModel(4, 0.5)
    tree = random_tree(np.random.default_rng(1234), 50)
    lo, hi = bench.strong_slice(5000, world, rank)
    names, codes = bench.strong_alignment(tree, model, rm.rates, 5000, lo, hi)
    tm = TreeModel(device=0)
    tm.set_alignment_codes(codes, np.eye(4), names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    ctx = tm._ctx
    print("rank", rank, "local", tm.likelihood(), flush=True)
    slot = torch.zeros(1, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    N.check(N.lib().pu_ctx_set_stream(ctx, ctypes.c_void_p(st.cuda_stream)), ctx)
    N.check(N.lib().pu_set_lnl_device_output(ctx, ctypes.c_void_p(slot.data_ptr())), ctx)
    for i in range(3):
        N.check(N.lib().pu_enqueue(ctx), ctx)
        torch.cuda.synchronize(dev)
        before = float(slot.item())
        w = dist.all_reduce(slot, async_op=True)
        w.wait()
        torch.cuda.synchronize(dev)
        print("rank", rank, "step", i, "before", before, "after", float(slot.item()),
              "stream", st.cuda_stream, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
