#!/usr/bin/env python
"""Throughput of the Felsenstein pruning hot path on MI355X (BASELINE.json metric).

One step = one complete likelihood evaluation of the configured workload on every
rank: P(t*r) for every branch and rate category, the whole post-order of partial
updates, the root combine + lnl_node + logsumexp over categories + pattern-weighted
sum (tree_model.py:160-217), and -- for N > 1 -- the RCCL all-reduce (sum) of the
per-rank lnL (site sharding).  Inputs are resident in HBM before
the timed region (tips uploaded once, as TreeModel.initialise does).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4]
    python bench.py --workload edges [--config ...]   # SURVEY 8(f) N1, secondary line
    python bench.py --config cfg5                      # tree sharding

Scaling is weak: every rank owns `sites` patterns of one larger alignment on the
same tree, so per-GPU work is fixed as N grows.
"""
import argparse
import glob
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# fp64 dense MFMA: 32 flop/cycle/SIMD (SQ_VALU_MFMA_BUSY_CYCLES: 64 cycles per
# v_mfma_f64_16x16x4, 16 per 4x4x4_4b) x 1024 SIMDs x 2.4 GHz = AMD's 78.6 TF spec
# (the guide lists no fp64 row)
FP64_MFMA_PEAK_TFS = 78.6

CONFIGS = {
    "cfg2": dict(subst="GTR+G4", alpha=0.5, ntax=50, sites=100_000, ncat=4,
                 desc="BASELINE cfg2: GTR+G4 (alpha 0.5), 50-taxon tree, 100k DNA sites per GPU"),
    "cfg3": dict(subst="LG+G4", alpha=0.8, ntax=200, sites=10_000, ncat=4,
                 desc="BASELINE cfg3: LG+G4 (alpha 0.8), 200-taxon tree, 10k AA sites per GPU"),
    "cfg4": dict(subst="GTR+G4", alpha=0.5, ntax=1000, sites=125_000, ncat=4,
                 desc="BASELINE cfg4 shard: GTR+G4, 1000-taxon tree, 125k DNA sites per GPU "
                      "(1M sites over 8 GPUs)"),
    "cfg5": dict(subst="GTR+G4", alpha=0.5, ntax=100, sites=50_000, ncat=4, trees=125,
                 desc="BASELINE cfg5 shard: GTR+G4, 125 bootstrap-replicate 100-taxon trees "
                      "per GPU (1000 over 8 GPUs) on one 50k-site DNA alignment"),
}


class LnlRing:
    """Two lnL slots for the per-step all-reduce.  The sum of step i (8 bytes over xGMI,
    latency-bound) runs on the collective stream while step i + 1's kernels run; step
    i + 2 reuses step i's slot, so it first waits for that all-reduce (Work.wait: on the
    device for RCCL, on the host for gloo).  drain() waits for every outstanding sum, so
    all of them complete inside the timed region."""

    def __init__(self, make_slot, world, all_reduce_async):
        self.slots = [make_slot(), make_slot()]
        self.world = world
        self.all_reduce_async = all_reduce_async
        self.works = [None, None]
        self.n = 0

    def step(self, fill):
        slot = self.n & 1
        self.n += 1
        if self.works[slot] is not None:
            self.works[slot].wait()
            self.works[slot] = None
        fill(slot)
        if self.world > 1:
            self.works[slot] = self.all_reduce_async(self.slots[slot])

    def drain(self):
        for k in range(2):
            if self.works[k] is not None:
                self.works[k].wait()
                self.works[k] = None

    def last(self):
        return self.slots[(self.n - 1) & 1]


def warm_for(seconds, batch, world, dev=None):
    """Untimed warm-up for `seconds` of rank 0's clock.  Every step issues a collective (the
    lnL all-reduce / all-gather), so each rank timing its own loop would run a different
    number of steps and pair one rank's collectives with another's later ones; rank 0
    decides after every batch and broadcasts it.  Returns the number of batches run."""
    import torch
    import torch.distributed as dist
    tw = time.perf_counter()
    n = 0
    while True:
        go = torch.tensor([1.0 if time.perf_counter() - tw < seconds else 0.0],
                          dtype=torch.float64, device=dev)
        if world > 1:
            dist.broadcast(go, 0)
        if float(go.item()) == 0.0:
            return n
        batch()
        n += 1


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_model(cfg):
    from phylo_utils_amd import substitution_models as SM
    from phylo_utils_amd.synthetic import CFG2_FREQS, CFG2_GTR_RATES
    if cfg["subst"].startswith("GTR"):
        return SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    return SM.LG()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--warm-seconds", type=float, default=2.0,
                    help="after the W warmup steps keep running untimed steps for at least "
                         "this long, so the GPU clocks are up before the timed region")
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--lnl-only", action="store_true",
                    help="PU_LNL_ONLY: do not keep every internal CLV in HBM")
    ap.add_argument("--workload", default="traversal",
                    choices=["traversal", "edges", "patterns"],
                    help="edges: branch-length derivatives on the resident CLVs and one "
                         "optimising-traversal sweep (SURVEY 8(f) N1) instead of the "
                         "headline traversal")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    # PU_BENCH_BACKEND=gloo: rehearsal of the multi-rank path with several ranks on one GPU
    # (RCCL refuses two ranks on one device); the measured runs use RCCL ("nccl")
    backend = os.environ.get("PU_BENCH_BACKEND", "nccl")
    gpu = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from phylo_utils_amd import TreeModel
    from phylo_utils_amd import _native as N
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import random_tree, simulate_states

    if args.workload == "patterns":
        if rank == 0:
            print(json.dumps(bench_patterns(args, dev)), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    if args.config == "cfg5":
        out = bench_trees(args, cfg, world, rank, local_rank, dev)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    model = make_model(cfg)
    K = len(model.freqs)
    rm = GammaRateModel(cfg["ncat"], cfg["alpha"])
    C = rm.ncat
    S = cfg["sites"]
    ntax = cfg["ntax"]
    t_setup = time.time()
    tree = random_tree(np.random.default_rng(1234), ntax)          # same tree on every rank
    states = simulate_states(np.random.default_rng(1000 + rank), tree, model, rm.rates, S)
    names = sorted(states, key=lambda s: int(s[1:]))
    codes = np.stack([states[n] for n in names]).astype(np.uint8)
    tm = TreeModel(device=dev.index, keep_partials=not args.lnl_only)
    tm.set_alignment_codes(codes, np.eye(K), names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    ctx = tm._ctx
    log("[bench] rank %d setup %.1fs, device bytes %.2f GB" %
        (rank, time.time() - t_setup, N.lib().pu_ctx_device_bytes(ctx) / 1e9))

    if args.workload == "edges":
        if rank == 0:
            print(json.dumps(bench_edges(tm, model, rm, codes, K, C, S, ntax, args, cfg)),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    ring = LnlRing(lambda: torch.zeros(1, dtype=torch.float64, device=dev), world,
                   lambda t: dist.all_reduce(t, async_op=True))
    ptrs = [ctypes.c_void_p(t.data_ptr()) for t in ring.slots]
    stream = torch.cuda.current_stream(dev)
    N.check(N.lib().pu_ctx_set_stream(ctx, ctypes.c_void_p(stream.cuda_stream)), ctx)
    enqueue = N.lib().pu_enqueue
    set_out = N.lib().pu_set_lnl_device_output

    def fill(slot):  # one evaluation, its lnL into ring slot `slot`
        set_out(ctx, ptrs[slot])
        rc = enqueue(ctx)
        if rc:
            N.check(rc, ctx, "pu_enqueue")

    def step():
        ring.step(fill)

    def drain():
        ring.drain()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        step()
    drain()
    def batch():
        for _ in range(50):
            step()
        drain()

    warm_for(args.warm_seconds, batch, world, dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # HIP events around every traversal launch of the timed region, on the launch stream
    N.check(N.lib().pu_ctx_profile(ctx, 1), ctx)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    lnl_total = float(ring.last().item())  # the last step's lnL

    trav_ms, tot_ms, nrec = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
    N.check(N.lib().pu_ctx_kernel_ms(ctx, ctypes.byref(trav_ms), ctypes.byref(tot_ms),
                                     ctypes.byref(nrec)), ctx)
    N.check(N.lib().pu_ctx_profile(ctx, 0), ctx)
    torch.cuda.synchronize(dev)

    updates_per_step = (ntax - 1) * S * C       # (N-2) ops + root combine, per rank
    total_updates = updates_per_step * world * args.steps
    value = total_updates / elapsed / 1e6
    # 8*(3K+3) B per update (2 child CLVs + parent + 3 scalers, tips as
    # dense fp64) + root scalers read + sitewise output
    alg_bytes = updates_per_step * 8 * (3 * K + 3) + S * C * 8 + S * 8
    achieved = alg_bytes / (trav_ms.value * 1e-3) / 1e9
    # what the fused kernel must move at minimum: every internal + root CLV and scaler
    # written once (TreeModel keeps them), tip codes read once
    min_bytes = (0 if args.lnl_only else (ntax - 2)) * S * C * (K + 1) * 8 + \
        S * C * (K + 1) * 8 + ntax * S + S * 8
    # HBM bytes per launch measured with rocprofv3 PMC passes (scripts/collect_profiles.py);
    # the newest round's file for this config and mode
    traffic = None
    mode = "_lnl" if args.lnl_only else ""
    tfs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic_%s%s.json" %
                                        (args.config, mode))))
    if tfs:
        try:
            traffic = json.load(open(tfs[-1])).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    kern_s = trav_ms.value * 1e-3
    common = {"traffic": traffic,
              "traffic_GBps": round(traffic / kern_s / 1e9, 1) if traffic else None,
              "kernel_ms": round(trav_ms.value, 5), "step_kernels_ms": round(tot_ms.value, 5),
              "events": nrec.value, "alg_bytes_per_launch": alg_bytes,
              "min_bytes_per_launch": min_bytes,
              "min_bytes_frac": round(min_bytes / kern_s / 1e9 / HBM_PEAK_GBS, 4)}
    if K == 20:
        # k_prune_mfma is fp64-MFMA-bound: per update 2 children x 2K^2 flop,
        # exactly what its 16-row + 4-row tiling executes
        flop = updates_per_step * 2 * 2 * K * K
        tfs_ach = flop / kern_s / 1e12
        roofline = dict({"bound": "mfma", "achieved": round(tfs_ach, 2),
                         "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": round(tfs_ach / FP64_MFMA_PEAK_TFS, 4),
                         "kernel": "k_prune_mfma", "flop_per_launch": flop,
                         "alg_GBps": round(achieved, 1)}, **common)
    else:
        roofline = dict({"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "kernel": "k_prune"}, **common)
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "M updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded random-joining tree, alignment simulated under the model)",
        "config": {"workload": cfg["desc"], "config": args.config, "substitution": cfg["subst"],
                   "taxa": ntax, "sites_per_gpu": S, "total_sites": S * world,
                   "categories": C, "states": K,
                   "updates_per_step": updates_per_step * world,
                   "partials": "lnl_only" if args.lnl_only else "all internal CLVs kept in HBM",
                   "parallelism": "site-sharded x%d, RCCL lnL all-reduce overlapped with the "
                                  "next step's kernels" % world},
        "roofline": roofline,
        "lnl": lnl_total,
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], out["lnl_rel_err_vs_cpu"] = cpu_baseline(
            tm, model, rm, codes, K, C, S, ntax, args, lnl_total)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_trees(args, cfg, world, rank, local_rank, dev):
    """SURVEY 8(e) G2 / BASELINE cfg5: many trees on one alignment, trees sharded over ranks
    (weak scaling: `trees` trees per rank).  One step = the lnL of every local tree (P,
    traversal, reduce per tree; PU_LNL_ONLY -- only the lnL is wanted) with the trees'
    launches spread over 4 HIP streams so that several fill the GPU at once, then one
    all-gather of the per-tree lnLs (the only collective)."""
    import torch
    import torch.distributed as dist
    from phylo_utils_amd import TreeModel
    from phylo_utils_amd import _native as N
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import random_tree, simulate_states
    model = make_model(cfg)
    K = len(model.freqs)
    rm = GammaRateModel(cfg["ncat"], cfg["alpha"])
    C, S, ntax, T = rm.ncat, cfg["sites"], cfg["ntax"], cfg["trees"]
    t_setup = time.time()
    true_tree = random_tree(np.random.default_rng(1234), ntax)
    states = simulate_states(np.random.default_rng(999), true_tree, model, rm.rates, S)
    names = sorted(states, key=lambda s: int(s[1:]))
    codes = np.stack([states[n] for n in names]).astype(np.uint8)
    lib = N.lib()
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    lnl = torch.zeros(T, dtype=torch.float64, device=dev)
    tms = []
    for i in range(T):
        tree = random_tree(np.random.default_rng(10_000 + rank * T + i), ntax)
        tm = TreeModel(device=dev.index, keep_partials=False)
        tm.set_alignment_codes(codes, np.eye(K), names)
        tm.set_substitution_model(model)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        ctx = tm._ctx
        N.check(lib.pu_ctx_set_stream(ctx, ctypes.c_void_p(streams[i % 4].cuda_stream)), ctx)
        N.check(lib.pu_set_lnl_device_output(ctx, ctypes.c_void_p(lnl.data_ptr() + 8 * i)),
                ctx)
        tms.append(tm)
    log("[bench] rank %d: %d trees set up in %.1fs" % (rank, T, time.time() - t_setup))
    ref = np.array([tm.likelihood() for tm in tms])  # synchronous pu_run values
    gathered = [torch.empty_like(lnl) for _ in range(world)] if world > 1 else None
    main_stream = torch.cuda.current_stream(dev)

    def step():
        ev = torch.cuda.Event()
        ev.record(main_stream)
        for st in streams:
            st.wait_event(ev)
        for tm in tms:
            rc = lib.pu_enqueue(tm._ctx)
            if rc:
                N.check(rc, tm._ctx, "pu_enqueue")
        for st in streams:
            main_stream.wait_stream(st)
        if world > 1:
            dist.all_gather(gathered, lnl)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    def batch():
        step()
        torch.cuda.synchronize(dev)

    warm_for(args.warm_seconds, batch, world, dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    got = lnl.cpu().numpy()
    max_rel = float(np.max(np.abs(got - ref) / np.abs(ref)))
    # per-launch kernel time of one context, measured with events on its stream
    ctx0 = tms[0]._ctx
    N.check(lib.pu_ctx_profile(ctx0, 1), ctx0)
    for _ in range(20):
        N.check(lib.pu_enqueue(ctx0), ctx0)
    trav_ms, tot_ms, nrec = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
    N.check(lib.pu_ctx_kernel_ms(ctx0, ctypes.byref(trav_ms), ctypes.byref(tot_ms),
                                 ctypes.byref(nrec)), ctx0)
    N.check(lib.pu_ctx_profile(ctx0, 0), ctx0)
    torch.cuda.synchronize(dev)
    upd_tree = (ntax - 1) * S * C
    value = upd_tree * T * world * args.steps / elapsed / 1e6
    alg = upd_tree * 8 * (3 * K + 3) + S * C * 8 + S * 8
    ach = alg / (trav_ms.value * 1e-3) / 1e9
    return {
        "metric": METRIC, "value": round(value, 3), "unit": "M updates/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded random-joining trees, alignment simulated on another)",
        "config": {"workload": cfg["desc"], "config": "cfg5", "taxa": ntax, "sites": S,
                   "categories": C, "states": K, "trees_per_gpu": T, "total_trees": T * world,
                   "updates_per_step": upd_tree * T * world, "partials": "lnl_only",
                   "parallelism": "tree-sharded x%d, 4 HIP streams per GPU, all-gather of "
                                  "the per-tree lnL" % world},
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "kernel": "k_prune",
                     "kernel_ms": round(trav_ms.value, 5), "events": nrec.value,
                     "alg_bytes_per_launch": alg, "traffic": None,
                     "note": "one tree's launch measured alone; the step overlaps 4"},
        "lnl_max_rel_diff_vs_sync_runs": max_rel,
    }


def bench_edges(tm, model, rm, codes, K, C, S, ntax, args, cfg):
    """SURVEY 8(f) N1 on the same workload: (1) `steps` evaluations of lnL, dlnL/dt and
    d2lnL/dt2 on the root edge (one k_edge launch + 24-byte read-back each, the unit of
    work of the Newton optimiser), (2) one full optimising-traversal sweep.  Roofline of
    k_edge: reads of both ends' CLVs and scalers (tips counted as dense fp64 CLVs, as in
    SURVEY 8(d) M3) + pattern weights, per launch."""
    from phylo_utils_amd import _native as N
    lib = N.lib()
    ctx = tm._ctx
    a, b = tm.traversal.root_edge
    t0 = tm.traversal.root_length()
    out = np.zeros(3)
    for k in range(args.warmup):
        N.check(lib.pu_edge_derivs(ctx, a, b, t0 * (1 + 0.01 * k), N.ptr(out)), ctx)
    N.check(lib.pu_ctx_profile(ctx, 1), ctx)
    t_start = time.perf_counter()
    for k in range(args.steps):
        N.check(lib.pu_edge_derivs(ctx, a, b, t0 * (1 + 1e-3 * (k % 7)), N.ptr(out)), ctx)
    el = time.perf_counter() - t_start
    kms, ems, nrec = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
    N.check(lib.pu_ctx_edge_kernel_ms2(ctx, ctypes.byref(kms), ctypes.byref(ems),
                                       ctypes.byref(nrec)), ctx)
    N.check(lib.pu_ctx_profile(ctx, 0), ctx)
    alg = S * C * (2 * K + 2) * 8 + S * 8
    ach = alg / (ems.value * 1e-3) / 1e9  # k_edge alone (its reduction launch follows)
    lnl0 = tm.likelihood()
    ts = time.perf_counter()
    lnl1 = tm.optimise_branch_lengths(tol=1e-8, max_iter=50, sweeps=1)
    sweep_s = time.perf_counter() - ts
    n_edges = 2 * ntax - 3
    res = {
        "metric": "edge evaluations/sec (lnL + dlnL/dt + d2lnL/dt2 over all sites), "
                  "GTR+G4; SURVEY 8(f) N1",
        "value": round(args.steps / el, 1), "unit": "evaluations/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 5), "higher_is_better": True,
        "scaling": "none", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": cfg["desc"] + "; edge derivatives on the root edge + one "
                   "optimising-traversal sweep", "config": args.config, "taxa": ntax,
                   "sites": S, "categories": C, "states": K},
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "kernel": "k_edge<%d, EDGE_DERIV>" % K, "kernel_ms": round(ems.value, 5),
                     "with_reduction_ms": round(kms.value, 5),
                     "events": nrec.value, "alg_bytes_per_launch": alg, "traffic": None},
        "sweep": {"edges": n_edges, "ms": round(sweep_s * 1e3, 3),
                  "newton_iterations": getattr(tm, "last_newton_iterations", None),
                  "lnl_before": lnl0, "lnl_after": lnl1},
    }
    if not args.no_cpu_baseline:
        from oracle import oracle as orc
        ea = tm.node_partials(a)
        eb = tm.node_partials(b)
        ev, elv, iv = model.engine_eigen()
        reps, tc = 0, time.perf_counter()
        while time.perf_counter() - tc < min(args.cpu_seconds, 10.0):
            orc.edge_derivs(ea[0], ea[1], eb[0], eb[1], ev, elv, iv, t0, rm.rates, rm.weights,
                            model.freqs)
            reps += 1
        cel = time.perf_counter() - tc
        res["cpu_baseline"] = {"value": round(reps / cel, 2), "unit": "evaluations/s",
                               "cores": 1, "kind": "port",
                               "sample": "%d root-edge evaluations (oracle or_edge_derivs, one "
                                         "thread, P/dP/d2P included)" % reps}
    return res


def bench_patterns(args, dev):
    """site-pattern compression of the BASELINE cfg4 alignment (1000 taxa x
    1M DNA columns) on one GPU -- np.unique(alignment, axis=1, return_inverse,
    return_counts) of alignment.py:40-57 as pu_compress_patterns_device, codes resident in
    HBM.  Roofline bytes: the codes read once, the unique columns, inverse index and counts
    written once."""
    import torch
    from phylo_utils_amd import _native as N
    from phylo_utils_amd.alignment import DNA, code_table
    lib = N.lib()
    table, lut = code_table(DNA)
    n_codes = len(table)
    nt, S = 1000, 1_000_000
    rng = np.random.default_rng(7)
    acgt = lut[np.frombuffer(b"ACGT", dtype=np.uint8)]
    codes = acgt[rng.integers(0, 4, size=(nt, S))]
    dup = rng.random(S) < 0.3        # 30% of the columns repeat another column
    codes[:, dup] = codes[:, rng.integers(0, S, size=int(dup.sum()))]
    amb = rng.random((nt, S)) < 0.001  # a few ambiguity codes (N, R, ...)
    codes[amb] = rng.integers(0, n_codes, size=int(amb.sum()))
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    d_codes = torch.from_numpy(codes).to(dev)
    ld = (S + 15) // 16 * 16   # unique rows padded to 16 bytes (4-byte stores)
    d_unique = torch.empty(nt * ld, dtype=torch.uint8, device=dev)
    d_counts = torch.empty(S, dtype=torch.int64, device=dev)
    d_inv = torch.empty(S, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)
    U = ctypes.c_int64()

    def run():
        N.check(lib.pu_compress_patterns_device(
            dev.index, ctypes.c_void_p(st.cuda_stream), ctypes.c_void_p(d_codes.data_ptr()), nt,
            S, n_codes, ctypes.c_void_p(d_unique.data_ptr()), ld,
            ctypes.c_void_p(d_counts.data_ptr()), ctypes.c_void_p(d_inv.data_ptr()),
            ctypes.byref(U)), None, "pu_compress_patterns_device")

    for _ in range(max(1, args.warmup // 5)):
        run()
    torch.cuda.synchronize(dev)
    steps = max(1, min(args.steps, 20))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    t0 = time.perf_counter()
    for e0, e1 in ev:
        e0.record(st)
        run()
        e1.record(st)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ms = sum(e0.elapsed_time(e1) for e0, e1 in ev) / steps
    Uv = U.value
    alg = nt * S + nt * Uv + 8 * S + 8 * Uv
    ach = alg / (ms * 1e-3) / 1e9
    # spot check against the reference's call on a slice of columns is in
    # tests/test_gpu_patterns.py; here: the counts add up and every column maps to a pattern
    cnt = d_counts[:Uv].cpu().numpy()
    inv = d_inv.cpu().numpy()
    assert cnt.sum() == S and inv.min() == 0 and inv.max() == Uv - 1
    res = {
        "metric": "alignment columns compressed per second (np.unique(axis=1) with inverse "
                  "and counts, alignment.py:40-57); SURVEY 8(f) N2",
        "value": round(S / (ms * 1e-3) / 1e6, 3), "unit": "M columns/s", "n_gpus": 1,
        "steps": steps, "warmup": max(1, args.warmup // 5),
        "ms_per_step": round(el / steps * 1e3, 4), "higher_is_better": True,
        "scaling": "none", "vs_baseline": None, "dtype": "u8", 
        "data": "synthetic (uniform A/C/G/T codes, 30% of columns duplicated, 0.1% ambiguity "
                "codes)",
        "config": {"workload": "BASELINE cfg4 alignment: 1000 taxa x 1M DNA columns",
                   "taxa": nt, "sites": S, "n_codes": n_codes, "patterns": Uv},
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "kernel": "pu_compress_patterns_device (pack, LSD radix sort, scan, "
                               "scatter, unpack)", "kernel_ms": round(ms, 4),
                     "alg_bytes_per_launch": alg, "traffic": None},
    }
    if not args.no_cpu_baseline:
        # the reference's own call on float partials [ntaxa][S][K] (alignment.py:53), on a
        # bounded slice of the same columns
        n = 4000
        parts = table[codes[:, :n]]
        reps, tc = 0, time.perf_counter()
        while time.perf_counter() - tc < min(args.cpu_seconds, 10.0) or reps == 0:
            np.unique(parts, return_inverse=True, return_counts=True, axis=1)
            reps += 1
        cel = time.perf_counter() - tc
        res["cpu_baseline"] = {"value": round(reps * n / cel / 1e6, 4), "unit": "M columns/s",
                               "cores": 1, "kind": "port",
                               "sample": "%d x np.unique(partials, axis=1, return_inverse, "
                                         "return_counts) over %d taxa x %d columns of the same "
                                         "alignment (alignment.py:53's call, float64 partials)"
                                         % (reps, nt, n)}
    return res


def cpu_baseline(tm, model, rm, codes, K, C, S, ntax, args, gpu_lnl):
    """The oracle's C restatement of the same loop nest (OpenMP over site blocks), timed on
    this host on the same workload: P matrices + all ops + root + lnL per repetition."""
    from oracle import oracle as orc
    tr = tm.traversal
    n_nodes = tr.n_nodes
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    log("[bench] cpu baseline: %d threads, ~%.0fs" % (threads, args.cpu_seconds))
    partials = np.zeros((n_nodes, S, C, K))
    scale = np.zeros((n_nodes, S, C))
    eye = np.eye(K)
    for name, node in tr.names.items():
        partials[node] = eye[codes[tm.names[name]]][:, None, :]
    ev, el, iv = model.engine_eigen()
    ops = np.ascontiguousarray(tr.postorder_traversal, dtype=np.int32)
    bl = tr.op_lengths()
    rates = np.ascontiguousarray(rm.rates)
    w = np.ascontiguousarray(rm.weights)
    sw = np.ones(S)
    fr = np.ascontiguousarray(model.freqs, dtype=np.float64)
    reps, t0 = 0, time.perf_counter()
    lnl = None
    while True:
        P = orc.pmatrix_c(ev, el, iv, bl.reshape(-1), rates).reshape(len(ops), 2, C, K, K)
        Pr = orc.pmatrix_c(ev, el, iv, np.array([0.0, tr.root_length()]), rates)
        lnl = orc.traverse_prepared(K, C, S, ops, np.ascontiguousarray(P),
                                    np.ascontiguousarray(Pr), tr.root_edge, partials, scale, fr,
                                    w, sw, threads)
        reps += 1
        el_t = time.perf_counter() - t0
        if el_t >= args.cpu_seconds or reps >= 5000:
            break
    ups = (ntax - 1) * S * C * reps / el_t / 1e6
    rel = abs(gpu_lnl - lnl) / abs(lnl)
    log("[bench] cpu: %d reps in %.2fs -> %.2f M updates/s; lnL cpu %.10f gpu %.10f rel %.2e"
        % (reps, el_t, ups, lnl, gpu_lnl, rel))
    return ({"value": round(ups, 3), "unit": "M updates/s", "cores": threads, "kind": "port",
             "sample": "%d full traversals of the same workload (oracle/pruning_oracle.c, "
                       "OpenMP over site blocks, P matrices included)" % reps}, rel)


if __name__ == "__main__":
    main()
