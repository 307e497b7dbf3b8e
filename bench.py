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

Scaling is weak by default: every rank owns `sites` patterns of one larger alignment on
the same tree, so per-GPU work is fixed as N grows.  `--total-sites T` is the strong form
(BASELINE cfg4 as stated: ONE T-site alignment split over the N ranks; the alignment is
simulated in fixed 125k-site blocks, block b from seed 1000 + b, so every N sees the same
sites and `config.total_sites` stays T).
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
# fp64 vector FMA: 16 lanes per SIMD per cycle x 2 flop x 1024 SIMDs x 2.4 GHz (the same 78.6 TF)
FP64_VALU_PEAK_TFS = 78.6

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


def spawn_ranks(n, argv=None):
    """`bench.py --gpus N` without a launcher: start N rank processes of this script with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set (one GPU each, RCCL), before anything in
    this process has touched the GPU (this process never does).  Returns the exit status:
    0, or the first non-zero status of a rank (the other ranks are then stopped)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        cmd = argv or [os.path.abspath(__file__)] + sys.argv[1:]
        procs.append(subprocess.Popen([sys.executable] + list(cmd), env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                log("[bench] a rank exited with status %d; stopping the others" % code)
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc


def event_times(ctx, steps):
    """Per-step hipEvent times of the timed region (pu_ctx_kernel_times): medians of the
    traversal launch alone and of the whole step's kernels."""
    from phylo_utils_amd import _native as N
    tr, tot = np.zeros(steps), np.zeros(steps)
    n = ctypes.c_int()
    N.check(N.lib().pu_ctx_kernel_times(ctx, N.ptr(tr), N.ptr(tot), steps, ctypes.byref(n)), ctx)
    k = n.value
    if k == 0:
        raise RuntimeError("no profiled runs recorded")
    tr, tot = tr[:k], tot[:k]
    return {"n": k, "trav_med": round(float(np.median(tr)), 5),
            "trav_mean": round(float(tr.mean()), 5), "step_med": round(float(np.median(tot)), 5)}


def latest_traffic(tag):
    """PMC HBM bytes per k_prune launch from the newest profiles/r*_traffic_<tag>.json
    (scripts/collect_profiles.py: 2*FETCH_SIZE + WRITE_SIZE, separate --pmc passes)."""
    tfs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic_%s.json" % tag))) \
        if tag else []
    if not tfs:
        return None, None
    try:
        return json.load(open(tfs[-1])).get("hbm_bytes_per_launch"), os.path.basename(tfs[-1])
    except (OSError, ValueError):
        return None, None


def latest_pmc(tag):
    """Instruction counters per traversal launch from the newest profiles/r*_pmc_<tag>.json
    (scripts/collect_profiles.py --insts: SQ_INSTS_VALU / SALU / SMEM / LDS, SQ_WAVES, and
    SQ_BUSY_CYCLES-style counters, each from its own --pmc pass)."""
    tfs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_%s.json" % tag))) if tag else []
    if not tfs:
        return None
    try:
        d = json.load(open(tfs[-1]))
    except (OSError, ValueError):
        return None
    d["file"] = os.path.basename(tfs[-1])
    return d


def pmc_tag(config, sites, lnl_only=False, override=False):
    """Key of the profiles/ files (PMC traffic, instruction counts, rocprof kernel stats) for
    one rank's traversal: the config at its own per-GPU size is `<cfg>`; a strong-scaling
    shard of another size is `<cfg>_s<sites>` (`--total-sites 1000000` on one GPU:
    cfg4_s1000000; on 8 GPUs each shard is 125k sites, the cfg4 shard itself); `_lnl` for
    lnL-only traversals.  A --sites override (tests, rehearsals) has none."""
    if override:
        return None
    tag = config if sites == CONFIGS[config]["sites"] else "%s_s%d" % (config, sites)
    return tag + ("_lnl" if lnl_only else "")


def latest_kernel_stats(tag, kernel="k_prune"):
    """(average ns, calls, file) of the traversal kernel in the newest
    profiles/r*_<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats)."""
    import csv
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_%s_kernel_stats.csv" % tag))) \
        if tag else []
    if not fs:
        return None
    try:
        for row in csv.DictReader(open(fs[-1])):
            if kernel in row["Name"]:
                return float(row["AverageNs"]), int(row["Calls"]), os.path.basename(fs[-1])
    except (OSError, ValueError, KeyError):
        return None
    return None


def traversal_roofline(ctx, ev, tag, alg_bytes, updates, K, lnl_only=False):
    """roofline object of the traversal kernel.  `achieved` uses bytes the kernel actually
    moves: the PMC traffic per launch when profiles/ holds it for this config, else the
    plan's compulsory bytes (pu_ctx_traffic: every kept parent and non-zero scaler tile
    written once, tip codes and read-backs read once).  SURVEY 8(d)'s algorithmic figure
    (tips as dense CLVs, three scalers per update) is reported beside it as `alg_ratio` --
    it is not a roofline: the fused kernel keeps children in registers and LDS and never
    moves those bytes."""
    from phylo_utils_amd import _native as N
    t = np.zeros(5, dtype=np.int64)
    N.check(N.lib().pu_ctx_traffic(ctx, N.ptr(t)), ctx)
    traffic, tfile = latest_traffic(tag)
    r = roofline_object(t, ev, traffic, tfile, alg_bytes, updates, K, lnl_only,
                        latest_pmc(tag) if lnl_only else None)
    ks = latest_kernel_stats(tag, "k_prune")
    if ks:
        r["rocprof_check"] = rocprof_check(r, ks, traffic, updates, K)
    return r


def rocprof_check(r, ks, traffic, updates, K):
    """The same roofline fraction on the rocprofv3 average duration of the committed kernel
    stats (profiles/), beside the live event median: the two must agree."""
    avg_ns, calls, fname = ks
    s = avg_ns * 1e-9
    out = {"file": fname, "calls": calls, "avg_ms": round(avg_ns * 1e-6, 5),
           "event_median_ms": r["kernel_ms"]}
    if K == 20:
        out["frac"] = round(updates * 4 * K * K / s / 1e12 / FP64_MFMA_PEAK_TFS, 4)
    elif r["bound"] == "valu":
        out["frac"] = round(updates * (4 * K * K + 2 * K - 1) / s / 1e12 / FP64_VALU_PEAK_TFS, 4)
    elif traffic:
        out["frac"] = round(traffic / s / 1e9 / HBM_PEAK_GBS, 4)
    return out


def roofline_object(t, ev, traffic, tfile, alg_bytes, updates, K, lnl_only=False, pmc=None):
    """traversal_roofline's arithmetic (pure; tests/test_bench.py): t = pu_ctx_traffic's five
    compulsory byte counts, ev = event_times(), traffic = PMC bytes per launch or None."""
    compulsory = int(np.sum(t))
    kern_s = ev["trav_med"] * 1e-3
    moved = traffic if traffic else compulsory
    gbs = moved / kern_s / 1e9
    common = {"kernel_ms": ev["trav_med"], "events": ev["n"],
              "bytes_basis": ("PMC 2*FETCH_SIZE + WRITE_SIZE per launch, profiles/%s" % tfile)
              if traffic else "compulsory bytes of the plan (no PMC file for this config)",
              "compulsory_bytes_per_launch": compulsory,
              "compulsory": {"clv_writes": int(t[0]), "scaler_writes": int(t[1]),
                             "tip_reads": int(t[2]), "readbacks": int(t[3]),
                             "site_lnl_and_weights": int(t[4])},
              "compulsory_frac": round(compulsory / kern_s / 1e9 / HBM_PEAK_GBS, 4),
              "alg_ratio": {"alg_bytes_per_launch": alg_bytes,
                            "alg_bytes_per_s_over_peak": round(alg_bytes / kern_s / 1e9 /
                                                               HBM_PEAK_GBS, 4),
                            "note": "SURVEY 8(d) M3 algorithmic bytes (8*(3K+3) per update, "
                                    "tips as dense fp64) over the kernel time -- NOT a "
                                    "roofline fraction: the fused kernel never moves them"}}
    if K == 20:
        # k_prune_mfma is fp64-MFMA-bound: per update 2 children x 2K^2 flop,
        # exactly what its 16-row + 4-row tiling executes
        flop = updates * 2 * 2 * K * K
        tfs_ach = flop / kern_s / 1e12
        return dict({"bound": "mfma", "achieved": round(tfs_ach, 2), "peak": FP64_MFMA_PEAK_TFS,
                     "unit": "TFLOP/s", "frac": round(tfs_ach / FP64_MFMA_PEAK_TFS, 4),
                     "traffic": traffic, "kernel": "k_prune_mfma", "flop_per_launch": flop,
                     "hbm_GBps": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)},
                    **common)
    # the fp64 VALU side of the same launch (2*2K^2 + K + (K-1) flop per
    # update); informative when few bytes move (lnL-only traversals)
    vflop = updates * (4 * K * K + 2 * K - 1)
    vtf = vflop / kern_s / 1e12
    common["fp64_valu"] = {"flop_per_launch": vflop, "achieved_TFs": round(vtf, 2),
                           "peak_TFs": FP64_VALU_PEAK_TFS,
                           "frac": round(vtf / FP64_VALU_PEAK_TFS, 4)}
    if lnl_only:
        # an lnL-only DNA traversal stores almost nothing: its binding roof is instruction
        # issue (the fp64 FMA chain plus the per-op scalar chain), not HBM
        issue = None
        if pmc:
            per = {k: round(v / updates, 4) for k, v in pmc.items()
                   if k.startswith("SQ_INSTS") and isinstance(v, (int, float))}
            issue = {"per_update": per, "source": "profiles/%s" % pmc["file"],
                     "note": "wave-instructions per (site, category, node) update = per-wave "
                             "count / 64 sites"}
            for k in ("SQ_BUSY_CU_CYCLES", "SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU"):
                if k in pmc:
                    issue[k] = pmc[k]
        return dict({"bound": "valu", "achieved": round(vtf, 2), "peak": FP64_VALU_PEAK_TFS,
                     "unit": "TFLOP/s", "frac": round(vtf / FP64_VALU_PEAK_TFS, 4),
                     "traffic": traffic, "kernel": "k_prune (lnL only)",
                     "flop_per_update": 4 * K * K + 2 * K - 1,
                     "hbm_GBps": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                     "issue": issue}, **common)
    return dict({"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": "k_prune"},
                **common)


def host_cpu_info():
    """The GPU box's host CPU as lscpu reports it, and the CPUs this process may use."""
    import subprocess
    info = {}
    try:
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in txt.splitlines():
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core",
                     "CPU(s)"):
                info[k] = v
    except (OSError, subprocess.SubprocessError):
        pass
    out = {"model": info.get("Model name"), "logical_cpus": info.get("CPU(s)"),
           "sockets": info.get("Socket(s)"), "cores_per_socket": info.get("Core(s) per socket"),
           "threads_per_core": info.get("Thread(s) per core")}
    try:
        out["physical_cores"] = int(out["sockets"]) * int(out["cores_per_socket"])
    except (TypeError, ValueError):
        out["physical_cores"] = None
    try:
        out["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        out["affinity_cpus"] = os.cpu_count()
    out["omp_num_threads_env"] = os.environ.get("OMP_NUM_THREADS")
    return out


def make_model(cfg):
    from phylo_utils_amd import substitution_models as SM
    from phylo_utils_amd.synthetic import CFG2_FREQS, CFG2_GTR_RATES
    if cfg["subst"].startswith("GTR"):
        return SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    return SM.LG()


STRONG_BLOCK = 125_000  # sites per simulation block of the strong-scaling alignment


def strong_slice(total, world, rank):
    """[lo, hi): the contiguous sites rank `rank` of `world` owns in the strong form."""
    return total * rank // world, total * (rank + 1) // world


def strong_alignment(tree, model, rates, total, lo, hi, block=STRONG_BLOCK):
    """(names, codes [ntaxa][hi - lo]) of sites [lo, hi) of the `total`-site alignment that is
    simulated on `tree` in blocks of `block` sites, block b from seed 1000 + b -- the same
    alignment for every rank count (block r is also rank r's weak-scaling cfg4 shard)."""
    if not 0 <= lo < hi <= total:
        raise ValueError("bad site range [%d, %d) of %d" % (lo, hi, total))
    names, parts = None, []
    for b in range(lo // block, (hi - 1) // block + 1):
        b0 = b * block
        n = min(block, total - b0)
        nm, codes = strong_block(tree, model, rates, b, n, block)
        if names is None:
            names = nm
        parts.append(codes[:, max(lo, b0) - b0:min(hi, b0 + n) - b0])
    return names, np.ascontiguousarray(np.concatenate(parts, axis=1))


# bump when synthetic.simulate_states changes what it draws (PU_BENCH_CACHE keys on it)
STRONG_SIM_VERSION = 1


def strong_block(tree, model, rates, b, n, block=STRONG_BLOCK):
    """(names, codes [ntaxa][n]) of block b of the strong alignment (seed 1000 + b).
    PU_BENCH_CACHE=<dir>: blocks are kept as .npy files there (scripts/presim.py fills it in
    parallel before the profiling runs of one GPU call, which would otherwise each spend
    ~15 s per 125k-site block of a 1000-taxon tree simulating)."""
    from phylo_utils_amd.synthetic import simulate_states
    cache = os.environ.get("PU_BENCH_CACHE")
    ntax = len(tree.leaf_nodes())
    path = None
    if cache:
        # keyed on everything the block depends on: the tree (topology and lengths), the
        # model's rates and frequencies, the category rates, the block and the simulator
        import hashlib
        key = repr((tree.as_newick(), np.asarray(model.q()).round(15).tolist(),
                    np.asarray(model.freqs).round(15).tolist(),
                    np.asarray(rates).round(15).tolist(), STRONG_SIM_VERSION))
        digest = hashlib.sha1(key.encode()).hexdigest()[:12]
        path = os.path.join(cache, "strong_t%d_b%d_n%d_blk%d_%s.npy" % (ntax, b, n, block,
                                                                         digest))
    names = ["t%d" % i for i in range(ntax)]
    if path and os.path.exists(path):
        return names, np.load(path)
    st = simulate_states(np.random.default_rng(1000 + b), tree, model, rates, n)
    log("[bench] simulated block %d (%d sites)" % (b, n))
    nm = sorted(st, key=lambda x: int(x[1:]))
    assert nm == names, "leaf labels are t0..t{N-1}"
    codes = np.stack([st[k] for k in nm]).astype(np.uint8)
    if path:
        os.makedirs(cache, exist_ok=True)
        tmp = path + ".%d.tmp.npy" % os.getpid()
        np.save(tmp, codes)
        os.replace(tmp, path)
    return names, codes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--warm-seconds", type=float, default=2.0,
                    help="after the W warmup steps keep running untimed steps for at least "
                         "this long, so the GPU clocks are up before the timed region")
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--sites", type=int, default=0,
                    help="override the config's sites per GPU (tests and rehearsals only; the "
                         "reported workload is the config's)")
    ap.add_argument("--total-sites", type=int, default=0,
                    help="strong scaling (cfg2 / cfg4 traversal): one alignment of this many "
                         "sites split over the ranks (BASELINE cfg4: 1000000), instead of "
                         "`sites` per rank")
    ap.add_argument("--trees", type=int, default=0,
                    help="cfg5: trees per rank (override; default the config's 125)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ceiling", action="store_true",
                    help="skip the same-device write-ceiling probe of the roofline")
    ap.add_argument("--no-rank-check", action="store_true",
                    help="skip the multi-rank oracle check of the job's lnL (world > 1)")
    ap.add_argument("--events", choices=["timed", "separate"], default="separate",
                    help="where the per-launch HIP events for the roofline are recorded: in "
                         "the timed steps (timed) or in a second pass of the same steps right "
                         "after them, so that the event packets do not sit in the timed "
                         "region (separate, default: they cost 7-10 us per step inside it)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the C baseline (0: every CPU this rank may use, capped by "
                         "OMP_NUM_THREADS when set)")
    ap.add_argument("--numpy-seconds", type=float, default=8.0)
    ap.add_argument("--lnl-only", action="store_true",
                    help="PU_LNL_ONLY: do not keep every internal CLV in HBM")
    ap.add_argument("--workload", default="traversal",
                    choices=["traversal", "edges", "patterns"],
                    help="edges: branch-length derivatives on the resident CLVs and one "
                         "optimising-traversal sweep (SURVEY 8(f) N1) instead of the "
                         "headline traversal")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.sites:
        cfg["sites"] = args.sites
        cfg["desc"] += " [--sites %d override]" % args.sites
    if args.trees and "trees" in cfg:
        cfg["trees"] = args.trees
        cfg["desc"] += " [--trees %d override]" % args.trees
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher around us: start the N ranks ourselves (nothing has touched the GPU)
        sys.exit(spawn_ranks(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    import torch
    import torch.distributed as dist
    # PU_BENCH_BACKEND=gloo: rehearsal of the multi-rank path with several ranks on one GPU
    # (RCCL refuses two ranks on one device); the measured runs use RCCL ("nccl")
    backend = os.environ.get("PU_BENCH_BACKEND", "nccl")
    n_dev = torch.cuda.device_count()
    if n_dev < 1:
        sys.exit("bench.py: no HIP device visible")
    if backend == "nccl" and local_rank >= n_dev:
        sys.exit("bench.py: rank %d (local %d) has no GPU of its own: %d visible for %d "
                 "ranks per node (RCCL needs one GPU per rank; PU_BENCH_BACKEND=gloo "
                 "rehearses several ranks on one GPU)" % (rank, local_rank, n_dev, world))
    gpu = local_rank if backend == "nccl" else local_rank % n_dev
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    # A stream of our own as torch's current stream, handed to pu_ctx_set_stream, so that the
    # context's kernels and the lnL collective run in one stream order.  (Before r03's fix
    # pu_ctx_set_stream read handle 0 -- torch's default stream -- as "the context's own
    # stream", and the collective could sum a slot before k_reduce wrote it; NULL now means
    # the HIP null stream and PU_OWN_STREAM the context's own.  A stream of our own also keeps
    # the null stream's implicit synchronisation out of the timed steps.)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
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
    ntax = cfg["ntax"]
    t_setup = time.time()
    tree = random_tree(np.random.default_rng(1234), ntax)          # same tree on every rank
    strong = args.total_sites > 0
    if strong:
        if args.total_sites < world:
            sys.exit("bench.py: --total-sites must be >= the rank count")
        lo, hi = strong_slice(args.total_sites, world, rank)
        names, codes = strong_alignment(tree, model, rm.rates, args.total_sites, lo, hi)
        S = hi - lo
    else:
        S = cfg["sites"]
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
    if strong:
        log("[bench] rank %d owns sites [%d, %d) of %d: local lnL %.10f" %
            (rank, lo, hi, args.total_sites, tm.likelihood()))

    if args.workload == "edges":
        if rank == 0:
            print(json.dumps(bench_edges(tm, model, rm, codes, K, C, S, ntax, args, cfg)),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    def all_reduce_async(t):
        if backend != "nccl":
            # gloo (one-GPU rehearsal) copies the tensor from its own thread: make sure the
            # kernels that wrote it have finished (RCCL is ordered on the stream itself)
            torch.cuda.current_stream(dev).synchronize()
        return dist.all_reduce(t, async_op=True)

    ring = LnlRing(lambda: torch.zeros(1, dtype=torch.float64, device=dev), world,
                   all_reduce_async)
    ptrs = [ctypes.c_void_p(t.data_ptr()) for t in ring.slots]
    stream = torch.cuda.current_stream(dev)
    N.check(N.lib().pu_ctx_set_stream(ctx, ctypes.c_void_p(stream.cuda_stream)), ctx)
    enqueue = N.lib().pu_enqueue
    set_out = N.lib().pu_set_lnl_device_output

    def fill_eager(slot):  # one evaluation, its lnL into ring slot `slot`
        set_out(ctx, ptrs[slot])
        rc = enqueue(ctx)
        if rc:
            N.check(rc, ctx, "pu_enqueue")

    # PU_BENCH_GRAPH=1: one HIP graph per lnL slot (P, traversal, reduce on the context's
    # stream, forked from and joined into the capture stream), replayed per step.  Off by
    # default: the GPU, not the host, paces these steps, and a replay cost more than three
    # launches (r03: cfg2 0.149-0.150 vs 0.142-0.144 ms per step, cfg3 0.356-0.360 vs
    # 0.355-0.356).  (--events timed records events inside pu_enqueue: always eager.)
    graphs = None
    if os.environ.get("PU_BENCH_GRAPH", "0") == "1" and args.events != "timed":
        try:
            gs = []
            for slot in range(len(ptrs)):
                fill_eager(slot)  # first-call work outside the capture
                torch.cuda.synchronize(dev)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    cs = torch.cuda.current_stream(dev)
                    ev = torch.cuda.Event()
                    ev.record(cs)
                    stream.wait_event(ev)
                    set_out(ctx, ptrs[slot])
                    rc = enqueue(ctx)
                    if rc:
                        N.check(rc, ctx, "pu_enqueue")
                    cs.wait_stream(stream)
                gs.append(g)
            graphs = gs
        except Exception as e:  # capture unsupported here: eager launches
            log("[bench] graph capture failed (%s); eager launches" % e)
            torch.cuda.synchronize(dev)

    mode = {"graph": graphs is not None}

    def fill(slot):
        if mode["graph"]:
            graphs[slot].replay()
        else:
            fill_eager(slot)

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
    # HIP events around every traversal launch, on the launch stream: in the timed steps
    # (--events timed) or in a second pass of the same number of steps (--events separate)
    if args.events == "timed":
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
    if args.events == "separate":
        mode["graph"] = False  # the events are recorded by pu_enqueue itself
        N.check(N.lib().pu_ctx_profile(ctx, 1), ctx)
        for _ in range(args.steps):
            step()
        drain()

    ev = event_times(ctx, args.steps)
    N.check(N.lib().pu_ctx_profile(ctx, 0), ctx)
    torch.cuda.synchronize(dev)

    updates_per_step = (ntax - 1) * S * C       # (N-2) ops + root combine, per rank
    # the job's updates per step: every rank's (weak: equal shards; strong: T sites in all)
    job_updates = (ntax - 1) * args.total_sites * C if strong else updates_per_step * world
    total_updates = job_updates * args.steps
    value = total_updates / elapsed / 1e6
    # 8*(3K+3) B per update (2 child CLVs + parent + 3 scalers, tips as
    # dense fp64) + root scalers read + sitewise output
    alg_bytes = updates_per_step * 8 * (3 * K + 3) + S * C * 8 + S * 8
    tag = pmc_tag(args.config, S, args.lnl_only, override=bool(args.sites))
    roofline = traversal_roofline(ctx, ev, tag, alg_bytes, updates_per_step, K, args.lnl_only)
    roofline["events_pass"] = ("a second pass of the same %d steps right after the timed one"
                               % args.steps if args.events == "separate"
                               else "the timed steps")
    if roofline.get("unit") == "GB/s" and not args.no_ceiling:
        # the same device's write-stream ceiling for the bytes one launch moves, after the
        # timed steps (r06): how far this box's HBM lets any store stream go, so that a slow
        # box shows as a low ceiling and a slow kernel as a low frac_of_ceiling
        nbytes = int(roofline["traffic"] or roofline["compulsory_bytes_per_launch"])
        cms = ctypes.c_double()
        N.check(N.lib().pu_write_ceiling(dev.index, nbytes, 50, ctypes.byref(cms)), None,
                "pu_write_ceiling")
        ceil_gbs = nbytes / (cms.value * 1e-3) / 1e9
        roofline["ceiling_GBps"] = round(ceil_gbs, 1)
        roofline["frac_of_ceiling"] = round(roofline["achieved"] / ceil_gbs, 4)
        roofline["ceiling_probe"] = ("hipMemsetAsync of the launch's %d bytes, median of 50 after "
                                     "3 warm-ups (pu_write_ceiling): the fastest write stream "
                                     "measured on MI355X (DESIGN 4.1)" % nbytes)
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "M updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded random-joining tree, alignment simulated under the model)",
        "config": {"workload": (("BASELINE %s as stated: one %d-site alignment split over the "
                                 "ranks (%d taxa)" % (args.config, args.total_sites, ntax))
                                if strong else cfg["desc"]),
                   "config": args.config, "substitution": cfg["subst"],
                   "taxa": ntax, "sites_per_gpu": S,
                   "total_sites": args.total_sites if strong else S * world,
                   "categories": C, "states": K,
                   "updates_per_step": job_updates,
                   "partials": "lnl_only" if args.lnl_only else "all internal CLVs kept in HBM",
                   "launch": "HIP graph of the step's launches, replayed per step"
                             if graphs is not None else "eager launches",
                   "parallelism": "site-sharded x%d, RCCL lnL all-reduce overlapped with the "
                                  "next step's kernels" % world},
        "roofline": roofline,
        "timing": {"source": "hipEvents on the launch stream around each timed step",
                   "runs": ev["n"], "step_ms_median": ev["step_med"],
                   "kernel_ms_median": ev["trav_med"], "kernel_ms_mean": ev["trav_mean"],
                   "value_at_step_median": round(job_updates / (ev["step_med"] * 1e-3) / 1e6,
                                                 3)},
        "lnl": lnl_total,
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        site_gpu = np.zeros(S)
        N.check(N.lib().pu_get_site_lnl(ctx, N.ptr(site_gpu)), ctx)
        cpu, acc = cpu_baseline(tm, model, rm, codes, K, C, S, ntax, args, lnl_total, site_gpu)
        out["cpu_baseline"] = cpu
        out.update(acc)
    if world > 1 and not args.no_rank_check:
        # every rank checks its own shard against the oracle; the job's lnL (the all-reduced
        # GPU sum) against the all-reduced oracle sums, and the ranks the collective spans
        site_gpu = np.zeros(S)
        N.check(N.lib().pu_get_site_lnl(ctx, N.ptr(site_gpu)), ctx)
        tc = time.perf_counter()
        cpu_lnl, site_cpu, _ = oracle_traversal(tm, model, rm, codes,
                                                cpu_threads(args, host_cpu_info()))
        site_rel = float(np.max(np.abs(site_gpu - site_cpu) / np.abs(site_cpu)))
        chk = rank_check(dist, dev, world, lnl_total, cpu_lnl, site_rel,
                         "%d-site shard" % S)
        chk["oracle_seconds_rank0"] = round(time.perf_counter() - tc, 2)
        out["rank_check"] = chk
        out["rccl_world"] = chk["rccl_world"]
        out["lnl_rel_err_vs_cpu"] = chk["lnl_rel_err_vs_cpu"]
        out["sitewise_max_rel_err_vs_cpu"] = chk["sitewise_max_rel_err_vs_cpu"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


_ORACLE_BUFS = {}


def oracle_traversal(tm, model, rm, codes, threads, block=32768):
    """One whole traversal of `tm`'s tree over `codes` ([ntaxa][S] uint8, rows in tm.names
    order) by the C oracle, in site blocks of `block` (bounded host memory: partials
    [n_nodes][block][C][K] fp64, reused between calls of the same shape).  Returns (lnL,
    site_lnl [S], seconds in P generation + traversal calls -- the tip fill, which the GPU's
    resident tips never pay per tree, excluded); pattern weights 1.  Outside every timed
    region: the checker, not the path."""
    from oracle import oracle as orc
    tr = tm.traversal
    K, C, S = len(model.freqs), rm.ncat, codes.shape[1]
    n_nodes = tr.n_nodes
    # at most ~1 GB of host buffers per process (8 ranks of a node run this at once)
    B = min(S, block, max(512, int(1e9 // (n_nodes * C * (K + 1) * 8))))
    key = (n_nodes, B, C, K)
    if key not in _ORACLE_BUFS:
        _ORACLE_BUFS.clear()
        _ORACLE_BUFS[key] = (np.zeros((n_nodes, B, C, K)), np.zeros((n_nodes, B, C)))
    partials, scale = _ORACLE_BUFS[key]
    ev, el, iv = model.engine_eigen()
    ops = np.ascontiguousarray(tr.postorder_traversal, dtype=np.int32)
    bl = tr.op_lengths()
    rates = np.ascontiguousarray(rm.rates)
    t_c = time.perf_counter()
    P = np.ascontiguousarray(orc.pmatrix_c(ev, el, iv, bl.reshape(-1), rates)
                             .reshape(len(ops), 2, C, K, K))
    Pr = np.ascontiguousarray(orc.pmatrix_c(ev, el, iv, np.array([0.0, tr.root_length()]),
                                            rates))
    fr = np.ascontiguousarray(model.freqs, dtype=np.float64)
    w = np.ascontiguousarray(rm.weights)
    eye = np.eye(K)
    site = np.zeros(S)
    total = 0.0
    t_compute = time.perf_counter() - t_c
    for lo in range(0, S, B):
        n = min(B, S - lo)
        part, sc = partials[:, :n], scale[:, :n]
        if n < B:  # the last, shorter block: contiguous buffers of its own size
            part, sc = np.zeros((n_nodes, n, C, K)), np.zeros((n_nodes, n, C))
        for name, node in tr.names.items():
            part[node] = eye[codes[tm.names[name], lo:lo + n]][:, None, :]
            sc[node] = 0.0  # (the reused buffers: this node may have been internal before)
        out = np.zeros(n)
        t_c = time.perf_counter()
        total += orc.traverse_prepared(K, C, n, ops, P, Pr, tr.root_edge, part, sc, fr, w,
                                       np.ones(n), threads, site_lnl=out)
        t_compute += time.perf_counter() - t_c
        site[lo:lo + n] = out
    return total, site, t_compute


def rank_check(dist, dev, world, gpu_job_lnl, cpu_lnl, site_rel, what, gpu_local=False):
    """Multi-rank self-check (r06), outside the timed region: the ranks the collective really
    spans (an all-reduce of ones over the process group, RCCL under --backend nccl) and the
    job's lnL against the C oracle's (each rank's share all-reduced the same way)."""
    import torch
    one = torch.ones(1, dtype=torch.float64, device=dev)
    dist.all_reduce(one)
    c = torch.tensor([cpu_lnl], dtype=torch.float64, device=dev)
    dist.all_reduce(c)
    m = torch.tensor([site_rel], dtype=torch.float64, device=dev)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    cpu_job = float(c.item())
    if gpu_local:  # the rank's own GPU sum: the job's by the same collective
        g = torch.tensor([gpu_job_lnl], dtype=torch.float64, device=dev)
        dist.all_reduce(g)
        gpu_job_lnl = float(g.item())
    return {"rccl_world": int(round(one.item())), "backend": str(dist.get_backend()),
            "lnl_job_gpu": gpu_job_lnl, "lnl_job_cpu": cpu_job,
            "lnl_rel_err_vs_cpu": abs(gpu_job_lnl - cpu_job) / abs(cpu_job),
            "sitewise_max_rel_err_vs_cpu": float(m.item()),
            "oracle": "oracle/pruning_oracle.c on every rank's own %s, after the timed steps; "
                      "the CPU lnLs summed by the same collective" % what}


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
    # PU_BENCH_BATCH=1 (default): every tree in one launch of each kernel (pu_batch, r05:
    # 511 G updates/s); 0: one P / traversal / reduce launch per tree, spread over
    # PU_BENCH_STREAMS streams (456 G, same box, alternating; profiles/r05_batch_ab/)
    # PU_BENCH_BATCH=k > 1: k batches of T / k trees, one per stream
    n_batch = int(os.environ.get("PU_BENCH_BATCH", "1") or 0)
    use_batch = n_batch >= 1
    n_streams = n_batch if use_batch else int(os.environ.get("PU_BENCH_STREAMS", "4"))
    streams = [torch.cuda.Stream(dev) for _ in range(n_streams)]
    lnl = torch.zeros(T, dtype=torch.float64, device=dev)
    tms = []
    # one resident alignment per GPU (r06): tree 0 uploads the tips, every
    # other tree reads them in place (TreeModel.share_alignment / pu_share_tips), so a batch's
    # trees fetch one copy of the codes.  PU_BENCH_SHARE=0: a copy per tree (r05), for the A/B
    share = os.environ.get("PU_BENCH_SHARE", "1") == "1"
    for i in range(T):
        tree = random_tree(np.random.default_rng(10_000 + rank * T + i), ntax)
        tm = TreeModel(device=dev.index, keep_partials=False)
        if share and tms:
            tm.share_alignment(tms[0])
        else:
            tm.set_alignment_codes(codes, np.eye(K), names)
        tm.set_substitution_model(model)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        ctx = tm._ctx
        sidx = (i * n_batch // T) if use_batch else i % n_streams  # a batch's trees: one stream
        N.check(lib.pu_ctx_set_stream(ctx, ctypes.c_void_p(streams[sidx].cuda_stream)),
                ctx)
        N.check(lib.pu_set_lnl_device_output(ctx, ctypes.c_void_p(lnl.data_ptr() + 8 * i)),
                ctx)
        tms.append(tm)
    log("[bench] rank %d: %d trees set up in %.1fs" % (rank, T, time.time() - t_setup))
    ref = np.array([tm.likelihood() for tm in tms])  # synchronous pu_run values
    tbatch, tbatches, bounds = None, [], []
    if use_batch:
        from phylo_utils_amd.batch import TreeBatch
        for k in range(n_batch):  # trees [lo, hi) of batch k, contiguous in the lnL vector
            lo, hi = k * T // n_batch, (k + 1) * T // n_batch
            tb = TreeBatch(tms[lo:hi])
            tb.set_stream(streams[k].cuda_stream)
            tbatches.append(tb)
            bounds.append((lo, hi))
        tbatch = tbatches[0]
    gathered = [torch.empty_like(lnl) for _ in range(world)] if world > 1 else None
    main_stream = torch.cuda.current_stream(dev)

    def launches(origin):
        # every tree's P, traversal and reduce, forked from `origin` over the streams and
        # joined back into it
        ev = torch.cuda.Event()
        ev.record(origin)
        for st in streams:
            st.wait_event(ev)
        if tbatch is not None:
            for tb, (lo, _) in zip(tbatches, bounds):
                tb.enqueue(lnl.data_ptr() + 8 * lo)
        else:
            for tm in tms:
                rc = lib.pu_enqueue(tm._ctx)
                if rc:
                    N.check(rc, tm._ctx, "pu_enqueue")
        for st in streams:
            origin.wait_stream(st)

    # The step's 3 x 125 launches are captured once in a HIP graph and replayed (every kernel
    # runs every step; only the host-side launch cost goes): the eager step is paced by the
    # host's 375 launches (r03: 302 -> 425 G updates/s, lnL identical).  PU_BENCH_GRAPH=0:
    # eager.
    graph = None
    if os.environ.get("PU_BENCH_GRAPH", "1") == "1":
        launches(main_stream)  # allocations and first-call work before capture
        torch.cuda.synchronize(dev)
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                launches(torch.cuda.current_stream(dev))
            graph = g
        except Exception as e:  # capture unsupported here: eager launches
            log("[bench] graph capture failed (%s); eager launches" % e)
            graph = None
            torch.cuda.synchronize(dev)

    def step():
        if graph is not None:
            graph.replay()
        else:
            launches(main_stream)
        if world > 1:
            if os.environ.get("PU_BENCH_BACKEND", "nccl") != "nccl":
                torch.cuda.current_stream(dev).synchronize()  # gloo: see all_reduce_async
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
    # the oracle on this rank's trees (as many as fit --cpu-seconds; every tree at cfg5's
    # size): rank 0 of a one-GPU run reports it as cpu_baseline, every rank of a multi-rank
    # run feeds rank_check.  After the timed steps.
    cpu_part = None
    if (world == 1 and rank == 0 and not args.no_cpu_baseline) or \
            (world > 1 and not args.no_rank_check):
        threads = cpu_threads(args, host_cpu_info())
        oracle_traversal(tms[0], model, rm, codes[:, :64], threads)  # library load, warm
        n_chk, rel_chk, cpu_sum, gpu_sum, el_c = 0, 0.0, 0.0, 0.0, 0.0
        tc = time.perf_counter()
        for i in range(T):
            lo_, _, t_i = oracle_traversal(tms[i], model, rm, codes, threads)
            rel_chk = max(rel_chk, abs(got[i] - lo_) / abs(lo_))
            cpu_sum += lo_
            gpu_sum += float(got[i])
            el_c += t_i
            n_chk += 1
            if time.perf_counter() - tc >= args.cpu_seconds:
                break
        cpu_part = (n_chk, rel_chk, cpu_sum, gpu_sum, el_c, threads)
    ctx0 = tms[0]._ctx
    upd_tree = (ntax - 1) * S * C
    value = upd_tree * T * world * args.steps / elapsed / 1e6
    alg = upd_tree * 8 * (3 * K + 3) + S * C * 8 + S * 8
    n_ev = max(20, min(args.steps, 200))
    if tbatch is not None:
        # the batched traversal launch (all T trees), events around it on the batch's stream
        tbatch._check(lib.pu_batch_profile(tbatch._b, 1), "pu_batch_profile")
        for _ in range(n_ev):
            tbatch.enqueue(lnl.data_ptr())  # batch 0 alone
        tr, tot = np.zeros(n_ev), np.zeros(n_ev)
        n = ctypes.c_int()
        tbatch._check(lib.pu_batch_kernel_times(tbatch._b, N.ptr(tr), N.ptr(tot), n_ev,
                                               ctypes.byref(n)), "pu_batch_kernel_times")
        tbatch._check(lib.pu_batch_profile(tbatch._b, 0), "pu_batch_profile")
        tr, tot = tr[:n.value], tot[:n.value]
        ev = {"n": n.value, "trav_med": round(float(np.median(tr)), 5),
              "trav_mean": round(float(tr.mean()), 5), "step_med": round(float(np.median(tot)), 5)}
        # compulsory bytes summed over batch 0's trees (each tree's own plan: its stored ops and
        # read-backs differ; r05-r06 early took 125 x tree 0's)
        lo0, hi0 = bounds[0]
        tsum = np.zeros(5, dtype=np.int64)
        for tm in tms[lo0:hi0]:
            t = np.zeros(5, dtype=np.int64)
            N.check(lib.pu_ctx_traffic(tm._ctx, N.ptr(t)), tm._ctx)
            tsum += t
        tag = None if args.sites else "cfg5_batch"
        if n_batch > 1:
            tag = None
        traffic, tfile = latest_traffic(tag)
        m0 = bounds[0][1] - bounds[0][0]  # trees in batch 0, timed alone
        if n_batch > 1:
            tag = None  # the PMC / rocprof files are for one batch of all T trees
        tb = tsum
        if share:  # one resident copy of the tip codes, read by every tree of the batch
            tb[2] = t[2]
        roofline = roofline_object(tb, ev, traffic, tfile, alg * m0, upd_tree * m0, K, True,
                                   latest_pmc(tag))
        ks = latest_kernel_stats(tag, "k_prune_trees")
        if ks:
            roofline["rocprof_check"] = rocprof_check(roofline, ks, traffic, upd_tree * m0, K)
        roofline["kernel"] = "k_prune_trees"
        roofline["note"] = ("the batched traversal of %d trees per launch (pu_batch, batch 0 of "
                            "%d timed alone); compulsory bytes summed over its %d trees' plans%s"
                            % (m0, n_batch, m0, ", tip codes once (shared)" if share else ""))
    else:
        # per-launch kernel time of one context, measured with events on its stream
        N.check(lib.pu_ctx_profile(ctx0, 1), ctx0)
        for _ in range(n_ev):
            N.check(lib.pu_enqueue(ctx0), ctx0)
        ev = event_times(ctx0, n_ev)
        N.check(lib.pu_ctx_profile(ctx0, 0), ctx0)
        roofline = traversal_roofline(ctx0, ev, None if args.sites else "cfg5_lnl", alg, upd_tree,
                                      K, lnl_only=True)
        roofline["note"] = ("one tree's launch measured alone; the step overlaps %d streams"
                            % n_streams)
    torch.cuda.synchronize(dev)
    extra = {}
    if cpu_part is not None:
        n_chk, rel_chk, cpu_sum, gpu_sum, el_c, threads = cpu_part
        if world == 1:
            host = host_cpu_info()
            extra["cpu_baseline"] = {
                "value": round(upd_tree * n_chk / el_c / 1e6, 3), "unit": "M updates/s",
                "cores": threads, "kind": "port",
                "sample": "the first %d of the %d trees, one full traversal each "
                          "(oracle/pruning_oracle.c, OpenMP over site blocks of 32768, %d "
                          "threads, P matrices included; the per-tree tip fill of the host "
                          "buffers excluded, as the GPU's tips are resident)"
                          % (n_chk, T, threads),
                "host": host}
            extra["lnl_rel_err_vs_cpu"] = rel_chk
            extra["accuracy_trees"] = n_chk
        else:
            chk = rank_check(dist, dev, world, gpu_sum, cpu_sum, rel_chk,
                             "first %d trees (rank 0; bounded by --cpu-seconds)" % n_chk,
                             gpu_local=True)
            chk["note"] = ("lnl_job_* = the sums over the checked trees of every rank; "
                           "sitewise_max_rel_err_vs_cpu is the largest per-tree lnL rel-err")
            extra["rank_check"] = chk
            extra["rccl_world"] = chk["rccl_world"]
            extra["lnl_rel_err_vs_cpu"] = max(chk["lnl_rel_err_vs_cpu"],
                                              chk["sitewise_max_rel_err_vs_cpu"])
    return dict({
        "metric": METRIC, "value": round(value, 3), "unit": "M updates/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded random-joining trees, alignment simulated on another)",
        "config": {"workload": cfg["desc"], "config": "cfg5", "taxa": ntax, "sites": S,
                   "categories": C, "states": K, "trees_per_gpu": T, "total_trees": T * world,
                   "updates_per_step": upd_tree * T * world, "partials": "lnl_only",
                   "alignment": ("one resident copy per GPU, shared by every tree "
                                 "(pu_share_tips)" if share else "a copy per tree"),
                   "device_bytes_all_trees": int(sum(lib.pu_ctx_device_bytes(m._ctx)
                                                     for m in tms)),
                   "launch": ("%s, %s" % ("one batched launch per kernel for all trees "
                                          "(pu_batch)" if tbatch is not None else
                                          "one launch per kernel and tree",
                                          "captured in a HIP graph, replayed per step"
                                          if graph is not None else "eager")),
                   "parallelism": "tree-sharded x%d, %s, all-gather of the per-tree lnL"
                                  % (world, "batched" if tbatch is not None else
                                     "%d HIP streams per GPU" % n_streams)},
        "roofline": roofline,
        "lnl_max_rel_diff_vs_sync_runs": max_rel,
    }, **extra)


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
    # bytes k_edge moves: the PMC traffic per EDGE_DERIV launch when profiles/ holds it
    # (r*_traffic_<cfg>_edges.json, scripts/collect_profiles.py --kernel "k_edge<K, 2>"),
    # else the algorithmic figure (both ends' CLVs and scalers + pattern weights)
    traffic, tfile = latest_traffic(args.config + "_edges") if not args.sites else (None, None)
    moved = traffic if traffic else alg
    ach = moved / (ems.value * 1e-3) / 1e9  # k_edge alone (its reduction launch follows)
    def newton_stats():
        ln, ne = ctypes.c_int(), ctypes.c_int()
        N.check(lib.pu_ctx_newton_stats(ctx, ctypes.byref(ln), ctypes.byref(ne)), ctx)
        return ln.value, ne.value

    # (r06) the Newton optimiser's own evaluations: pu_optimise_edge runs newton()'s whole loop
    # in one persistent launch (k_edge_newton).  The root edge from several starting lengths
    # (set, and the traversal re-run, outside the timed calls); evaluations from the library's
    # counters, time host to host around each pu_optimise_edge.
    key = (min(a, b), max(a, b))
    tr_bl = tm.traversal.brlens
    k_root = key if key in tr_bl else (a, b)
    dn_time, dn_runs = 0.0, 0
    l_start, e_start = newton_stats()
    out_t, out_l = ctypes.c_double(), ctypes.c_double()
    for k in range(max(10, min(args.steps, 100))):
        tr_bl[k_root] = t0 * (0.5 + 0.25 * (k % 5))
        tm.update_branch_lengths()
        tm.likelihood()
        tc = time.perf_counter()
        N.check(lib.pu_optimise_edge(ctx, a, b, 1e-8, 50, ctypes.byref(out_t),
                                     ctypes.byref(out_l)), ctx)
        dn_time += time.perf_counter() - tc
        dn_runs += 1
    l_end, e_end = newton_stats()
    dn_launch, dn_evals = l_end - l_start, e_end - e_start

    # (r06) the reference's own minimisers (brent / dbrent, src/optimisation.pyx) through
    # pu_minimise_edge, over [1e-8, 10] from the same starting lengths: the device driver (one
    # persistent launch per call) and the host driver (PU_EDGE_DEVICE_NEWTON=0, one k_edge
    # launch per evaluation), evaluations = the reference's iteration count + its first one
    def minimise(method, device):
        os.environ["PU_EDGE_DEVICE_NEWTON"] = "1" if device else "0"
        tt, ne, out3 = 0.0, 0, np.zeros(3)
        for k in range(10):
            tr_bl[k_root] = t0 * (0.5 + 0.25 * (k % 5))
            tm.update_branch_lengths()
            tm.likelihood()
            tc = time.perf_counter()
            N.check(lib.pu_minimise_edge(ctx, a, b, method, 1e-8, tr_bl[k_root], 10.0, 1.5e-8,
                                         N.ptr(out3)), ctx)
            tt += time.perf_counter() - tc
            ne += int(out3[2]) + 1
        os.environ.pop("PU_EDGE_DEVICE_NEWTON", None)
        return {"us_per_call": round(tt / 10 * 1e6, 2), "evaluations_per_call": ne / 10,
                "us_per_evaluation": round(tt / ne * 1e6, 2)}
    mins = {name: {"device": minimise(code, True), "host": minimise(code, False)}
            for name, code in (("brent", 1), ("dbrent", 2))}
    tr_bl[k_root] = t0
    tm.update_branch_lengths()
    lnl0 = tm.likelihood()
    s_l0, s_e0 = newton_stats()
    ts = time.perf_counter()
    lnl1 = tm.optimise_branch_lengths(tol=1e-8, max_iter=50, sweeps=1)
    sweep_s = time.perf_counter() - ts
    s_l1, s_e1 = newton_stats()
    n_edges = 2 * ntax - 3
    dev_rate = dn_evals / dn_time if dn_launch and dn_evals else None
    res = {
        "metric": "edge evaluations/sec (lnL + dlnL/dt + d2lnL/dt2 over all sites) in the "
                  "Newton branch-length optimiser, GTR+G4; SURVEY 8(f) N1",
        "value": round(dev_rate if dev_rate else args.steps / el, 1),
        "unit": "evaluations/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round((dn_time / dn_evals if dev_rate else el / args.steps) * 1e3, 5),
        "higher_is_better": True,
        "device_newton": {"optimisations": dn_runs, "launches": dn_launch,
                          "evaluations": dn_evals,
                          "us_per_evaluation": round(dn_time / dn_evals * 1e6, 2)
                          if dn_evals else None,
                          "us_per_optimisation": round(dn_time / dn_runs * 1e6, 2),
                          "note": "value: evaluations inside pu_optimise_edge's persistent "
                                  "k_edge_newton launches over the host-to-host time of those "
                                  "calls (root edge, 5 starting lengths, tol 1e-8)"},
        "minimisers": dict(mins, note="pu_minimise_edge: the reference's brent / dbrent "
                           "(tol 1.5e-8, bracket [1e-8, 10]) on the root edge from 5 starting "
                           "lengths, host to host per call; device = one persistent launch per "
                           "call, host = one k_edge launch per evaluation"),
        "single_call": {"value": round(args.steps / el, 1), "unit": "evaluations/s",
                        "ms_per_call": round(el / args.steps * 1e3, 5),
                        "note": "pu_edge_derivs: one k_edge launch + host sum per call, host "
                                "to host (the brent / dbrent minimisers' unit)"},
        "scaling": "none", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": cfg["desc"] + "; edge derivatives on the root edge + one "
                   "optimising-traversal sweep", "config": args.config, "taxa": ntax,
                   "sites": S, "categories": C, "states": K},
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "kernel": "k_edge<%d, EDGE_DERIV>" % K, "kernel_ms": round(ems.value, 5),
                     "with_reduction_ms": round(kms.value, 5),
                     "events": nrec.value, "alg_bytes_per_launch": alg, "traffic": traffic,
                     "bytes_basis": ("PMC 2*FETCH_SIZE + WRITE_SIZE per launch, profiles/%s"
                                     % tfile) if traffic else "algorithmic bytes (no PMC file)"},
        "sweep": {"edges": n_edges, "ms": round(sweep_s * 1e3, 3),
                  "newton_launches": s_l1 - s_l0, "newton_evaluations": s_e1 - s_e0,
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
    # PMC bytes per compression, when a profile holds them (scripts/r05/patterns_traffic.py)
    traffic, traffic_src = latest_traffic("patterns")
    if traffic is None:
        tfs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic_patterns.json")))
        if tfs:
            try:
                traffic = json.load(open(tfs[-1])).get("hbm_bytes_per_call")
                traffic_src = os.path.basename(tfs[-1])
            except (OSError, ValueError):
                traffic = None
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
                     "kernel": "pu_compress_patterns_device (pack, prefix-refinement radix "
                               "sorts, scan, unpack)", "kernel_ms": round(ms, 4),
                     "alg_bytes_per_launch": alg,
                     "traffic": None if traffic is None else round(traffic),
                     "traffic_source": traffic_src},
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


def cpu_threads(args, host):
    """Threads of the C baseline: --cpu-threads, else every CPU this process may run on
    (affinity), capped by OMP_NUM_THREADS when the host sets it.  The GPU box leases each GPU
    a share of its host (16 CPUs per GPU, exported as OMP_NUM_THREADS; its run contract says
    to size worker pools to that share, not to the whole machine that nproc shows), so the
    measured baseline uses the share, and `all_physical_cores_projection` scales it to every
    physical core as an upper bound (linear scaling; not measured)."""
    if args.cpu_threads:
        return args.cpu_threads
    n = host.get("affinity_cpus") or os.cpu_count() or 1
    env = host.get("omp_num_threads_env")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, n)


def cpu_baseline(tm, model, rm, codes, K, C, S, ntax, args, gpu_lnl, site_gpu):
    """SURVEY 8(d) M4 on the GPU box's host: (a) the oracle's C restatement of the same loop
    nest, OpenMP over site blocks, on all the CPUs this rank may use; (b) the numpy-vectorised
    restatement (oracle.traverse_numpy) in one process on a bounded slice of the same sites.
    Both run whole traversals including P generation.  Also returns M1's accuracy figures:
    total lnL and sitewise max relative error of the GPU against (a) on the same inputs."""
    from oracle import oracle as orc
    tr = tm.traversal
    n_nodes = tr.n_nodes
    S_full = S
    # bounded host memory (partials [n_nodes][S][C][K] fp64): at most 125k sites -- the whole
    # workload for every config but the strong-scaling cfg4 on few ranks
    S = min(S, STRONG_BLOCK)
    codes = codes[:, :S]
    host = host_cpu_info()
    threads = cpu_threads(args, host)
    log("[bench] cpu baseline: %d threads, ~%.0fs (host %s)" % (threads, args.cpu_seconds, host))
    partials = np.zeros((n_nodes, S, C, K))
    scale = np.zeros((n_nodes, S, C))
    eye = np.eye(K)
    tip_rows = {}
    for name, node in tr.names.items():
        tip_rows[node] = eye[codes[tm.names[name]]]
        partials[node] = tip_rows[node][:, None, :]
    ev, el, iv = model.engine_eigen()
    ops = np.ascontiguousarray(tr.postorder_traversal, dtype=np.int32)
    bl = tr.op_lengths()
    rates = np.ascontiguousarray(rm.rates)
    w = np.ascontiguousarray(rm.weights)
    sw = np.ones(S)
    fr = np.ascontiguousarray(model.freqs, dtype=np.float64)
    site_cpu = np.zeros(S)

    def pmats():
        P = orc.pmatrix_c(ev, el, iv, bl.reshape(-1), rates).reshape(len(ops), 2, C, K, K)
        Pr = orc.pmatrix_c(ev, el, iv, np.array([0.0, tr.root_length()]), rates)
        return np.ascontiguousarray(P), np.ascontiguousarray(Pr)

    reps, t0 = 0, time.perf_counter()
    lnl = None
    while True:
        P, Pr = pmats()
        lnl = orc.traverse_prepared(K, C, S, ops, P, Pr, tr.root_edge, partials, scale, fr, w, sw,
                                    threads, site_lnl=site_cpu)
        reps += 1
        el_t = time.perf_counter() - t0
        if el_t >= args.cpu_seconds or reps >= 5000:
            break
    ups = (ntax - 1) * S * C * reps / el_t / 1e6
    rel = abs(gpu_lnl - lnl) / abs(lnl) if S == S_full else None
    site_rel = float(np.max(np.abs(site_gpu[:S] - site_cpu) / np.abs(site_cpu)))
    log("[bench] cpu: %d reps in %.2fs -> %.2f M updates/s; lnL cpu %.10f gpu %.10f rel %s; "
        "sitewise max rel %.2e" % (reps, el_t, ups, lnl, gpu_lnl, rel, site_rel))
    del partials, scale

    # (b) numpy, one process, on the first S_np sites (bounded: ~numpy-seconds of work)
    S_np = min(S, 20_000 if K <= 4 else 2_000)
    np_part = np.zeros((n_nodes, S_np, C, K))
    np_scale = np.zeros((n_nodes, S_np, C))
    for node, rows in tip_rows.items():
        np_part[node] = rows[:S_np, None, :]
    nreps, t1 = 0, time.perf_counter()
    while True:
        P, Pr = pmats()
        lnl_np, site_np = orc.traverse_numpy(ops, P, Pr, tr.root_edge, np_part, np_scale, fr, w,
                                             np.ones(S_np))
        nreps += 1
        el_np = time.perf_counter() - t1
        if el_np >= args.numpy_seconds:
            break
    ups_np = (ntax - 1) * S_np * C * nreps / el_np / 1e6
    np_site_rel = float(np.max(np.abs(site_np - site_gpu[:S_np]) / np.abs(site_np)))
    log("[bench] numpy: %d traversals of %d sites in %.2fs -> %.3f M updates/s; sitewise max rel "
        "vs gpu %.2e" % (nreps, S_np, el_np, ups_np, np_site_rel))
    phys = host.get("physical_cores")
    cpu = {"value": round(ups, 3), "unit": "M updates/s", "cores": threads, "kind": "port",
           "sample": "%d full traversals of %s (oracle/pruning_oracle.c, OpenMP over site "
                     "blocks, %d threads, P matrices included)"
                     % (reps, "the same workload" if S == S_full else
                        "the first %d of the %d sites" % (S, S_full), threads),
           "host": host,
           "cpu_share_note": "threads = the GPU's lease of the host: the box exports "
                             "OMP_NUM_THREADS=%s per GPU and its run contract says to size worker "
                             "pools to that share, not to the %s physical cores nproc shows"
                             % (host.get("omp_num_threads_env"), phys),
           "all_physical_cores_projection": (
               {"value": round(ups * phys / threads, 3), "unit": "M updates/s", "cores": phys,
                "note": "linear scaling of the measured value to every physical core: an upper "
                        "bound for this memory-bound loop, NOT measured (the lease forbids it)"}
               if phys and phys > threads else None),
           "numpy_single_process": {
               "value": round(ups_np, 4), "unit": "M updates/s", "cores": 1, "kind": "port",
               "sample": "%d traversals over the first %d sites (oracle.traverse_numpy: the "
                         "vectorised clv / lnl_node loop of tree_model.py:160-217, P included)"
                         % (nreps, S_np)}}
    acc = {"lnl_rel_err_vs_cpu": rel, "sitewise_max_rel_err_vs_cpu": site_rel,
           "accuracy_sites": S,
           "sitewise_max_rel_err_vs_numpy": np_site_rel}
    return cpu, acc


if __name__ == "__main__":
    main()
