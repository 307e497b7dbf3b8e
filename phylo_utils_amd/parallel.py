"""Multi-GPU evaluation: one process per GPU, torch.distributed (RCCL over xGMI).

SURVEY 8(e):
* G1 site sharding -- every site pattern is independent through the whole
  post-order, so rank r owns a contiguous block of patterns, holds all tips for
  it and runs the full schedule; the only exchange is ONE all-reduce (sum) of
  the per-rank lnL (pattern weights applied locally).  Sitewise output, when
  asked for, is an all-gather of the per-rank slices.
* G2 tree sharding -- independent trees (e.g. bootstrap replicates) on the same
  alignment: rank r evaluates its contiguous block of trees; no collective
  during compute, one all-gather of the lnLs at the end.
* G1 x N1 -- branch-length optimisation of a site-sharded alignment: every rank
  re-orients its own partials, and each Newton (or brent / dbrent) evaluation is
  the ranks' (lnL, dlnL/dt, d2lnL/dt2) on their shards summed by one all-reduce of
  3 doubles; every rank then takes the same step, so the lengths never diverge.

The per-rank engine is phylo_utils_amd.TreeModel on `cuda:<local rank>`; tests
inject a CPU engine through `engine_factory` to exercise the same sharding and
collective code with the gloo backend.
"""
from __future__ import annotations

import numpy as np

from .tree_model import TreeModel


def _dist():
    import torch.distributed as dist
    return dist


def rank_world(group=None):
    dist = _dist()
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def shard_range(n, rank, world):
    """Contiguous [lo, hi) block of n items for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _device_for_collective(group=None):
    import torch
    dist = _dist()
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gpu_engine(device):
    def make(tree, codes, table, names, siteweights, model, rate_model):
        tm = TreeModel(device=device)
        tm.set_alignment_codes(codes, table, names, siteweights)
        tm.set_substitution_model(model)
        tm.set_rate_model(rate_model)
        tm.set_tree(tree)
        tm.initialise()
        return tm
    return make


# Newton-Raphson on one edge length, as pu_edge.cpp's newton() (same bounds, safeguard and
# stopping rule), over an evaluate(t) -> (lnL, d1, d2) of the whole alignment
MIN_LEN, MAX_LEN = 1e-8, 100.0


def newton_edge(evaluate, t, tol, max_iter):
    """Returns (t, lnL at t, iterations).  A step that lowers the lnL is halved (up to 30
    times); a non-concave point moves by expansion (d1 > 0) or halving (pu_edge.cpp:163-206)."""
    t = min(max(float(t), MIN_LEN), MAX_LEN)
    r = evaluate(t)
    it = 0
    while it < max_iter:
        l, d1, d2 = r
        if not np.isfinite(l):
            break
        step = -d1 / d2 if d2 < 0.0 else (t + 0.1 if d1 > 0.0 else -0.5 * t)
        tn = min(max(t + step, MIN_LEN), MAX_LEN)
        if tn == t:
            break
        ok = False
        for _ in range(30):
            rn = evaluate(tn)
            if rn[0] >= l - 1e-13 * abs(l):
                ok = True
                break
            tn = 0.5 * (t + tn)
        if not ok:
            break  # no ascent along this direction: t is (numerically) optimal
        dt = abs(tn - t)
        t, r = tn, rn
        it += 1
        if dt <= tol * (1.0 + t):
            break
    return t, r[0], it


class SiteShardedLikelihood(object):
    """Whole-alignment lnL with the site patterns split across ranks (G1)."""

    def __init__(self, tree, codes, table, names, model, rate_model, siteweights=None,
                 group=None, device=None, engine_factory=None):
        self.group = group
        self.rank, self.world = rank_world(group)
        codes = np.asarray(codes)
        self.n_patterns = codes.shape[1]
        self.lo, self.hi = shard_range(self.n_patterns, self.rank, self.world)
        if self.hi <= self.lo:
            raise ValueError("rank %d has no site patterns (S=%d, world=%d)" %
                             (self.rank, self.n_patterns, self.world))
        sw = np.ones(self.n_patterns) if siteweights is None else np.asarray(siteweights)
        if engine_factory is None:
            import torch
            engine_factory = gpu_engine(torch.cuda.current_device() if device is None
                                        else device)
        self.engine = engine_factory(tree, np.ascontiguousarray(codes[:, self.lo:self.hi]),
                                     table, names, sw[self.lo:self.hi], model, rate_model)

    def local_likelihood(self):
        return float(self.engine.likelihood())

    def likelihood(self):
        """Sum of per-rank lnL: one all-reduce (RCCL over xGMI with the nccl backend)."""
        local = self.local_likelihood()
        if self.world == 1:
            return local
        import torch
        t = torch.tensor([local], dtype=torch.float64, device=_device_for_collective(self.group))
        _dist().all_reduce(t, group=self.group)
        return float(t.item())

    def sitewise_patterns(self):
        """Per-pattern lnL of the whole alignment (all-gather of equal-size padded slices)."""
        local = np.asarray(self.engine.sitewise_patterns(), dtype=np.float64)
        if self.world == 1:
            return local
        import torch
        dev = _device_for_collective(self.group)
        width = shard_range(self.n_patterns, 0, self.world)[1]
        buf = torch.full((width,), float("nan"), dtype=torch.float64, device=dev)
        buf[:len(local)] = torch.from_numpy(local).to(dev)
        parts = [torch.empty_like(buf) for _ in range(self.world)]
        _dist().all_gather(parts, buf, group=self.group)
        out = []
        for r, p in enumerate(parts):
            lo, hi = shard_range(self.n_patterns, r, self.world)
            out.append(p[:hi - lo].cpu().numpy())
        return np.concatenate(out)

    def optimise_branch_lengths(self, tol=1e-8, max_iter=50, sweeps=1, lnl_tol=None, method="newton",
                          bracket=(1e-8, 10.0)):
        """Branch-length optimisation (G1 x N1): the optimising traversal (utils.py:137-188)
        on every rank's shard, each evaluation of the whole-alignment (lnL, d1, d2) one
        all-reduce of 3 doubles; Newton as pu_edge.cpp (newton_edge) or the reference's brent
        / dbrent over `bracket`.  Every rank takes the same steps.  Returns the lnL."""
        from . import optimisation
        eng = self.engine
        tr = eng.traversal
        rows = np.asarray(tr.optimising_traversal)
        L = lambda u, v: tr.brlens[tuple(sorted((int(u), int(v))))]
        if method not in ("newton", "brent", "dbrent"):
            raise ValueError("method must be 'newton', 'brent' or 'dbrent'")
        n_eval = [0]

        def global_derivs(a, b, t):
            n_eval[0] += 1
            loc = np.asarray(eng.edge_derivatives(a, b, t), dtype=np.float64)
            return tuple(float(x) for x in self._allreduce(loc))

        prev = self.likelihood()
        lnl = prev
        for _ in range(int(sweeps)):
            for row in rows:
                if row[0] >= 0:  # re-orient / restore (PAR, SIB, GPA) or (NOD, CH1, CH2)
                    eng.update_partials([row[:3]], [[L(row[0], row[1]), L(row[0], row[2])]])
                if row[3] >= 0:
                    a, b = int(row[3]), int(row[4])
                    key = tuple(sorted((a, b)))
                    if method == "newton":
                        t, _, _ = newton_edge(lambda x: global_derivs(a, b, x), tr.brlens[key],
                                              tol, max_iter)
                    else:
                        lo, hi = float(bracket[0]), float(bracket[1])
                        last = {}

                        def ev(x):
                            if x not in last:
                                last.clear()
                                last[x] = global_derivs(a, b, x)
                            return last[x]
                        out = np.zeros(3)
                        t0 = min(max(tr.brlens[key], lo), hi)
                        if method == "brent":
                            optimisation.brent(lo, t0, hi, lambda x: -ev(x)[0], tol, out)
                        else:
                            optimisation.dbrent(lo, t0, hi, lambda x: -ev(x)[0],
                                                lambda x: -ev(x)[1], tol, out)
                        t = float(out[0])
                    tr.brlens[key] = t
            eng.update_branch_lengths()
            eng.compute_partials()
            lnl = self.likelihood()
            if lnl_tol is not None and lnl - prev < lnl_tol:
                break
            prev = lnl
        self.last_evaluations = n_eval[0]
        return lnl

    def _allreduce(self, arr):
        if self.world == 1:
            return np.asarray(arr, dtype=np.float64)
        import torch
        t = torch.tensor(np.asarray(arr, dtype=np.float64),
                         device=_device_for_collective(self.group))
        _dist().all_reduce(t, group=self.group)
        return t.cpu().numpy()


class TreeShardedLikelihoods(object):
    """lnL of many trees on one alignment, trees split across ranks (G2)."""

    def __init__(self, trees, codes, table, names, model, rate_model, siteweights=None,
                 group=None, device=None, engine_factory=None):
        self.group = group
        self.rank, self.world = rank_world(group)
        self.n_trees = len(trees)
        self.lo, self.hi = shard_range(self.n_trees, self.rank, self.world)
        if engine_factory is None:
            import torch
            engine_factory = gpu_engine(torch.cuda.current_device() if device is None
                                        else device)
        self._make = lambda t: engine_factory(t, codes, table, names, siteweights, model,
                                              rate_model)
        self.trees = trees

    def local_likelihoods(self):
        out = []
        eng = None
        for t in self.trees[self.lo:self.hi]:
            if eng is None or not hasattr(eng, "set_tree"):
                eng = self._make(t)
            else:  # reuse the device context's tips/model; new topology + lengths
                eng.set_tree(t)
                eng.initialise()
            out.append(float(eng.likelihood()))
        return np.array(out)

    def likelihoods(self):
        local = self.local_likelihoods()
        if self.world == 1:
            return local
        import torch
        dev = _device_for_collective(self.group)
        width = shard_range(self.n_trees, 0, self.world)[1]
        buf = torch.full((width,), float("nan"), dtype=torch.float64, device=dev)
        buf[:len(local)] = torch.from_numpy(local).to(dev)
        parts = [torch.empty_like(buf) for _ in range(self.world)]
        _dist().all_gather(parts, buf, group=self.group)
        out = []
        for r, p in enumerate(parts):
            lo, hi = shard_range(self.n_trees, r, self.world)
            out.append(p[:hi - lo].cpu().numpy())
        return np.concatenate(out)
