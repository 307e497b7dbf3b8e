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
