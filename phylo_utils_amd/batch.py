"""Several trees' lnL per launch: `pu_batch_*` of include/phylo_hip.h.

The reference evaluates many trees on one alignment by a loop of set_tree / compute_partials /
likelihood (tree_model.py:87-89, 160-176), one tree at a time.  `TreeBatch` takes the
lnL-only GPU models of such trees (`TreeModel(keep_partials=False)`, one per tree, coded DNA
tips) and evaluates all of them with one P launch, one traversal launch and one reduction;
each tree's lnL is bitwise the one its own model gives.
"""
import ctypes

import numpy as np

from . import _native as N


def _addr(ctx):
    return ctx.value if isinstance(ctx, ctypes.c_void_p) else ctx


class TreeBatch(object):
    def __init__(self, models):
        self.models = list(models)
        if not self.models:
            raise ValueError("TreeBatch needs at least one model")
        for m in self.models:
            m._ensure()  # the device context exists and holds its schedule
        self._b = None
        self._stream = None
        self._create()

    def _create(self):
        n = len(self.models)
        self._ctxs = [_addr(m._ctx) for m in self.models]
        ctxs = (ctypes.c_void_p * n)(*self._ctxs)
        h = ctypes.c_void_p()
        N.check(N.lib().pu_batch_create(ctypes.byref(h), n, ctxs), None, "pu_batch_create")
        self._b = h
        if self._stream is not None:
            self.set_stream(self._stream)

    def _check(self, rc, what):
        if rc != 0:
            msg = N.lib().pu_batch_last_error(self._b)
            raise N.PhyloHipError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))

    def set_stream(self, stream):
        """HIP stream handle (int / c_void_p) of the batch's launches; None: the null stream."""
        self._stream = stream
        self._check(N.lib().pu_batch_set_stream(self._b, ctypes.c_void_p(stream)
                                                if stream is not None else None),
                    "pu_batch_set_stream")

    def enqueue(self, lnl_dev=None):
        """Enqueue one evaluation of every tree; lnl_dev: device address of len(models)
        doubles for the lnLs (None: each model's own output, read by `likelihoods`)."""
        for m in self.models:
            m._ensure()
        # a model whose context was rebuilt (new alignment, rate categories, ascertainment
        # correction): the native batch holds the old pointer, so it is built again
        if any(_addr(m._ctx) != c for m, c in zip(self.models, self._ctxs)):
            N.lib().pu_batch_destroy(self._b)
            self._b = None
            self._create()
        self._check(N.lib().pu_batch_enqueue(self._b, ctypes.c_void_p(lnl_dev)
                                             if lnl_dev is not None else None),
                    "pu_batch_enqueue")

    def synchronize(self):
        self._check(N.lib().pu_batch_synchronize(self._b), "pu_batch_synchronize")

    def likelihoods(self):
        """lnL of every tree, one batched evaluation (host values)."""
        self.enqueue()
        self.synchronize()
        out = np.empty(len(self.models))
        v = ctypes.c_double()
        for i, m in enumerate(self.models):
            N.check(N.lib().pu_synchronize(m._ctx, ctypes.byref(v)), m._ctx, "pu_synchronize")
            out[i] = v.value
        return out

    def sitewise(self, i):
        """Per-pattern lnL of tree i from the last batched evaluation."""
        m = self.models[i]
        self.synchronize()  # the batch's launches write the tree's sitewise lnL
        out = np.empty(m._n_patterns())
        N.check(N.lib().pu_get_site_lnl(m._ctx, N.ptr(out)), m._ctx, "pu_get_site_lnl")
        return out

    def close(self):
        if getattr(self, "_b", None):
            N.lib().pu_batch_destroy(self._b)
            self._b = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
