"""HIP likelihood engine -- drop-in for ``phylo_utils.likelihood.numba_likelihood_engine``.

The reference picks its engine by import (``phylo_utils/tree_model.py:1``)::

    from phylo_utils.likelihood.numba_likelihood_engine import clv, lnl_node

and this module exports the same two callables with the same argument order,
shapes, in-place ``cml_scaler`` write and ``out`` handling, computed by the gfx950
kernels in libphylo_hip.so (``pu_clv`` / ``pu_lnl_node``).  Host arrays are copied
to the device and back on every call; for whole traversals use
``phylo_utils_amd.tree_model.TreeModel``, which keeps everything in HBM.
"""
from __future__ import annotations

import os

import numpy as np

from .. import _native as N

DEVICE = int(os.environ.get("PHYLO_HIP_DEVICE", "0"))


def _as_c(a, name):
    a = np.asarray(a)
    if a.dtype != np.float64:
        raise TypeError("%s must be float64 (got %s)" % (name, a.dtype))
    return np.ascontiguousarray(a)


def clv(p1, p2, clv1, clv2, scaler_a, scaler_b, cml_scaler, out=None):
    """Conditional likelihood vector at the parent of A and B.

    numba_likelihood_engine.py:10-46 -- layout
    ``(ncat,nstate,nstate),(ncat,nstate,nstate),(ncat,nstate),(ncat,nstate),(ncat),(ncat),(ncat)
    -> (ncat,nstate)`` broadcast over a leading site axis.  ``cml_scaler`` is
    written in place (numba :40,:44); ``out`` is allocated when omitted,
    otherwise filled and returned.
    """
    p1 = _as_c(p1, "p1")
    p2 = _as_c(p2, "p2")
    c1 = _as_c(clv1, "clv1")
    c2 = _as_c(clv2, "clv2")
    sa = _as_c(scaler_a, "scaler_a")
    sb = _as_c(scaler_b, "scaler_b")
    if p1.ndim != 3 or p1.shape[1] != p1.shape[2] or p2.shape != p1.shape:
        raise ValueError("p1/p2 must be (ncat, nstate, nstate) and equal shapes")
    C, K = p1.shape[0], p1.shape[1]
    if c1.shape[-2:] != (C, K) or c2.shape != c1.shape:
        raise ValueError("clv1/clv2 must end in (ncat=%d, nstate=%d)" % (C, K))
    lead = c1.shape[:-2]
    S = int(np.prod(lead)) if lead else 1
    if sa.shape != lead + (C,) or sb.shape != sa.shape:
        raise ValueError("scalers must have shape %s" % ((lead + (C,)),))
    if not isinstance(cml_scaler, np.ndarray) or cml_scaler.shape != sa.shape \
            or cml_scaler.dtype != np.float64:
        raise ValueError("cml_scaler must be a float64 array of shape %s" % ((lead + (C,)),))
    res = np.empty(c1.shape, dtype=np.float64)
    cml = cml_scaler if cml_scaler.flags.c_contiguous else np.empty(sa.shape)
    N.check(N.lib().pu_clv(DEVICE, K, C, S, N.ptr(p1), N.ptr(p2), N.ptr(c1), N.ptr(c2),
                           N.ptr(sa), N.ptr(sb), N.ptr(cml), N.ptr(res)), what="pu_clv")
    if cml is not cml_scaler:
        cml_scaler[...] = cml
    if out is None:
        return res
    out[...] = res
    return out


def lnl_node(pi, partials, scale, out=None):
    """Site x category log-likelihood at a root node (numba_likelihood_engine.py:82-87):
    ``log(sum_i pi_i * partials[..., c, i]) + scale[..., c]``, ``-inf`` when the sum <= 0."""
    pi = _as_c(pi, "pi")
    pa = _as_c(partials, "partials")
    sc = _as_c(scale, "scale")
    K = pi.shape[0]
    if pa.shape[-1] != K or sc.shape != pa.shape[:-1]:
        raise ValueError("partials (..., ncat, nstate) / scale (..., ncat) mismatch")
    C = pa.shape[-2]
    S = int(np.prod(pa.shape[:-2])) if pa.ndim > 2 else 1
    res = np.empty(sc.shape, dtype=np.float64)
    N.check(N.lib().pu_lnl_node(DEVICE, K, C, S, N.ptr(pi), N.ptr(pa), N.ptr(sc), N.ptr(res)),
            what="pu_lnl_node")
    if out is None:
        return res
    out[...] = res
    return out
