"""HIP likelihood engine -- drop-in for ``phylo_utils.likelihood.numba_likelihood_engine``.

The reference picks its engine by import (``phylo_utils/tree_model.py:1``)::

    from phylo_utils.likelihood.numba_likelihood_engine import clv, lnl_node

and this module exports the engine interface the three reference engines share
(``clv``, ``lnl_node``, ``lnl_branch``, ``lnl_branch_derivs``; numba :14,51,62,84)
with the same argument order, gufunc shapes and broadcasting, in-place
``cml_scaler`` write and ``out`` handling, computed by the gfx950 kernels in
libphylo_hip.so (``pu_clv`` / ``pu_lnl_node`` / ``pu_lnl_branch[_derivs]``).  Host arrays are copied
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


def _branch(probs, pi, partials_a, partials_b, scale_a, scale_b, out, derivs):
    """Shared body of lnl_branch / lnl_branch_derivs: numpy broadcasting of the gufunc
    loop dimensions, then one flat launch (item e uses probs[e % n_p], or an explicit
    probs index when probs does not broadcast along leading dimensions only)."""
    core = 3 if derivs else 2
    probs = _as_c(probs, "probs")
    pi = _as_c(pi, "pi")
    pa = np.asarray(partials_a, dtype=np.float64)
    pb = np.asarray(partials_b, dtype=np.float64)
    sa = np.asarray(scale_a, dtype=np.float64)
    sb = np.asarray(scale_b, dtype=np.float64)
    if pi.ndim != 1:
        raise ValueError("pi must be (nstate,)")
    K = pi.shape[0]
    if probs.ndim < core or probs.shape[-2:] != (K, K) or (derivs and probs.shape[-3] != 3):
        raise ValueError("probs must end in %s" % (("3, " if derivs else "") + "%d, %d" % (K, K)))
    if pa.shape[-1:] != (K,) or pb.shape[-1:] != (K,):
        raise ValueError("partials must end in nstate=%d" % K)
    pl = probs.shape[:-core]
    try:
        L = np.broadcast_shapes(pl, pa.shape[:-1], pb.shape[:-1], sa.shape, sb.shape)
    except ValueError as e:
        raise ValueError("lnl_branch operands do not broadcast: %s" % e)
    E = int(np.prod(L)) if L else 1
    n_p = int(np.prod(pl)) if pl else 1
    pls = tuple(pl)
    while pls and pls[0] == 1:
        pls = pls[1:]
    if not pls or pls == tuple(L[len(L) - len(pls):]):
        pidx = None  # probs broadcast along leading dimensions only: index e % n_p
    else:
        pidx = np.ascontiguousarray(
            np.broadcast_to(np.arange(n_p, dtype=np.int32).reshape(pl), L).reshape(-1))
    flat = lambda a, tail: np.ascontiguousarray(np.broadcast_to(a, L + tail)).reshape(-1)
    a_, b_ = flat(pa, (K,)), flat(pb, (K,))
    sa_, sb_ = flat(sa, ()), flat(sb, ())
    res = np.empty(L + ((3,) if derivs else ()), dtype=np.float64)
    fn = N.lib().pu_lnl_branch_derivs if derivs else N.lib().pu_lnl_branch
    N.check(fn(DEVICE, K, E, n_p, N.ptr(pidx), N.ptr(probs), N.ptr(pi), N.ptr(a_), N.ptr(b_),
               N.ptr(sa_), N.ptr(sb_), N.ptr(res)),
            what="pu_lnl_branch_derivs" if derivs else "pu_lnl_branch")
    if out is None:
        return res
    out[...] = res
    return out


def lnl_branch(probs, pi, partials_a, partials_b, scale_a, scale_b, out=None):
    """Log-likelihood across the branch between A and B (numba_likelihood_engine.py:60-79),
    gufunc ``(n,n),(n),(n),(n),(),()->()``: ``log(sum((probs . a) * b * pi)) + sa + sb``."""
    return _branch(probs, pi, partials_a, partials_b, scale_a, scale_b, out, False)


def lnl_branch_derivs(probs, pi, partials_a, partials_b, scale_a, scale_b, out=None):
    """lnL and its first and second derivatives across a branch
    (numba_likelihood_engine.py:49-57), gufunc ``(m,n,n),(n),(n),(n),(),()->(m)`` with
    probs = (P, dP/dt, d2P/dt2): ``[log f + sa + sb, f'/f, (f'' f - f'^2) / f^2]``."""
    return _branch(probs, pi, partials_a, partials_b, scale_a, scale_b, out, True)
