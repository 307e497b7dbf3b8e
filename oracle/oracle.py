"""CPU oracle for the Felsenstein pruning path -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module.  The product package (``phylo_utils_amd``) never does: the
shipped path runs on the GPU through ``libphylo_hip.so`` and fails loudly when
that library is missing.

Contents
--------
* ``clv`` / ``lnl_node``: numpy restatements of the live numba engine
  (``phylo_utils/likelihood/numba_likelihood_engine.py:14-46`` and ``:82-87``),
  same argument order and in-place ``cml_scaler`` semantics.
* ``pmatrix``: ``Model.p`` via ``Eigen.exp``
  (``phylo_utils/substitution_models/abstract.py:49-59, 99-105``).
* ``tree_lnl``: ``TreeModel.initialise -> compute_partials ->
  compute_likelihood_at_edge`` (``phylo_utils/tree_model.py:101-217``) on an
  explicit schedule, backed by the C restatement in ``pruning_oracle.c``.
* ``ref_discrete_gamma``: the reference's own PAML routine
  (``src/c_discrete_gamma.c:285-321``) compiled from /root/reference by
  ``oracle/Makefile`` into ``oracle/_ref``.

Pinning: tests/test_oracle_golden.py checks all of the above against
tests/golden/*.npz, which tests/golden/make_golden.py generated from the
reference's own numpy engine (``python_likelihood_engine.py``), its
substitution models and its PAML C.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SCALE_THRESHOLD = 2.0 ** -128  # numba_likelihood_engine.py:7

_lib = None
_ref = None
_D = ctypes.POINTER(ctypes.c_double)


def _dp(a):
    return a.ctypes.data_as(_D)


def build():
    """Compile the oracle (and, when /root/reference exists, oracle/_ref)."""
    subprocess.check_call(["make", "-s", "-C", HERE], stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "_build", "liboracle.so")
        if not os.path.exists(path):
            build()
        _lib = ctypes.CDLL(path)
        _lib.or_traverse.restype = ctypes.c_double
    return _lib


def ref_lib():
    global _ref
    if _ref is None:
        path = os.path.join(HERE, "_ref", "libref_dgamma.so")
        if not os.path.exists(path):
            build()
        _ref = ctypes.CDLL(path)
        _ref.DiscreteGamma.restype = ctypes.c_int
        _ref.DiscreteGamma.argtypes = [_D, _D, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_int, ctypes.c_int]
    return _ref


def ref_discrete_gamma(alpha, ncat, median_rates=False):
    """Reference PAML rates (src/discrete_gamma.pyx:30-47 calling c_discrete_gamma.c)."""
    w = np.zeros(ncat)
    r = np.zeros(ncat)
    ref_lib().DiscreteGamma(_dp(w), _dp(r), float(alpha), float(alpha), int(ncat),
                            int(bool(median_rates)))
    return r


# ---------------------------------------------------------------- numpy restatements
def clv(p1, p2, clv1, clv2, scaler_a, scaler_b, cml_scaler, out=None):
    """numba_likelihood_engine.py:14-46 (vectorised over sites)."""
    p1 = np.asarray(p1, dtype=np.float64)
    p2 = np.asarray(p2, dtype=np.float64)
    x = np.einsum("cij,scj->sci", p1, clv1)
    y = np.einsum("cij,scj->sci", p2, clv2)
    res = x * y
    m = res.max(axis=-1)
    do = (m < SCALE_THRESHOLD) & (m > 0)
    base = scaler_a + scaler_b
    with np.errstate(divide="ignore", invalid="ignore"):
        cml_scaler[...] = np.where(do, base + np.log(np.where(do, m, 1.0)), base)
        res = np.where(do[..., None], res / np.where(do, m, 1.0)[..., None], res)
    if out is None:
        return res
    out[...] = res
    return out


def lnl_node(pi, partials, scale, out=None):
    """numba_likelihood_engine.py:82-87."""
    f = np.einsum("sci,i->sc", partials, pi)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(f > 0, np.log(np.where(f > 0, f, 1.0)) + scale, -np.inf)
    if out is None:
        return r
    out[...] = r
    return out


def pmatrix(evecs, evals, ivecs, t, rates):
    """Model.p(t, rates) via Eigen.exp (abstract.py:49-59, 99-105) -> [C][K][K]."""
    return np.stack([(evecs * np.exp(evals * (t * r))).dot(ivecs) for r in rates], axis=0)


def logsumexp_cats(sw, weights):
    """tree_model.py:216 -- scipy.special.logsumexp(sw + log w, axis=1) (scipy 1.15 form:
    maximal terms separated, log1p of the rest)."""
    a = sw + np.log(weights)[None, :]
    amax = a.max(axis=1)
    ismax = a == amax[:, None]
    m = ismax.sum(axis=1).astype(np.float64)
    shift = np.where(np.isfinite(amax), amax, 0.0)
    with np.errstate(divide="ignore", invalid="ignore"):
        s = np.where(ismax, 0.0, np.exp(a - shift[:, None])).sum(axis=1)
        s = np.where(s == 0, s, s / m)
        return np.log1p(s) + np.log(m) + amax


# ---------------------------------------------------------------- whole traversal
def tree_lnl(tips, ops, brlens_ops, root_edge, root_len, evecs, evals, ivecs, freqs, rates,
             weights, site_weights=None, n_nodes=None, nthreads=1, return_all=False):
    """TreeModel restatement on an explicit schedule (tree_model.py:101-217).

    tips        dict node_index -> [S][K] tip partials
    ops         int [n_ops][3] (par, ch1, ch2) in post-order (traversal.py:28-29)
    brlens_ops  float [n_ops][2] lengths of (par,ch1), (par,ch2)
    root_edge   (a, b) node indices, root_len its length (tree_model.py:178-198)
    Returns (lnL, site_lnl[S]) or a dict with every buffer when return_all.
    """
    C = len(rates)
    P = np.zeros((len(ops), 2, C, evecs.shape[0], evecs.shape[0]))
    for o in range(len(ops)):
        P[o, 0] = pmatrix(evecs, evals, ivecs, brlens_ops[o][0], rates)
        P[o, 1] = pmatrix(evecs, evals, ivecs, brlens_ops[o][1], rates)
    Proot = np.stack([pmatrix(evecs, evals, ivecs, 0.0, rates),
                      pmatrix(evecs, evals, ivecs, root_len, rates)])
    return tree_lnl_p(tips, ops, P, Proot, root_edge, freqs, weights, site_weights, n_nodes,
                      nthreads, return_all)


def tree_lnl_p(tips, ops, P, Proot, root_edge, freqs, weights, site_weights=None,
               n_nodes=None, nthreads=1, return_all=False):
    """tree_lnl on given transition matrices: P [n_ops][2][C][K][K] per op and child,
    Proot [2][C][K][K] for (root_a, root_b) -- what TreeModel.compute_partials feeds clv
    for any model (tree_model.py:166-176, :189-197), e.g. the non-reversible
    expm(Q r t) (abstract.py:172-177)."""
    ops = np.ascontiguousarray(ops, dtype=np.int32)
    P = np.ascontiguousarray(P, dtype=np.float64)
    _, _, C, K, _ = P.shape
    S = next(iter(tips.values())).shape[0]
    if n_nodes is None:
        n_nodes = int(max(ops.max(), max(root_edge)) + 1)
    if site_weights is None:
        site_weights = np.ones(S)
    partials = np.zeros((n_nodes, S, C, K))
    scale = np.zeros((n_nodes, S, C))
    for n, t in tips.items():
        partials[n] = np.asarray(t, dtype=np.float64)[:, None, :]
    Proot = np.ascontiguousarray(Proot, dtype=np.float64)
    root_partials = np.zeros((S, C, K))
    root_scale = np.zeros((S, C))
    site_lnl = np.zeros(S)
    sw = np.ascontiguousarray(site_weights, dtype=np.float64)
    fr = np.ascontiguousarray(freqs, dtype=np.float64)
    wt = np.ascontiguousarray(weights, dtype=np.float64)
    total = lib().or_traverse(
        ctypes.c_int(K), ctypes.c_int(C), ctypes.c_long(S), ctypes.c_int(len(ops)),
        ops.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), _dp(P), _dp(Proot),
        ctypes.c_int(root_edge[0]), ctypes.c_int(root_edge[1]), _dp(partials), _dp(scale),
        _dp(root_partials), _dp(root_scale), _dp(fr), _dp(wt), _dp(sw), _dp(site_lnl),
        ctypes.c_int(nthreads))
    if return_all:
        return dict(lnl=total, site_lnl=site_lnl, partials=partials, scale=scale,
                    root_partials=root_partials, root_scale=root_scale, P=P, Proot=Proot)
    return total, site_lnl


def traverse_prepared(K, C, S, ops, P, Proot, root_edge, partials, scale, freqs, weights,
                      site_weights, nthreads, site_lnl=None):
    """Timed CPU-baseline entry (bench.py): all buffers preallocated by the caller
    (`site_lnl`, when given, receives the sitewise lnL)."""
    root_partials = np.zeros((S, C, K))
    root_scale = np.zeros((S, C))
    if site_lnl is None:
        site_lnl = np.zeros(S)
    return lib().or_traverse(
        ctypes.c_int(K), ctypes.c_int(C), ctypes.c_long(S), ctypes.c_int(len(ops)),
        ops.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), _dp(P), _dp(Proot),
        ctypes.c_int(root_edge[0]), ctypes.c_int(root_edge[1]), _dp(partials), _dp(scale),
        _dp(root_partials), _dp(root_scale), _dp(freqs), _dp(weights), _dp(site_weights),
        _dp(site_lnl), ctypes.c_int(nthreads))


def traverse_numpy(ops, P, Proot, root_edge, partials, scale, freqs, weights, site_weights):
    """Single-process numpy restatement of TreeModel.compute_partials +
    compute_likelihood_at_edge (tree_model.py:160-217) over the vectorised `clv` /
    `lnl_node` above: one numpy call sequence per op, all sites at once (SURVEY 8(d) M4(b),
    bench.py's second CPU baseline).  partials [n_nodes][S][C][K] (tips filled), scale
    [n_nodes][S][C]; returns (lnL, site_lnl)."""
    for o, (par, c1, c2) in enumerate(ops):
        partials[par] = clv(P[o, 0], P[o, 1], partials[c1], partials[c2], scale[c1], scale[c2],
                            scale[par])
    a, b = root_edge
    S, C = scale.shape[1:]
    root_scale = np.zeros((S, C))
    root = clv(Proot[0], Proot[1], partials[a], partials[b], scale[a], scale[b], root_scale)
    site = logsumexp_cats(lnl_node(freqs, root, root_scale), weights)
    return float(np.dot(site_weights, site)), site


def pmatrix_c(evecs, evals, ivecs, brlens, rates):
    """C restatement of Model.p for many branches -> [n_br][C][K][K]."""
    K = evecs.shape[0]
    C = len(rates)
    out = np.zeros((len(brlens), C, K, K))
    ev = np.ascontiguousarray(evecs, dtype=np.float64)
    el = np.ascontiguousarray(evals, dtype=np.float64)
    iv = np.ascontiguousarray(ivecs, dtype=np.float64)
    bl = np.ascontiguousarray(brlens, dtype=np.float64)
    rt = np.ascontiguousarray(rates, dtype=np.float64)
    lib().or_pmatrix(ctypes.c_int(K), ctypes.c_int(C), ctypes.c_int(len(bl)), _dp(ev), _dp(el),
                     _dp(iv), _dp(bl), _dp(rt), _dp(out))
    return out


def clv_c(p1, p2, clv1, clv2, sa, sb, cml):
    """C restatement of `clv` (same semantics as `clv`, sequential arithmetic)."""
    S, C, K = clv1.shape
    out = np.zeros_like(clv1)
    a = [np.ascontiguousarray(x, dtype=np.float64) for x in (p1, p2, clv1, clv2, sa, sb)]
    lib().or_clv(ctypes.c_int(K), ctypes.c_int(C), ctypes.c_long(S), *[_dp(x) for x in a],
                 _dp(cml), _dp(out))
    return out


# ---------------------------------------------------------------- edges
def lnl_branch(probs, pi, partials_a, partials_b, scale_a, scale_b):
    """numba_likelihood_engine.py:60-79 with numpy broadcasting of the gufunc loop dims."""
    x = np.einsum("...ij,...j->...i", probs, partials_a)
    f = (x * partials_b * pi).sum(axis=-1)
    return np.log(f) + scale_a + scale_b


def lnl_branch_derivs(probs, pi, partials_a, partials_b, scale_a, scale_b):
    """numba_likelihood_engine.py:49-57: probs (..., 3, K, K) = (P, dP, d2P)."""
    x = np.einsum("...mij,...j->...mi", probs, partials_a)
    f = (x * partials_b[..., None, :] * pi).sum(axis=-1)
    f0, f1, f2 = f[..., 0], f[..., 1], f[..., 2]
    return np.stack([np.log(f0) + scale_a + scale_b, f1 / f0,
                     ((f2 * f0) - (f1 * f1)) / (f0 * f0)], axis=-1)


def pmatrix_deriv(evecs, evals, ivecs, t, rates, order):
    """d^order/dt^order P(t r) = evecs diag((l r)^order e^{l t r}) ivecs -> [C][K][K]
    (Model.dp_dt / d2p_dt2, abstract.py:61-77, with the chain-rule factor r they omit)."""
    return np.stack([(evecs * ((evals * r) ** order * np.exp(evals * (t * r)))).dot(ivecs)
                     for r in rates], axis=0)


def edge_derivs(pa, sa, pb, sb, evecs, evals, ivecs, t, rates, weights, freqs,
                site_weights=None):
    """(lnL, dlnL/dt, d2lnL/dt2) of the root on an edge: P(0) on a, P(t) on b
    (or_edge_derivs in pruning_oracle.c); pa, pb [S][C][K], sa, sb [S][C]."""
    S, C, K = pa.shape
    if site_weights is None:
        site_weights = np.ones(S)
    P0 = pmatrix(evecs, evals, ivecs, 0.0, rates)
    mats = [np.ascontiguousarray(pmatrix_deriv(evecs, evals, ivecs, t, rates, k))
            for k in range(3)]
    out = np.zeros(3)
    args = [np.ascontiguousarray(x, dtype=np.float64) for x in
            (pa, sa, pb, sb, P0, mats[0], mats[1], mats[2], freqs, weights, site_weights)]
    lib().or_edge_derivs(ctypes.c_int(K), ctypes.c_int(C), ctypes.c_long(S),
                         *[_dp(x) for x in args], _dp(out), None)
    return out


def edge_lnl(pa, sa, pb, sb, evecs, evals, ivecs, t, rates, weights, freqs):
    """compute_likelihood_at_edge (tree_model.py:178-217) on given end partials:
    clv(P(0), P(t)) -> lnl_node -> logsumexp over categories; returns sitewise lnL."""
    P0 = pmatrix(evecs, evals, ivecs, 0.0, rates)
    P1 = pmatrix(evecs, evals, ivecs, t, rates)
    cml = np.zeros(sa.shape)
    root = clv(P0, P1, pa, pb, sa, sb, cml)
    return logsumexp_cats(lnl_node(freqs, root, cml), weights)


# Newton-Raphson as in pu_edge.cpp (same bounds, safeguard and stopping rule)
MIN_LEN, MAX_LEN = 1e-8, 100.0


def newton_edge(evaluate, t, tol, max_iter):
    """evaluate(t) -> (lnL, d1, d2); returns (t, lnL, iterations)."""
    t = min(max(t, MIN_LEN), MAX_LEN)
    r = evaluate(t)
    it = 0
    while it < max_iter:
        l, d1, d2 = r
        if not np.isfinite(l):
            break
        step = -d1 / d2 if d2 < 0 else (t + 0.1 if d1 > 0 else -0.5 * t)
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
            break
        dt = abs(tn - t)
        t, r = tn, rn
        it += 1
        if dt <= tol * (1.0 + t):
            break
    return t, r[0], it


def optimise_sweep(tips, ops, brlens_ops, root_edge, root_len, evecs, evals, ivecs, freqs,
                   rates, weights, rows, n_nodes, site_weights=None, tol=1e-8, max_iter=50,
                   edge_opt=None):
    """One pass of the optimising traversal (utils.py:137-188) on the CPU: re-orient,
    Newton on each edge, restore.  Returns (lengths {sorted pair: t}, final lnL).
    edge_opt(evaluate, t0) -> t replaces Newton (evaluate(t) -> (lnL, d1, d2))."""
    st = tree_lnl(tips, ops, brlens_ops, root_edge, root_len, evecs, evals, ivecs, freqs,
                  rates, weights, site_weights=site_weights, n_nodes=n_nodes, return_all=True)
    partials, scale = st["partials"], st["scale"]
    lens = {}
    for (p, a, b), (la, lb) in zip(np.asarray(ops), np.asarray(brlens_ops)):
        lens[tuple(sorted((int(p), int(a))))] = float(la)
        lens[tuple(sorted((int(p), int(b))))] = float(lb)
    lens[tuple(sorted(map(int, root_edge)))] = float(root_len)
    L = lambda u, v: lens[tuple(sorted((int(u), int(v))))]
    for row in np.asarray(rows):
        if row[0] >= 0:
            p, x, y = int(row[0]), int(row[1]), int(row[2])
            P1 = pmatrix(evecs, evals, ivecs, L(p, x), rates)
            P2 = pmatrix(evecs, evals, ivecs, L(p, y), rates)
            cml = np.zeros(scale[p].shape)
            partials[p] = clv_c(P1, P2, partials[x], partials[y], scale[x], scale[y], cml)
            scale[p] = cml
        if row[3] >= 0:
            n, q = int(row[3]), int(row[4])
            ev = lambda t: edge_derivs(partials[n], scale[n], partials[q], scale[q], evecs,
                                       evals, ivecs, t, rates, weights, freqs, site_weights)
            if edge_opt is None:
                t, _, _ = newton_edge(ev, L(n, q), tol, max_iter)
            else:
                t = edge_opt(ev, L(n, q))
            lens[tuple(sorted((n, q)))] = t
    bl = np.array([[L(p, a), L(p, b)] for p, a, b in np.asarray(ops)])
    lnl, _ = tree_lnl(tips, ops, bl, root_edge, L(*root_edge), evecs, evals, ivecs, freqs,
                      rates, weights, site_weights=site_weights, n_nodes=n_nodes)
    return lens, lnl


def edge_derivs_p(pa, sa, pb, sb, mats, weights, freqs, site_weights=None):
    """edge_derivs on given matrices mats = (P(0), P(t), dP/dt, d2P/dt2), each [C][K][K]
    (models without an eigen-decomposition: the non-reversible DNA models)."""
    S, C, K = pa.shape
    if site_weights is None:
        site_weights = np.ones(S)
    out = np.zeros(3)
    args = [np.ascontiguousarray(x, dtype=np.float64) for x in
            (pa, sa, pb, sb, mats[0], mats[1], mats[2], mats[3], freqs, weights, site_weights)]
    lib().or_edge_derivs(ctypes.c_int(K), ctypes.c_int(C), ctypes.c_long(S),
                         *[_dp(x) for x in args], _dp(out), None)
    return out


def optimise_sweep_p(tips, ops, brlens_ops, root_edge, root_len, pm, freqs, weights, rows,
                     n_nodes, site_weights=None, tol=1e-8, max_iter=50):
    """optimise_sweep for models given as a matrix function pm(t, order) -> [C][K][K]
    (d^order/dt^order P(t r) per category, the chain-rule factor r included), e.g. the
    non-reversible models' expm(Q r t) (abstract.py:172-192).  Same rows, Newton and final
    traversal; returns (lengths {sorted pair: t}, final lnL)."""
    P = np.stack([np.stack([pm(la, 0), pm(lb, 0)]) for la, lb in np.asarray(brlens_ops)])
    Proot = np.stack([pm(0.0, 0), pm(root_len, 0)])
    st = tree_lnl_p(tips, ops, P, Proot, root_edge, freqs, weights, site_weights, n_nodes,
                    return_all=True)
    partials, scale = st["partials"], st["scale"]
    lens = {}
    for (p, a, b), (la, lb) in zip(np.asarray(ops), np.asarray(brlens_ops)):
        lens[tuple(sorted((int(p), int(a))))] = float(la)
        lens[tuple(sorted((int(p), int(b))))] = float(lb)
    lens[tuple(sorted(map(int, root_edge)))] = float(root_len)
    L = lambda u, v: lens[tuple(sorted((int(u), int(v))))]
    for row in np.asarray(rows):
        if row[0] >= 0:
            p, x, y = int(row[0]), int(row[1]), int(row[2])
            cml = np.zeros(scale[p].shape)
            partials[p] = clv_c(pm(L(p, x), 0), pm(L(p, y), 0), partials[x], partials[y],
                                scale[x], scale[y], cml)
            scale[p] = cml
        if row[3] >= 0:
            n, q = int(row[3]), int(row[4])
            ev = lambda t: edge_derivs_p(partials[n], scale[n], partials[q], scale[q],
                                         (pm(0.0, 0), pm(t, 0), pm(t, 1), pm(t, 2)), weights,
                                         freqs, site_weights)
            t, _, _ = newton_edge(ev, L(n, q), tol, max_iter)
            lens[tuple(sorted((n, q)))] = t
    P = np.stack([np.stack([pm(L(p, a), 0), pm(L(p, b), 0)]) for p, a, b in np.asarray(ops)])
    Proot = np.stack([pm(0.0, 0), pm(L(*root_edge), 0)])
    lnl, _ = tree_lnl_p(tips, ops, P, Proot, root_edge, freqs, weights, site_weights, n_nodes)
    return lens, lnl


# ---------------------------------------------------------------- ascertainment
def lse_flat(a):
    """scipy.special.logsumexp over all entries (scipy 1.15 form)."""
    a = np.asarray(a, dtype=np.float64).ravel()
    amax = a.max()
    ismax = a == amax
    m = float(ismax.sum())
    shift = amax if np.isfinite(amax) else 0.0
    s = np.exp(a[~ismax] - shift).sum()
    if s != 0:
        s /= m
    return np.log1p(s) + np.log(m) + amax


def tree_lnl_ascbias(tips, ops, brlens_ops, root_edge, root_len, evecs, evals, ivecs, freqs,
                     rates, weights, site_weights=None, n_nodes=None, weighted=False):
    """TreeModel with set_ascertainment_bias_correction (tree_model.py:92-98, 113-114,
    151-156, 200-217): K dummy invariant sites appended (site k: every tip one-hot in k),
    correction = log(1 - exp(logsumexp(swlnls[-K:]))) over all K x C lnl_node values
    (unweighted, :213), subtracted from the other sites before the logsumexp over
    categories (:214-216).  weighted=True: the weighted mixture instead.
    Returns (lnL over the real patterns, sitewise [S + K], correction)."""
    K = evecs.shape[0]
    S = next(iter(tips.values())).shape[0]
    if site_weights is None:
        site_weights = np.ones(S)
    eye = np.eye(K)
    tips_x = {n: np.vstack([np.asarray(t, dtype=np.float64), eye]) for n, t in tips.items()}
    sw_x = np.concatenate([site_weights, np.zeros(K)])
    st = tree_lnl(tips_x, ops, brlens_ops, root_edge, root_len, evecs, evals, ivecs, freqs,
                  rates, weights, site_weights=sw_x, n_nodes=n_nodes, return_all=True)
    with np.errstate(divide="ignore", invalid="ignore"):
        swl = lnl_node(freqs, st["root_partials"], st["root_scale"])
        if weighted:
            x = lse_flat(logsumexp_cats(swl[-K:], weights))
        else:
            x = lse_flat(swl[-K:])
        corr = np.log(1 - np.exp(x))
        swl[:-K] -= corr
        site = logsumexp_cats(swl, weights)
    return float((site[:S] * site_weights).sum()), site, float(corr)
