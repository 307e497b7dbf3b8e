"""GPU parity of the edge operations through the C ABI against the CPU
oracle: the root on any edge (tree_model.py:178-217 on current partials), branch-length
derivatives, in-place re-orientation updates, Newton on one edge and the optimising-
traversal sweep (utils.py:137-188), and the stateless lnl_branch / lnl_branch_derivs.

Tolerances (fp64, written per assertion): sitewise / total lnL 1e-12 relative (root edge:
bit-identical to the traversal), derivatives 1e-10 relative to max(1, |value|), partials
1e-12 relative to each vector's largest entry, optimised lengths 1e-6 relative (Newton
stops at tol = 1e-8 on either side), lnL after the sweep 1e-9 relative (north-star bound).
"""
import ctypes

import numpy as np
import pytest

from phylo_utils_amd import TreeModel
from phylo_utils_amd import _native as N
from phylo_utils_amd import substitution_models as SM
from phylo_utils_amd.likelihood import hip_likelihood_engine as E
from phylo_utils_amd.rate_models import GammaRateModel, InvariantGammaModel
from phylo_utils_amd.synthetic import CFG2_FREQS, CFG2_GTR_RATES, make_problem

pytestmark = pytest.mark.gpu


def _model(kind):
    if kind == "dna":
        return SM.GTR(CFG2_GTR_RATES, CFG2_FREQS), GammaRateModel(4, 0.5)
    return SM.LG(), GammaRateModel(4, 0.8)


def _setup(kind="dna", n_taxa=14, n_sites=700, seed=2, compact=True, keep=True):
    m, rm = _model(kind)
    K = len(m.freqs)
    tree, names, st = make_problem(n_taxa, n_sites, m, rm.rates, seed=seed)
    tm = TreeModel(device=0, keep_partials=keep, compact_tips=compact)
    if compact:
        tm.set_alignment_codes(st.astype(np.uint8), np.eye(K), names)
    else:  # dense fp64 tips (pu_set_tip_partials)
        tm.set_alignment_partials(np.eye(K)[st], names)
    tm.set_substitution_model(m)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    tr = tm.traversal
    tips = {tr.names[n]: np.eye(K)[st[i]] for i, n in enumerate(names)}
    return tm, m, rm, tr, tips


def _oracle_state(orc, tm, m, rm, tr, tips):
    ev, el, iv = m.engine_eigen()
    return orc.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                        tr.root_length(), ev, el, iv, m.freqs, rm.rates, rm.weights,
                        n_nodes=tr.n_nodes, return_all=True)


def _close(x, y, rtol):
    assert abs(x - y) <= rtol * max(1.0, abs(y)), (x, y, abs(x - y))


@pytest.mark.parametrize("kind", ["dna", "protein"])
def test_root_edge_lnl_bitwise_equals_traversal(kind):
    tm, m, rm, tr, tips = _setup(kind)
    site_trav = tm.sitewise_patterns().copy()
    lnl, site = tm._edge_lnl(*tr.root_edge)
    if kind == "dna":  # same P arithmetic, same fma chains, same logsumexp
        assert np.array_equal(site, site_trav)
    else:  # the traversal runs K = 20 on the MFMA units (different summation order)
        np.testing.assert_allclose(site, site_trav, rtol=1e-12, atol=1e-10)
    _close(lnl, tm.likelihood(), 1e-12)


@pytest.mark.parametrize("kind,compact", [("dna", True), ("dna", False), ("protein", True)])
def test_any_edge_uses_current_partials(oracle_mod, kind, compact):
    """compute_likelihood_at_edge off the root: the reference combines the nodes' stored
    (post-order) partials with P(0) / P(len) -- reproduced, not 'corrected'."""
    orc = oracle_mod
    tm, m, rm, tr, tips = _setup(kind, compact=compact)
    st = _oracle_state(orc, tm, m, rm, tr, tips)
    ev, el, iv = m.engine_eigen()
    P, S = st["partials"], st["scale"]
    for p, a, b in tr.postorder_traversal[:: max(1, len(tr.postorder_traversal) // 5)]:
        for u, v in ((int(a), int(p)), (int(p), int(b))):
            site = tm.compute_likelihood_at_edge(u, v)
            ref = orc.edge_lnl(P[u], S[u], P[v], S[v], ev, el, iv, tr.brlens[u, v], rm.rates,
                               rm.weights, m.freqs)
            np.testing.assert_allclose(site, ref, rtol=1e-12, atol=1e-9)
            # the root combine itself, on the device's own child partials (the K = 20
            # traversal's MFMA rounding already separates those from the oracle's ~1e-13)
            rp, rs = tm.root_partials, tm.root_scale
            gu, gsu = tm.node_partials(u)
            gv, gsv = tm.node_partials(v)
            cml = np.zeros(rs.shape)
            rref = orc.clv(orc.pmatrix(ev, el, iv, 0.0, rm.rates),
                           orc.pmatrix(ev, el, iv, tr.brlens[u, v], rm.rates),
                           gu, gv, gsu, gsv, cml)
            vscale = np.abs(rref).max(axis=-1, keepdims=True)
            assert np.all(np.abs(rp - rref) <= 1e-13 * vscale)
            np.testing.assert_allclose(rs, cml, rtol=1e-14, atol=1e-12)
    # the traversal's own results are untouched by the edge calls
    _close(tm.likelihood(), st["lnl"], 1e-12)
    np.testing.assert_allclose(tm.compute_likelihood_at_edge(*tr.root_edge), st["site_lnl"],
                               rtol=1e-12, atol=1e-9)
    t0, t1 = sorted(tr.names.values())[:2]  # two leaves are never adjacent (N > 3)
    with pytest.raises(ValueError, match="There is no edge"):
        tm.compute_likelihood_at_edge(t0, t1)


@pytest.mark.parametrize("kind", ["dna", "protein"])
def test_edge_derivatives_vs_oracle(oracle_mod, kind):
    orc = oracle_mod
    tm, m, rm, tr, tips = _setup(kind, n_sites=900)
    st = _oracle_state(orc, tm, m, rm, tr, tips)
    ev, el, iv = m.engine_eigen()
    P, S = st["partials"], st["scale"]
    a, b = tr.root_edge
    for t in (None, 1e-6, 0.05, 0.7, 3.0):
        got = tm.edge_derivatives(a, b, t)
        tt = tr.root_length() if t is None else t
        ref = orc.edge_derivs(P[a], S[a], P[b], S[b], ev, el, iv, tt, rm.rates, rm.weights,
                              m.freqs)
        for k in range(3):
            _close(got[k], ref[k], 1e-10)
    _close(tm.edge_derivatives(a, b)[0], tm.likelihood(), 1e-12)


@pytest.mark.parametrize("kind", ["dna", "protein"])
def test_reorientation_pulley_principle(oracle_mod, kind):
    """The optimising traversal's update rows on the device give the oracle's partials, and
    every re-oriented edge gives the root lnL."""
    orc = oracle_mod
    tm, m, rm, tr, tips = _setup(kind, n_taxa=11, n_sites=500, seed=9)
    st = _oracle_state(orc, tm, m, rm, tr, tips)
    ev, el, iv = m.engine_eigen()
    P, S = st["partials"], st["scale"]
    lnl0 = tm.likelihood()
    for row in tr.optimising_traversal:
        if row[0] >= 0:
            p, x, y = (int(v) for v in row[:3])
            bl = [tr.brlens[p, x], tr.brlens[p, y]]
            tm.update_partials([row[:3]], [bl])
            cml = np.zeros(S[p].shape)
            P[p] = orc.clv_c(orc.pmatrix(ev, el, iv, bl[0], rm.rates),
                             orc.pmatrix(ev, el, iv, bl[1], rm.rates), P[x], P[y], S[x], S[y],
                             cml)
            S[p] = cml
            gp, gs = tm.node_partials(p)
            scale = np.abs(P[p]).max(axis=-1, keepdims=True)
            assert np.all(np.abs(gp - P[p]) <= 1e-11 * scale)
            np.testing.assert_allclose(gs, S[p], rtol=1e-12, atol=1e-9)
        if row[3] >= 0:
            n, q = int(row[3]), int(row[4])
            _close(tm.edge_derivatives(n, q)[0], lnl0, 1e-11)


@pytest.mark.parametrize("kind,compact", [("dna", True), ("dna", False), ("protein", True)])
def test_optimise_sweep_vs_oracle(oracle_mod, kind, compact):
    orc = oracle_mod
    tm, m, rm, tr, tips = _setup(kind, n_taxa=10, n_sites=600, seed=4, compact=compact)
    ev, el, iv = m.engine_eigen()
    ops, bl0, root, rl0 = tr.postorder_traversal.copy(), tr.op_lengths(), tr.root_edge, \
        tr.root_length()
    lens, lnl_ref = orc.optimise_sweep(tips, ops, bl0, root, rl0, ev, el, iv, m.freqs,
                                       rm.rates, rm.weights, tr.optimising_traversal,
                                       tr.n_nodes)
    lnl0 = tm.likelihood()
    lnl = tm.optimise_branch_lengths(tol=1e-8, max_iter=50)
    assert lnl > lnl0
    _close(lnl, lnl_ref, 1e-9)
    for key, t in lens.items():
        got = tr.brlens[key]
        assert abs(got - t) <= 1e-6 * max(t, 1e-3), (key, got, t)
    # the device state is a consistent traversal at the new lengths
    _close(tm.likelihood(), lnl, 1e-12)
    ref2, _ = orc.tree_lnl(tips, ops, tr.op_lengths(), root, tr.root_length(), ev, el, iv,
                           m.freqs, rm.rates, rm.weights, n_nodes=tr.n_nodes)
    _close(lnl, ref2, 1e-12)


def test_optimise_single_edge_and_convergence():
    tm, m, rm, tr, tips = _setup("dna", n_taxa=8, n_sites=2000, seed=6)
    a, b = tr.root_edge
    lnl0 = tm.likelihood()
    t, lnl = tm.optimise_edge(a, b)
    assert lnl >= lnl0 - 1e-9 * abs(lnl0)
    assert abs(tr.brlens[a, b] - t) == 0.0
    d = tm.edge_derivatives(a, b)
    assert abs(d[1]) <= 1e-4 * abs(d[2]) or t <= 1.0001e-8  # stationary (or at the bound)
    _close(tm.likelihood(), lnl, 1e-12)
    # repeated sweeps converge
    l1 = tm.optimise_branch_lengths(sweeps=4, lnl_tol=1e-6)
    l2 = tm.optimise_branch_lengths(sweeps=1)
    assert l2 - l1 < 1e-3 and l1 >= lnl - 1e-9 * abs(lnl)


def test_edges_need_kept_partials():
    tm, m, rm, tr, tips = _setup("dna", keep=False)
    p, a, b = (int(v) for v in tr.postorder_traversal[0])
    with pytest.raises(ValueError, match="keep_partials"):
        tm.compute_likelihood_at_edge(a, p)
    with pytest.raises(ValueError):
        tm.optimise_branch_lengths()
    # the root edge itself still works from the traversal
    assert np.isfinite(tm.compute_likelihood_at_edge(*tr.root_edge)).all()


@pytest.mark.parametrize("K,C,S", [(4, 4, 333), (20, 3, 97), (5, 2, 64)])
def test_lnl_branch_dropin_vs_oracle(oracle_mod, K, C, S):
    orc = oracle_mod
    rng = np.random.default_rng(K + C)
    pi = rng.dirichlet(np.ones(K))
    probs = rng.dirichlet(np.ones(K), (C, K))
    a, b = rng.random((S, C, K)), rng.random((S, C, K))
    sa, sb = rng.normal(size=(S, C)), rng.normal(size=(S, C))
    np.testing.assert_allclose(E.lnl_branch(probs, pi, a, b, sa, sb),
                               orc.lnl_branch(probs, pi, a, b, sa, sb), rtol=1e-13, atol=1e-14)
    d3 = np.stack([probs, rng.normal(size=(C, K, K)), rng.normal(size=(C, K, K))], axis=1)
    got = E.lnl_branch_derivs(d3, pi, a, b, sa, sb)
    ref = orc.lnl_branch_derivs(d3, pi, a, b, sa, sb)
    assert got.shape == (S, C, 3)
    np.testing.assert_allclose(got, ref, rtol=1e-11, atol=1e-12)
    # probs varying along a leading loop dim (explicit index path) and scalar broadcasts
    pp = rng.dirichlet(np.ones(K), (S, 1, K))
    np.testing.assert_allclose(E.lnl_branch(pp, pi, a, b, 0.0, sb),
                               orc.lnl_branch(pp, pi, a, b, 0.0, sb), rtol=1e-13, atol=1e-14)
    out = np.empty(S)
    r = E.lnl_branch(probs[0], pi, a[:, 0], b[:, 0], sa[:, 0], sb[:, 0], out)
    assert r is out
    with pytest.raises(ValueError):
        E.lnl_branch(probs, pi[:-1], a, b, sa, sb)


# ---------------------------------------------------------------- ascertainment
@pytest.mark.parametrize("kind,ncat,weighted,compact", [
    ("dna", 1, False, True), ("dna", 1, False, False), ("dna", 4, True, True),
    ("dna", 4, False, True), ("protein", 1, False, True), ("protein", 4, True, True)])
def test_ascertainment_vs_oracle(oracle_mod, kind, ncat, weighted, compact):
    """Lewis correction (tree_model.py:92-98, 151-156, 209-214) against the oracle's
    restatement: sitewise 1e-12, total 1e-9 relative; the reference's unweighted form gives
    NaN for Gamma C > 1 and so does the engine."""
    orc = oracle_mod
    m, _ = _model(kind)
    rm = GammaRateModel(ncat, 0.5)
    K = len(m.freqs)
    tree, names, st = make_problem(12, 800, m, rm.rates, seed=21)
    tm = TreeModel(device=0, compact_tips=compact)
    if compact:
        tm.set_alignment_codes(st.astype(np.uint8), np.eye(K), names)
    else:
        tm.set_alignment_partials(np.eye(K)[st], names)
    tm.set_substitution_model(m)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.set_ascertainment_bias_correction(weighted=weighted)
    tm.initialise()
    tr = tm.traversal
    tips = {tr.names[n]: np.eye(K)[st[i]] for i, n in enumerate(names)}
    ev, el, iv = m.engine_eigen()
    lnl, site, corr = orc.tree_lnl_ascbias(tips, tr.postorder_traversal, tr.op_lengths(),
                                           tr.root_edge, tr.root_length(), ev, el, iv, m.freqs,
                                           rm.rates, rm.weights, n_nodes=tr.n_nodes,
                                           weighted=weighted)
    got_site = tm.compute_likelihood_at_edge(*tr.root_edge)
    assert got_site.shape == (800,)
    c = np.zeros(1)
    N.check(N.lib().pu_get_ascertainment_correction(tm._ctx, N.ptr(c)), tm._ctx)
    if np.isnan(corr):
        assert np.isnan(c[0]) and np.isnan(tm.likelihood())
        return
    np.testing.assert_allclose(c[0], corr, rtol=1e-12)
    np.testing.assert_allclose(got_site, site[:800], rtol=1e-12, atol=1e-9)
    _close(tm.likelihood(), lnl, 1e-9)
    # the root on another edge gets the same correction applied
    p, a, b = (int(v) for v in tr.postorder_traversal[-1])
    tm.compute_likelihood_at_edge(a, p)
    with pytest.raises(N.PhyloHipError):
        tm.edge_derivatives(*tr.root_edge)


@pytest.mark.parametrize("method", ["brent", "dbrent"])
def test_reference_minimisers_on_device_vs_oracle(oracle_mod, method):
    """optimise_branch_lengths / optimise_edge with the reference's brent / dbrent
    (src/optimisation.pyx, restated in phylo_utils_amd.optimisation and pinned bit for bit
    by tests/test_optimisation.py), every evaluation on the GPU, against the same pass on the
    CPU oracle.  Both minimise to tol = 1e-10 over [1e-8, 10]: lengths agree to 1e-6
    relative, the lnL to 1e-9, and the optimum agrees with Newton's to 1e-8 relative."""
    from phylo_utils_amd import optimisation as opt
    orc = oracle_mod
    tm, m, rm, tr, tips = _setup("dna", n_taxa=10, n_sites=800, seed=5)
    ev, el, iv = m.engine_eigen()
    ops, bl0, root, rl0 = tr.postorder_traversal.copy(), tr.op_lengths(), tr.root_edge, \
        tr.root_length()
    tol = 1e-10

    def edge_opt(evaluate, t0):
        out = np.zeros(3)
        f = lambda t: -evaluate(t)[0]
        if method == "brent":
            opt.brent(1e-8, min(max(t0, 1e-8), 10.0), 10.0, f, tol, out)
        else:
            opt.dbrent(1e-8, min(max(t0, 1e-8), 10.0), 10.0, f, lambda t: -evaluate(t)[1],
                       tol, out)
        return out[0]

    lens, lnl_ref = orc.optimise_sweep(tips, ops, bl0, root, rl0, ev, el, iv, m.freqs,
                                       rm.rates, rm.weights, tr.optimising_traversal,
                                       tr.n_nodes, edge_opt=edge_opt)
    lnl0 = tm.likelihood()
    lnl = tm.optimise_branch_lengths(tol=tol, method=method)
    assert lnl > lnl0
    _close(lnl, lnl_ref, 1e-9)
    for key, t in lens.items():
        got = tr.brlens[key]
        assert abs(got - t) <= 1e-6 * max(t, 1e-3), (key, got, t)
    _close(tm.likelihood(), lnl, 1e-12)
    # coordinate ascent: further passes converge, and Newton from there gains nothing
    lnl_c = tm.optimise_branch_lengths(tol=tol, method=method, sweeps=20, lnl_tol=1e-9)
    assert lnl_c >= lnl - 1e-9 * abs(lnl)
    lnl_n = tm.optimise_branch_lengths(tol=1e-8)
    assert abs(lnl_n - lnl_c) <= 1e-6, (lnl_n, lnl_c)
    # one edge: the minimiser's optimum is Newton's
    a, b = tr.root_edge
    t_m, l_m = tm.optimise_edge(a, b, tol=tol, method=method)
    t_n, l_n = tm.optimise_edge(a, b, tol=1e-10)
    assert abs(t_m - t_n) <= 1e-6 * max(t_n, 1e-3) and abs(l_m - l_n) <= 1e-10 * abs(l_n)
    with pytest.raises(ValueError):
        tm.optimise_edge(a, b, method="golden")


@pytest.mark.parametrize("method", ["brent", "dbrent"])
@pytest.mark.parametrize("ncat,n_sites", [(4, 3000), (1, 700), (4, 40000)])
def test_minimise_edge_state_machine_is_the_reference_minimiser(monkeypatch, method, ncat,
                                                                 n_sites):
    """pu_minimise_edge (r06) runs brent / dbrent (src/optimisation.pyx) as one state machine
    (pu_minimise.h) for both of its drivers.  Its host driver (PU_EDGE_DEVICE_NEWTON=0: one
    k_edge launch per evaluation) takes exactly the Python restatement's steps over the same
    evaluations (PU_PY_MINIMISE=1: phylo_utils_amd.optimisation over pu_edge_derivs, pinned
    bit for bit to the compiled reference by tests/test_optimisation.py): the same length, lnL
    and iteration count, bit for bit, from several starting lengths and brackets.  The device
    driver (one persistent launch, eigen-space evaluations) reaches the same optimum (dbrent to
    its tolerance, brent to 1e-6 relative) and lnL to 1e-12, in one launch per call."""
    m = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    rm = GammaRateModel(ncat, 0.5)
    tree, names, st = make_problem(14, n_sites, m, rm.rates, seed=41)
    tm = TreeModel(device=0)
    tm.set_alignment_codes(st.astype(np.uint8), np.eye(4), names)
    tm.set_substitution_model(m)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    a, b = tm.traversal.root_edge
    key = tuple(sorted((a, b)))
    t_true = tm.traversal.brlens[key]
    for t0, bracket, tol in ((t_true, (1e-8, 10.0), 1e-8), (0.5 * t_true, (1e-6, 2.0), 1e-10),
                             (3.0 * t_true, (1e-8, 10.0), 1.5e-8), (1e-8, (1e-8, 0.05), 1e-8)):
        res = {}
        for mode in ("py", "host", "device"):
            monkeypatch.setenv("PU_EDGE_DEVICE_NEWTON", "1" if mode == "device" else "0")
            if mode == "py":
                monkeypatch.setenv("PU_PY_MINIMISE", "1")
            else:
                monkeypatch.delenv("PU_PY_MINIMISE", raising=False)
            tm.traversal.brlens[key] = t0
            tm.update_branch_lengths()
            tm.likelihood()
            l0, e0 = _newton_stats(tm)
            t, lnl = tm.optimise_edge(a, b, tol=tol, method=method, bracket=bracket)
            l1, e1 = _newton_stats(tm)
            res[mode] = (t, lnl, tm.last_edge_evaluations, l1 - l0)
        assert res["host"][:3] == res["py"][:3], (t0, bracket, res)
        assert res["host"][3] == 0 and res["device"][3] == 1
        t_h, l_h = res["host"][:2]
        t_d, l_d = res["device"][:2]
        # brent compares f values only: near the optimum f is flat to its rounding (~1e-16
        # relative), so where the device's eigen-space f and k_edge's differ in the last bits
        # its comparisons can go the other way -- its optimum is resolved to ~sqrt(eps), 1e-7
        # relative (measured 3-7e-8); dbrent follows f' and agrees to its tolerance
        lim = (1e-6 if method == "brent" else 10 * tol) * max(t_h, 1e-3) + 1e-9
        assert abs(t_d - t_h) <= lim, (t_d, t_h)
        _close(l_d, l_h, 1e-12)


def test_site_sharded_optimisation_one_rank_equals_library_sweep(monkeypatch):
    """parallel.SiteShardedLikelihood.optimise_branch_lengths (the G1 x N1 driver: host
    Newton over all-reduced edge derivatives) on one rank takes exactly the library's
    pu_optimise_sweep steps when the library runs its host loop (PU_EDGE_DEVICE_NEWTON=0,
    the same evaluation arithmetic): the same lengths bit for bit and the same lnL."""
    monkeypatch.setenv("PU_EDGE_DEVICE_NEWTON", "0")
    from phylo_utils_amd.parallel import SiteShardedLikelihood, gpu_engine
    m, rm = _model("dna")
    tree, names, st = make_problem(12, 900, m, rm.rates, seed=8)
    codes = st.astype(np.uint8)
    sh = SiteShardedLikelihood(tree, codes, np.eye(4), names, m, rm,
                               engine_factory=gpu_engine(0))
    lnl_sh = sh.optimise_branch_lengths(tol=1e-8, max_iter=50)
    ref = gpu_engine(0)(tree, codes, np.eye(4), names, None, m, rm)
    lnl_ref = ref.optimise_branch_lengths(tol=1e-8, max_iter=50)
    assert sh.engine.traversal.brlens == ref.traversal.brlens
    assert lnl_sh == lnl_ref


def test_edge_derivative_paths_agree(monkeypatch):
    """The derivative evaluation's alternative paths (pu_edge.cpp, read per call): matrices in
    the launch (PU_EDGE_INLINE_P) or built per workgroup; partials summed by the host
    (PU_EDGE_HOST_SUM), by the k_edge_sum launch, or by a last-workgroup ticket
    (PU_EDGE_TWO_PASS=0).  They differ only in rounding: 1e-12 relative to max(1, |value|) on
    every edge, and a sweep lands on the same lengths to 1e-9."""
    tm, m, rm, tr, tips = _setup("dna", n_taxa=12, n_sites=900, seed=5)
    edges = [tuple(sorted(k)) for k in tr.brlens.keys()][:8]
    paths = [{}, {"PU_EDGE_INLINE_P": "0"}, {"PU_EDGE_HOST_SUM": "0"},
             {"PU_EDGE_INLINE_P": "0", "PU_EDGE_HOST_SUM": "0"}, {"PU_EDGE_TWO_PASS": "0"}]
    got = []
    for env in paths:
        for k in ("PU_EDGE_INLINE_P", "PU_EDGE_HOST_SUM", "PU_EDGE_TWO_PASS"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        got.append([tm.edge_derivatives(a, b) for a, b in edges])
    for g in got[1:]:
        for x, y in zip(np.ravel(g), np.ravel(got[0])):
            _close(x, y, 1e-12)
    for k in ("PU_EDGE_INLINE_P", "PU_EDGE_HOST_SUM", "PU_EDGE_TWO_PASS"):
        monkeypatch.delenv(k, raising=False)
    l_new = tm.optimise_branch_lengths(tol=1e-8, max_iter=50)
    len_new = dict(tm.traversal.brlens)
    tm2, *_ = _setup("dna", n_taxa=12, n_sites=900, seed=5)
    monkeypatch.setenv("PU_EDGE_INLINE_P", "0")
    monkeypatch.setenv("PU_EDGE_HOST_SUM", "0")
    l_old = tm2.optimise_branch_lengths(tol=1e-8, max_iter=50)
    for k, v in len_new.items():
        assert abs(tm2.traversal.brlens[k] - v) <= 1e-9 * max(v, 1e-3), k
    _close(l_new, l_old, 1e-12)


def _newton_stats(tm):
    launches, evals = ctypes.c_int(), ctypes.c_int()
    N.check(N.lib().pu_ctx_newton_stats(tm._ctx, ctypes.byref(launches), ctypes.byref(evals)),
            tm._ctx)
    return launches.value, evals.value


@pytest.mark.parametrize("ncat,n_sites", [(1, 700), (2, 5000), (4, 20000), (4, 900), ("+I", 6000)])
def test_device_newton_matches_the_host_loop(monkeypatch, ncat, n_sites):
    """Newton in one persistent launch (k_edge_newton, r06) takes newton()'s steps on the
    eigen-space form of the evaluation (K coefficients per site and category, pu_edge.hip):
    against the host loop of per-evaluation k_edge launches, the optimised length of one edge
    agrees to 1e-9 relative and its lnL to 1e-12, every length of a sweep to 1e-9 and the
    sweep's lnL to 1e-12 -- rounding only -- and every optimisation ran on the device."""
    m = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    # "+I": a rate-0 category, whose f_c is ~0 (either sign) at variable sites -- the kernel's
    # masked category mix (not every f_c > 0)
    rm = InvariantGammaModel(0.2, 3, 0.5) if ncat == "+I" else GammaRateModel(ncat, 0.5)
    tree, names, st = make_problem(16, n_sites, m, rm.rates, seed=31)

    def run(device):
        monkeypatch.setenv("PU_EDGE_DEVICE_NEWTON", "1" if device else "0")
        tm = TreeModel(device=0)
        tm.set_alignment_codes(st.astype(np.uint8), np.eye(4), names)
        tm.set_substitution_model(m)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        a, b = tm.traversal.root_edge
        t1, l1 = tm.optimise_edge(a, b, tol=1e-10)
        p, c1, _ = (int(v) for v in tm.traversal.postorder_traversal[2])
        t2, l2 = tm.optimise_edge(p, c1, tol=1e-8, max_iter=3)
        lnl = tm.optimise_branch_lengths(tol=1e-8, max_iter=50)
        return (t1, l1, t2, l2, lnl, dict(tm.traversal.brlens)), _newton_stats(tm)

    host, hs = run(False)
    dev, ds = run(True)
    assert hs == (0, 0)
    assert ds[0] == 2 + 2 * 16 - 3 and ds[1] > ds[0]  # every optimisation ran on the device
    for i in (0, 2):
        assert abs(dev[i] - host[i]) <= 1e-9 * max(host[i], 1e-3), (i, dev[i], host[i])
    for i in (1, 3, 4):
        _close(dev[i], host[i], 1e-12)
    for k, v in host[5].items():
        assert abs(dev[5][k] - v) <= 1e-9 * max(v, 1e-3), (k, dev[5][k], v)


def test_device_newton_timeout_falls_back_to_the_host_loop(monkeypatch):
    """A grid whose workgroups give up waiting (PU_NT_SPINS=1: one poll each, as when part of
    the grid never becomes resident) leaves without a result and the optimisation runs on the
    host loop: the same lengths and lnL as PU_EDGE_DEVICE_NEWTON=0, bit for bit, no device
    evaluation counted, and the next launch (slots started afresh) is exact again."""
    m = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    rm = GammaRateModel(4, 0.5)
    tree, names, st = make_problem(12, 40000, m, rm.rates, seed=33)

    def run(mode, spins=None):
        monkeypatch.setenv("PU_EDGE_DEVICE_NEWTON", mode)
        if spins:
            monkeypatch.setenv("PU_NT_SPINS", spins)
        else:
            monkeypatch.delenv("PU_NT_SPINS", raising=False)
        tm = TreeModel(device=0)
        tm.set_alignment_codes(st.astype(np.uint8), np.eye(4), names)
        tm.set_substitution_model(m)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        a, b = tm.traversal.root_edge
        return tm, tm.optimise_edge(a, b, tol=1e-10), (a, b)

    _, host, _ = run("0")
    tm, timed_out, (a, b) = run("1", spins="1")
    assert timed_out == host
    launches, evals = _newton_stats(tm)
    assert launches == 1 and evals == 0
    monkeypatch.delenv("PU_NT_SPINS")
    tm.traversal.brlens[tuple(sorted((a, b)))] *= 1.7
    tm.update_branch_lengths()
    tm.likelihood()
    t, lnl = tm.optimise_edge(a, b, tol=1e-10)
    assert _newton_stats(tm) == (2, _newton_stats(tm)[1]) and _newton_stats(tm)[1] > 0
    assert abs(t - host[0]) <= 1e-9 * host[0]
    _close(lnl, host[1], 1e-12)


def test_device_newton_from_two_threads():
    """Two contexts on one device optimised from two host threads at once (ctypes drops the
    GIL): the device-Newton grids take turns (one per device at a time in a process), each
    context's results are those of running it alone, bit for bit."""
    import threading
    m = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    rm = GammaRateModel(4, 0.5)
    probs = [make_problem(12, n, m, rm.rates, seed=50 + n) for n in (20000, 9000)]

    def build(k):
        tree, names, st = probs[k]
        tm = TreeModel(device=0)
        tm.set_alignment_codes(st.astype(np.uint8), np.eye(4), names)
        tm.set_substitution_model(m)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        return tm

    def work(tm, out):
        a, b = tm.traversal.root_edge
        res = [tm.optimise_edge(a, b, tol=1e-10)]
        for _ in range(3):
            res.append(tm.optimise_branch_lengths(tol=1e-8))
        out.append((res, dict(tm.traversal.brlens), _newton_stats(tm)))

    alone = []
    for k in range(2):
        work(build(k), alone)
    tms = [build(0), build(1)]
    outs = [[], []]
    ths = [threading.Thread(target=work, args=(tms[k], outs[k])) for k in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for k in range(2):
        assert outs[k][0][0] == alone[k][0] and outs[k][0][1] == alone[k][1], k
        assert outs[k][0][2][0] > 0  # every optimisation ran on the device


def test_device_newton_falls_back_to_the_host_loop(monkeypatch):
    """Contexts the persistent kernel does not take (C > 4 here) run the host loop, with the
    same steps as before."""
    monkeypatch.delenv("PU_EDGE_DEVICE_NEWTON", raising=False)
    m = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    rm = GammaRateModel(8, 0.5)
    tree, names, st = make_problem(10, 500, m, rm.rates, seed=32)
    tm = TreeModel(device=0)
    tm.set_alignment_codes(st.astype(np.uint8), np.eye(4), names)
    tm.set_substitution_model(m)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    lnl0 = tm.likelihood()
    assert tm.optimise_branch_lengths() > lnl0
    assert _newton_stats(tm) == (0, 0)
