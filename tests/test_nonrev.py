"""Non-reversible DNA models (Strsym, Unrest; substitution_models/abstract.py:163-180,
strsym.py, unrest.py) on host-supplied transition matrices.

The reference's TreeModel feeds clv whatever Model.p returns (tree_model.py:166-169,
:189-190); for these models that is expm(Q r t) with no eigen step.  The engine takes
those matrices through pu_set_model_p + pu_set_pmatrices (include/phylo_hip.h).  Golden
vectors: tests/golden/nonrev.npz (tests/golden/make_golden.py nonrev, the reference's
Unrest/Strsym and python engine).  Tolerances as tests/test_gpu_parity.py: sitewise 1e-12
relative (1e-9 absolute), total lnL 1e-9 relative.
"""
import ctypes

import numpy as np
import pytest

from conftest import golden_charmap, load_golden

from phylo_utils_amd import substitution_models as SM

LNL_RTOL = 1e-9
CASES = ["unrest_g4", "strsym_g1", "unrest_deep"]


def _golden():
    return load_golden("nonrev")


def _model(g, name):
    if name.startswith("unrest"):
        return SM.Unrest(g["unrest_rates"])
    return SM.Strsym(list(g["strsym_rates"]))


def _case(name):
    g = _golden()
    d = {k[len(name) + 1:]: g[k] for k in g.files if k.startswith(name + "_")}
    d["seq_strings"] = ["".join(map(chr, row)) for row in d["seqs"]]
    cm = golden_charmap("dna")
    d["tips"] = {int(i): np.array([cm[ch] for ch in s])
                 for i, s in zip(d["tip_index"], d["seq_strings"])}
    d["model"] = _model(g, name)
    return d


def _pmatrices(model, rates, lens, root_len):
    """[n_ops + 1][2][C][K][K]: per op (child1, child2), then (root_a P(0), root_b P(len))."""
    P = [np.stack([model.p(l1, rates), model.p(l2, rates)]) for l1, l2 in lens]
    P.append(np.stack([model.p(0, rates), model.p(root_len, rates)]))
    return np.ascontiguousarray(np.stack(P), dtype=np.float64)


# ------------------------------------------------------------------ CPU: mirror + oracle
def test_p_derivative_chain_rule_on_reference_forms():
    """Model.p_derivative = r x the reference's dp_dt / d2p_dt2 at (t, rates) (edges.npz from
    the reference's Unrest, GTR, LG), and matches central differences of P(t r)."""
    from edge_golden import MODELS, edges
    g = edges()
    for name in ("unrest", "gtr", "lg"):
        mdl = MODELS[name]()
        r = g["rates"]
        for i, t in enumerate(g["ts"]):
            np.testing.assert_allclose(mdl.p_derivative(t, r, 1),
                                       g[name + "_dp"][i] * r[:, None, None], rtol=1e-12,
                                       atol=1e-14)
            np.testing.assert_allclose(mdl.p_derivative(t, r, 2),
                                       g[name + "_d2p"][i] * (r * r)[:, None, None],
                                       rtol=1e-11, atol=1e-13)
        h, t = 1e-5, 0.3
        fd = (mdl.p_derivative(t + h, r, 0) - mdl.p_derivative(t - h, r, 0)) / (2 * h)
        np.testing.assert_allclose(mdl.p_derivative(t, r, 1), fd, rtol=1e-6, atol=1e-8)


def test_oracle_host_matrix_sweep_equals_eigen_sweep(oracle_mod):
    """optimise_sweep_p on the eigen form's matrix function reproduces optimise_sweep (the
    sweep the GPU Newton is pinned to), so the non-reversible GPU test inherits that pin."""
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import CFG2_FREQS, CFG2_GTR_RATES, make_problem
    from phylo_utils_amd.tree import Traversal, prepare_tree
    m = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    rm = GammaRateModel(4, 0.5)
    tree, names, states = make_problem(12, 300, m, rm.rates, seed=5)
    tr = Traversal(prepare_tree(tree))
    tips = {tr.names[n]: np.eye(4)[states[i]] for i, n in enumerate(names)}
    ev, el, iv = m.engine_eigen()
    rows = tr.optimising_traversal
    l1, lnl1 = oracle_mod.optimise_sweep(tips, tr.postorder_traversal, tr.op_lengths(),
                                         tr.root_edge, tr.root_length(), ev, el, iv, m.freqs,
                                         rm.rates, rm.weights, rows, tr.n_nodes)
    pm = lambda t, k: oracle_mod.pmatrix_deriv(ev, el, iv, t, rm.rates, k)
    l2, lnl2 = oracle_mod.optimise_sweep_p(tips, tr.postorder_traversal, tr.op_lengths(),
                                           tr.root_edge, tr.root_length(), pm, m.freqs,
                                           rm.weights, rows, tr.n_nodes)
    assert abs(lnl1 - lnl2) <= 1e-12 * abs(lnl1)
    for k in l1:
        assert abs(l1[k] - l2[k]) <= 1e-9 * max(l1[k], 1e-8)
@pytest.mark.parametrize("name", ["unrest", "strsym"])
def test_nonrev_models_match_reference(name):
    g = _golden()
    m = _model(g, name)
    assert not m.reversible
    np.testing.assert_allclose(m.q(), g[name + "_q"], rtol=1e-15, atol=1e-15)
    np.testing.assert_allclose(m.freqs, g[name + "_freqs"], rtol=1e-13, atol=1e-15)
    for i, t in enumerate(g["ts"]):
        np.testing.assert_allclose(m.p(t, g["rates"]), g[name + "_p"][i], rtol=1e-13,
                                   atol=1e-16, err_msg="t=%g" % t)
    with pytest.raises(NotImplementedError):
        m.engine_eigen()


@pytest.mark.parametrize("name", CASES)
def test_nonrev_tree_lnl_matches_reference(oracle_mod, name):
    c = _case(name)
    P = _pmatrices(c["model"], c["rates"], c["lens"], float(c["root_len"]))
    res = oracle_mod.tree_lnl_p(c["tips"], c["ops"], P[:-1], P[-1], tuple(c["root_edge"]),
                                c["model"].freqs, c["weights"], n_nodes=int(c["n_nodes"]),
                                return_all=True)
    np.testing.assert_allclose(res["site_lnl"], c["site_lnl"], rtol=1e-12, atol=1e-10)
    assert abs(res["lnl"] - float(c["lnl"])) <= 1e-11 * abs(float(c["lnl"]))
    if name == "unrest_deep":
        assert np.count_nonzero(res["scale"]) > 0  # the 2^-128 rescale is exercised


# ------------------------------------------------------------------ GPU: the C ABI
def _ctx_for(c, dense, n_nodes=None):
    from phylo_utils_amd import _native as N
    nodes = np.array(sorted(c["tips"]), dtype=np.int32)
    part = np.ascontiguousarray(np.stack([c["tips"][int(n)] for n in nodes]), dtype=np.float64)
    table, codes = np.unique(part.reshape(-1, 4), axis=0, return_inverse=True)
    codes = np.ascontiguousarray(codes.reshape(len(nodes), -1).astype(np.uint8))
    table = np.ascontiguousarray(table)
    S = part.shape[1]
    C = len(c["rates"])
    ctx = ctypes.c_void_p()
    N.check(N.lib().pu_ctx_create(ctypes.byref(ctx), 0, int(n_nodes or c["n_nodes"]),
                                  len(nodes), S, C, 4, 0))
    w = np.ones(S)
    N.check(N.lib().pu_set_tips(ctx, len(nodes), N.ptr(nodes), len(table), N.ptr(table),
                                None if dense else N.ptr(codes),
                                N.ptr(part) if dense else None, N.ptr(w)), ctx)
    return ctx, S


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("dense", [False, True])
def test_gpu_nonrev_golden(oracle_mod, name, dense):
    from phylo_utils_amd import _native as N
    c = _case(name)
    m = c["model"]
    ops = np.ascontiguousarray(c["ops"], dtype=np.int32)
    lens = N.f64(c["lens"])
    a, b = (int(x) for x in c["root_edge"])
    rl = float(c["root_len"])
    P = _pmatrices(m, c["rates"], c["lens"], rl)
    ref_lnl, ref_site = oracle_mod.tree_lnl_p(c["tips"], ops, P[:-1], P[-1], (a, b), m.freqs,
                                              c["weights"], n_nodes=int(c["n_nodes"]))
    ctx, S = _ctx_for(c, dense)
    try:
        N.check(N.lib().pu_set_model_p(ctx, N.ptr(N.f64(m.freqs)), N.ptr(N.f64(c["rates"])),
                                       N.ptr(N.f64(c["weights"]))), ctx)
        N.check(N.lib().pu_set_schedule(ctx, len(ops), N.ptr(ops), N.ptr(lens), a, b, rl), ctx)
        N.check(N.lib().pu_set_pmatrices(ctx, N.ptr(P)), ctx)
        lnl, site = ctypes.c_double(), np.zeros(S)
        N.check(N.lib().pu_run(ctx, ctypes.byref(lnl), N.ptr(site)), ctx)
        back = np.zeros_like(P)
        N.check(N.lib().pu_get_pmatrices(ctx, N.ptr(back)), ctx)
    finally:
        N.lib().pu_ctx_destroy(ctx)
    np.testing.assert_array_equal(back, P)  # stored as given, in the caller's order
    np.testing.assert_allclose(site, c["site_lnl"], rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(site, ref_site, rtol=1e-12, atol=1e-10)
    assert abs(lnl.value - float(c["lnl"])) <= LNL_RTOL * abs(float(c["lnl"]))


@pytest.mark.gpu
def test_gpu_nonrev_state_errors():
    """Stale matrices after new lengths, edge operations and pu_set_pmatrices without
    pu_set_model_p all fail with PU_E_STATE; pu_set_model switches back to device P."""
    from phylo_utils_amd import _native as N
    c = _case("unrest_g4")
    m = c["model"]
    ops = np.ascontiguousarray(c["ops"], dtype=np.int32)
    lens = N.f64(c["lens"])
    a, b = (int(x) for x in c["root_edge"])
    rl = float(c["root_len"])
    P = _pmatrices(m, c["rates"], c["lens"], rl)
    fr, rates, w = N.f64(m.freqs), N.f64(c["rates"]), N.f64(c["weights"])
    ctx, S = _ctx_for(c, False)
    lib = N.lib()
    try:
        gtr = SM.GTR()
        ev, el, iv = gtr.engine_eigen()
        N.check(lib.pu_set_model(ctx, N.ptr(ev), N.ptr(el), N.ptr(iv), N.ptr(fr), N.ptr(rates),
                                 N.ptr(w)), ctx)
        N.check(lib.pu_set_schedule(ctx, len(ops), N.ptr(ops), N.ptr(lens), a, b, rl), ctx)
        assert lib.pu_set_pmatrices(ctx, N.ptr(P)) == N.PU_E_STATE  # eigen mode
        lnl = ctypes.c_double()
        N.check(lib.pu_run(ctx, ctypes.byref(lnl), None), ctx)
        N.check(lib.pu_set_model_p(ctx, N.ptr(fr), N.ptr(rates), N.ptr(w)), ctx)
        assert lib.pu_run(ctx, ctypes.byref(lnl), None) == N.PU_E_STATE  # no P yet
        N.check(lib.pu_set_pmatrices(ctx, N.ptr(P)), ctx)
        N.check(lib.pu_run(ctx, ctypes.byref(lnl), None), ctx)
        first = lnl.value
        assert abs(first - float(c["lnl"])) <= LNL_RTOL * abs(float(c["lnl"]))
        # edge kernels build P from an eigen-decomposition or take it from a provider: refused
        # without one
        out3 = np.zeros(3)
        assert lib.pu_edge_derivs(ctx, a, b, rl, N.ptr(out3)) == N.PU_E_STATE
        # new lengths make the host matrices stale until they are set again
        N.check(lib.pu_set_branch_lengths(ctx, N.ptr(lens * 1.5), rl * 1.5), ctx)
        assert lib.pu_run(ctx, ctypes.byref(lnl), None) == N.PU_E_STATE
        P2 = _pmatrices(m, c["rates"], c["lens"] * 1.5, rl * 1.5)
        N.check(lib.pu_set_pmatrices(ctx, N.ptr(P2)), ctx)
        N.check(lib.pu_run(ctx, ctypes.byref(lnl), None), ctx)
        assert lnl.value != first
        bad = P2.copy()
        bad[0, 0, 0, 0, 0] = np.nan
        assert lib.pu_set_pmatrices(ctx, N.ptr(bad)) == N.PU_E_ARG
        # back to the eigen path: no host matrices needed
        N.check(lib.pu_set_model(ctx, N.ptr(ev), N.ptr(el), N.ptr(iv), N.ptr(fr), N.ptr(rates),
                                 N.ptr(w)), ctx)
        N.check(lib.pu_run(ctx, ctypes.byref(lnl), None), ctx)
    finally:
        lib.pu_ctx_destroy(ctx)


@pytest.mark.gpu
@pytest.mark.parametrize("keep", [True, False])
def test_gpu_treemodel_unrest_vs_oracle(oracle_mod, keep):
    """TreeModel with Unrest + Gamma: its own traversal and root edge, matrices from the
    host mirror (Model.p), against the oracle on the same schedule; then new lengths."""
    from phylo_utils_amd import TreeModel
    from phylo_utils_amd import alignment as A
    from phylo_utils_amd.rate_models import GammaRateModel
    c = _case("unrest_g4")
    m = c["model"]
    rm = GammaRateModel(4, 0.5)
    tm = TreeModel(keep_partials=keep)
    tm.set_alignment([("t%d" % i, s) for i, s in enumerate(c["seq_strings"])], A.DNA,
                     compress=False)
    tm.set_substitution_model(m)
    tm.set_rate_model(rm)
    tm.set_tree(bytes(c["newick"]).decode())
    tm.initialise()
    cm = golden_charmap("dna")

    def oracle():
        tr = tm.traversal
        tips = {tr.names["t%d" % i]: np.array([cm[ch] for ch in s])
                for i, s in enumerate(c["seq_strings"])}
        P = _pmatrices(m, rm.rates, tr.op_lengths(), tr.root_length())
        return oracle_mod.tree_lnl_p(tips, tr.postorder_traversal, P[:-1], P[-1],
                                     tr.root_edge, m.freqs, rm.weights, n_nodes=tr.n_nodes)

    ref_lnl, ref_site = oracle()
    assert abs(tm.likelihood() - ref_lnl) <= LNL_RTOL * abs(ref_lnl)
    np.testing.assert_allclose(tm.sitewise_patterns(), ref_site, rtol=1e-12, atol=1e-10)
    for k in list(tm.traversal.brlens):
        tm.traversal.brlens[k] = tm.traversal.brlens[k] * 0.7
    tm.update_branch_lengths()
    ref_lnl2, _ = oracle()
    assert ref_lnl2 != ref_lnl
    assert abs(tm.likelihood() - ref_lnl2) <= LNL_RTOL * abs(ref_lnl2)
    if not keep:
        with pytest.raises(RuntimeError):  # edge operations need the kept partials
            tm.edge_derivatives(*tm.traversal.root_edge)
        return
    # edge derivatives on host matrices (the provider) vs the oracle on the same matrices
    tr = tm.traversal
    tips = {tr.names["t%d" % i]: np.array([cm[ch] for ch in s])
            for i, s in enumerate(c["seq_strings"])}
    P = _pmatrices(m, rm.rates, tr.op_lengths(), tr.root_length())
    st = oracle_mod.tree_lnl_p(tips, tr.postorder_traversal, P[:-1], P[-1], tr.root_edge,
                               m.freqs, rm.weights, n_nodes=tr.n_nodes, return_all=True)
    a, b = tr.root_edge
    for t in (1e-5, 0.05, tr.root_length(), 1.3):
        got = tm.edge_derivatives(a, b, t)
        mats = [m.p_derivative(0.0, rm.rates, 0)] + [m.p_derivative(t, rm.rates, k)
                                                      for k in range(3)]
        ref = oracle_mod.edge_derivs_p(st["partials"][a], st["scale"][a], st["partials"][b],
                                       st["scale"][b], mats, rm.weights, m.freqs)
        assert abs(got[0] - ref[0]) <= 1e-10 * abs(ref[0])
        for k in (1, 2):
            assert abs(got[k] - ref[k]) <= 1e-8 * max(abs(ref[k]), 1.0), (t, k, got, ref)


@pytest.mark.gpu
def test_gpu_unrest_branch_length_optimisation_vs_oracle(oracle_mod):
    """optimise_branch_lengths on Unrest + Gamma (the reference's Unrest fixture): the
    library's Newton sweep over the optimising traversal with P, dP/dt, d2P/dt2 from the host
    provider (expm(Q r t), r Q expm, r^2 Q^2 expm) against oracle.optimise_sweep_p on the same
    matrix function.  Lengths agree to 1e-6 relative, the final lnL to 1e-9."""
    from phylo_utils_amd import TreeModel
    from phylo_utils_amd import alignment as A
    from phylo_utils_amd.rate_models import GammaRateModel
    c = _case("unrest_g4")
    m = c["model"]
    rm = GammaRateModel(4, 0.5)
    tm = TreeModel()
    tm.set_alignment([("t%d" % i, s) for i, s in enumerate(c["seq_strings"])], A.DNA,
                     compress=False)
    tm.set_substitution_model(m)
    tm.set_rate_model(rm)
    tm.set_tree(bytes(c["newick"]).decode())
    tm.initialise()
    tr = tm.traversal
    cm = golden_charmap("dna")
    tips = {tr.names["t%d" % i]: np.array([cm[ch] for ch in s])
            for i, s in enumerate(c["seq_strings"])}
    rows = tr.optimising_traversal
    lens_ref, lnl_ref = oracle_mod.optimise_sweep_p(
        tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge, tr.root_length(),
        lambda t, k: m.p_derivative(t, rm.rates, k), m.freqs, rm.weights, rows, tr.n_nodes)
    lnl0 = tm.likelihood()
    lnl = tm.optimise_branch_lengths(tol=1e-8, max_iter=50)
    assert lnl > lnl0
    assert abs(lnl - lnl_ref) <= 1e-9 * abs(lnl_ref), (lnl, lnl_ref)
    for key, t in lens_ref.items():
        assert abs(tr.brlens[key] - t) <= 1e-6 * max(t, 1e-6), (key, tr.brlens[key], t)



@pytest.mark.gpu
def test_gpu_unrest_invariant_gamma_edge_derivatives_deep_tree():
    """Unrest + I + Gamma on host matrices.  P(0) = expm(0) = I exactly, so the
    invariant category's CLV is exactly zero at variable sites and keeps an unrescaled
    scaler, while the Gamma categories' scalers reach thousands of nats on a 700-taxon tree
    with long branches.  The edge derivatives' category mix must ignore the f = 0 category
    (lnl_node's -inf, numba_likelihood_engine.py:82-87): lnL at the root edge equals the
    traversal's and the derivatives match central differences of it."""
    from phylo_utils_amd import TreeModel
    from phylo_utils_amd.rate_models import InvariantGammaModel
    from phylo_utils_amd.synthetic import make_problem
    m = _model(_golden(), "unrest_g4")
    rm = InvariantGammaModel(0.2, 4, 0.5)
    tree, names, states = make_problem(700, 96, m, rm.rates, seed=4, lo=0.4, hi=1.2)
    tm = TreeModel()
    tm.set_alignment_partials(np.eye(4)[states], names)
    tm.set_substitution_model(m)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    lnl = tm.likelihood()
    assert np.isfinite(lnl)
    rs = tm.root_scale  # [S][C]
    assert (rs[:, 1:].min(axis=1) - rs[:, 0]).min() < -745.0  # the underflow regime
    a, b = tm.traversal.root_edge
    t0 = tm.traversal.brlens[a, b]
    l0, d1, d2 = tm.edge_derivatives(a, b)
    assert np.isfinite([l0, d1, d2]).all(), (l0, d1, d2)
    assert abs(l0 - lnl) <= 1e-9 * abs(lnl), (l0, lnl)
    h = 1e-4 * max(t0, 1e-3)
    lp = tm.edge_derivatives(a, b, t0 + h)[0]
    lm = tm.edge_derivatives(a, b, t0 - h)[0]
    assert abs(d1 - (lp - lm) / (2 * h)) <= 1e-4 * max(1.0, abs(d1)), (d1, (lp - lm) / (2 * h))
    assert abs(d2 - (lp - 2 * l0 + lm) / h ** 2) <= 1e-2 * max(1.0, abs(d2))
