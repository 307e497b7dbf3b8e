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
        # edge kernels build P from an eigen-decomposition: refused
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
    with pytest.raises(RuntimeError):
        tm.edge_derivatives(*tm.traversal.root_edge)

