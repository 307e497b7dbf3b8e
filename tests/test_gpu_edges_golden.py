"""SURVEY 8(f) N1 on the GPU against fixtures generated from the reference
(tests/golden/make_golden.py make_edges / make_cfg5_small):
* the drop-in lnl_branch / lnl_branch_derivs (pu_lnl_branch*) vs the reference's python
  engine (python_likelihood_engine.py:40-46 == numba_likelihood_engine.py:49-57);
* pu_edge_derivs at the root edge of a context built through the C ABI on the fixture's own
  schedule vs the reference's per-category derivatives on its own post-order partials, mixed
  over the rate categories (the chain-rule factor r included);
* a reduced cfg5: 4 x 100-taxon trees on one resident 2k-site alignment (TreeModel.set_tree
  re-binds the tips) vs the reference's lnL.
Tolerances as tests/test_edges_golden.py: lnL 1e-10 relative, derivatives 1e-8 relative."""
import ctypes

import numpy as np
import pytest

from edge_golden import cfg5_small, edges, tree_problem

from phylo_utils_amd import TreeModel
from phylo_utils_amd import _native as N
from phylo_utils_amd import alignment as A
from phylo_utils_amd import substitution_models as SM
from phylo_utils_amd.likelihood import hip_likelihood_engine as E
from phylo_utils_amd.rate_models import GammaRateModel
from phylo_utils_amd.synthetic import CFG2_FREQS, CFG2_GTR_RATES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["gtr", "lg"])
def test_dropin_lnl_branch_derivs_vs_reference(name):
    g = edges()
    k = lambda x: g["seam_%s_%s" % (name, x)]
    got = E.lnl_branch_derivs(k("probs3"), k("pi"), k("clv_a"), k("clv_b"), k("sa"), k("sb"))
    np.testing.assert_allclose(got, k("derivs"), rtol=1e-12, atol=1e-12)
    lnl = E.lnl_branch(np.ascontiguousarray(k("probs3")[:, 0]), k("pi"), k("clv_a"), k("clv_b"),
                       k("sa"), k("sb"))
    np.testing.assert_allclose(lnl, k("lnl"), rtol=1e-13)


@pytest.mark.parametrize("name", ["tree_gtr", "tree_lg"])
def test_edge_derivatives_vs_reference(name):
    p = tree_problem(edges(), name)
    m = p["model"]
    ev, el, iv = m.engine_eigen()
    K = len(m.freqs)
    nodes = np.array(sorted(p["tips"]), dtype=np.int32)
    part = np.ascontiguousarray(np.stack([p["tips"][int(n)] for n in nodes]))
    S = part.shape[1]
    ops = np.ascontiguousarray(p["ops"], dtype=np.int32)
    a, b = p["root_edge"]
    ctx = ctypes.c_void_p()
    N.check(N.lib().pu_ctx_create(ctypes.byref(ctx), 0, p["n_nodes"], len(nodes), S, len(
        p["rates"]), K, 0))
    try:
        N.check(N.lib().pu_set_tips(ctx, len(nodes), N.ptr(nodes), 0, None, None, N.ptr(part),
                                    None), ctx)
        N.check(N.lib().pu_set_model(ctx, N.ptr(ev), N.ptr(el), N.ptr(iv),
                                     N.ptr(N.f64(m.freqs)), N.ptr(N.f64(p["rates"])),
                                     N.ptr(N.f64(p["weights"]))), ctx)
        N.check(N.lib().pu_set_schedule(ctx, len(ops), N.ptr(ops), N.ptr(N.f64(p["lens"])), a, b,
                                        p["root_len"]), ctx)
        lnl = ctypes.c_double()
        N.check(N.lib().pu_run(ctx, ctypes.byref(lnl), None), ctx)
        ref0 = p["totals"][0][0]
        assert abs(lnl.value - ref0) <= 1e-10 * abs(ref0)
        out = np.zeros(3)
        for i, t in enumerate(p["t"]):
            N.check(N.lib().pu_edge_derivs(ctx, a, b, float(t), N.ptr(out)), ctx)
            ref = p["totals"][i]
            assert abs(out[0] - ref[0]) <= 1e-10 * abs(ref[0]), (t, out, ref)
            for k in (1, 2):
                assert abs(out[k] - ref[k]) <= 1e-8 * max(abs(ref[k]), 1.0), (t, k, out, ref)
    finally:
        N.lib().pu_ctx_destroy(ctx)


def test_cfg5_small_trees_on_one_resident_alignment_vs_reference():
    seqs, trees, lnl, rates, weights = cfg5_small()
    rm = GammaRateModel(4, 0.5)
    np.testing.assert_array_equal(rm.rates, rates)
    tm = TreeModel(keep_partials=False)
    tm.set_alignment([("t%d" % i, s) for i, s in enumerate(seqs)], A.DNA, compress=False)
    tm.set_substitution_model(SM.GTR(CFG2_GTR_RATES, CFG2_FREQS))
    tm.set_rate_model(rm)
    for nwk, ref in zip(trees, lnl):
        tm.set_tree(nwk)
        tm.initialise()
        got = tm.likelihood()
        assert abs(got - ref) <= 1e-10 * abs(ref), (got, ref)
