"""SURVEY 8(f) N1 pinned on the reference (CPU): the host models' dp_dt / d2p_dt2
(abstract.py:61-77, 180-192, the reference's own forms, chain-rule factor r omitted as
there), the oracle's lnl_branch / lnl_branch_derivs against the reference's python engine
(python_likelihood_engine.py:40-46 == numba_likelihood_engine.py:49-57), the oracle's
root-edge derivatives of the rate mixture against the reference's per-category derivatives on
its own post-order partials, and a reduced cfg5 (4 x 100-taxon trees on one 2k-site
alignment).  Tolerances: matrices 1e-12 relative to the largest entry;
lnL 1e-10 relative; derivatives 1e-8 relative (sums of ~1e2-1e3 terms of mixed sign)."""
import numpy as np
import pytest

from edge_golden import MODELS, cfg5_small, edges, tree_problem

from phylo_utils_amd import alignment as A
from phylo_utils_amd import substitution_models as SM
from phylo_utils_amd.synthetic import CFG2_FREQS, CFG2_GTR_RATES
from phylo_utils_amd.tree import Traversal, prepare_tree, parse_newick


def _mat_close(got, ref, rtol=1e-12):
    scale = np.abs(ref).max()
    assert np.abs(got - ref).max() <= rtol * scale, np.abs(got - ref).max() / scale


@pytest.mark.parametrize("name", ["gtr", "lg", "unrest"])
def test_model_derivatives_match_reference(name):
    g = edges()
    m = MODELS[name]()
    for i, t in enumerate(g["ts"]):
        _mat_close(np.asarray(m.dp_dt(t, g["rates"])), g[name + "_dp"][i])
        _mat_close(np.asarray(m.d2p_dt2(t, g["rates"])), g[name + "_d2p"][i])
        _mat_close(np.asarray(m.dp_dt(t)), g[name + "_dp1"][i])
        _mat_close(np.asarray(m.d2p_dt2(t)), g[name + "_d2p1"][i])


@pytest.mark.parametrize("name", ["gtr", "lg"])
def test_oracle_lnl_branch_derivs_match_reference(oracle_mod, name):
    g = edges()
    k = lambda x: g["seam_%s_%s" % (name, x)]
    probs = np.broadcast_to(k("probs3"), k("clv_a").shape[:1] + k("probs3").shape)
    got = oracle_mod.lnl_branch_derivs(probs, k("pi"), k("clv_a"), k("clv_b"), k("sa"), k("sb"))
    np.testing.assert_allclose(got, k("derivs"), rtol=1e-12, atol=1e-12)
    lnl = oracle_mod.lnl_branch(probs[:, :, 0], k("pi"), k("clv_a"), k("clv_b"), k("sa"), k("sb"))
    np.testing.assert_allclose(lnl, k("lnl"), rtol=1e-13)


@pytest.mark.parametrize("name", ["tree_gtr", "tree_lg"])
def test_oracle_edge_derivatives_match_reference(oracle_mod, name):
    p = tree_problem(edges(), name)
    m = p["model"]
    ev, el, iv = m.engine_eigen()
    st = oracle_mod.tree_lnl(p["tips"], p["ops"], p["lens"], p["root_edge"], p["root_len"],
                             ev, el, iv, m.freqs, p["rates"], p["weights"],
                             n_nodes=p["n_nodes"], return_all=True)
    a, b = p["root_edge"]
    P, S = st["partials"], st["scale"]
    for i, t in enumerate(p["t"]):
        got = oracle_mod.edge_derivs(P[a], S[a], P[b], S[b], ev, el, iv, t, p["rates"],
                                     p["weights"], m.freqs)
        ref = p["totals"][i]
        assert abs(got[0] - ref[0]) <= 1e-10 * abs(ref[0])
        for k in (1, 2):
            assert abs(got[k] - ref[k]) <= 1e-8 * max(abs(ref[k]), 1.0), (t, k, got, ref)


def test_oracle_cfg5_small_matches_reference(oracle_mod):
    seqs, trees, lnl, rates, weights = cfg5_small()
    m = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    ev, el, iv = m.engine_eigen()
    for nwk, ref in zip(trees, lnl):
        tr = Traversal(prepare_tree(parse_newick(nwk)))
        tips = {node: A.seq_to_partials(seqs[int(name[1:])], A.DNA)
                for name, node in tr.names.items()}
        got, _ = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                     tr.root_length(), ev, el, iv, m.freqs, rates, weights,
                                     n_nodes=tr.n_nodes)
        assert abs(got - ref) <= 1e-11 * abs(ref), (got, ref)
