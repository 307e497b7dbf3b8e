"""Pin the CPU oracle to the reference's own outputs (tests/golden, made by
tests/golden/make_golden.py from the reference's numpy engine, substitution
models and PAML C).  CPU only."""
import numpy as np
import pytest

from conftest import (band_tree, check_band_case, check_partials_repr, golden_charmap,
                      load_golden, tree_case)

TREE_CASES = ["cfg1_jc", "cfg2_small", "cfg3_small", "deep_scaling", "ambig_dna",
              "ambig_prot", "k80_g1", "long_branches"]


def test_golden_files_present():
    for f in ("clv", "clv_band", "gamma", "models", "charmaps", "pulley", "trees"):
        load_golden(f)


@pytest.mark.parametrize("impl", ["numpy", "c"])
def test_clv_matches_reference_engine(oracle_mod, impl):
    g = load_golden("clv")
    for k in g["cases"]:
        a = {n: g[str(k) + "_" + n] for n in ("p1", "p2", "clv1", "clv2", "sa", "sb", "out",
                                              "cml")}
        cml = np.zeros_like(a["sa"])
        if impl == "numpy":
            out = oracle_mod.clv(a["p1"], a["p2"], a["clv1"], a["clv2"], a["sa"], a["sb"], cml)
        else:
            out = oracle_mod.clv_c(a["p1"], a["p2"], a["clv1"], a["clv2"], a["sa"], a["sb"],
                                   cml)
        np.testing.assert_allclose(out, a["out"], rtol=1e-13, atol=0, err_msg=str(k))
        np.testing.assert_allclose(cml, a["cml"], rtol=1e-14, atol=1e-12, err_msg=str(k))


@pytest.mark.parametrize("impl", ["numpy", "c"])
def test_clv_band_between_thresholds(oracle_mod, impl):
    """Vectors whose largest entry is in [2^-128, eps): the reference's python engine
    rescales them, the live numba engine (and this oracle) does not.  Pinned on the
    python engine's output through representation-free quantities (conftest)."""
    g = load_golden("clv_band")
    fn = oracle_mod.clv if impl == "numpy" else oracle_mod.clv_c
    for k in g["cases"]:
        k = str(k)
        cml = np.zeros_like(g[k + "_sa"])
        with np.errstate(divide="ignore"):
            out = fn(g[k + "_p1"], g[k + "_p2"], g[k + "_clv1"], g[k + "_clv2"], g[k + "_sa"],
                     g[k + "_sb"], cml)
            sw = oracle_mod.lnl_node(g[k + "_pi"], out, cml)
            check_band_case(g, k, out, cml, sw)


# tol: the GPU / host model builds P from its own eigen-decomposition, which agrees with
# the reference's Model.p to rtol 1e-10 (test_host.py); on the 40-taxon LG tree with
# branches up to 1.2 that alone moves the normalised partials by 1.6e-11 (the oracle on the
# host model's eigen shows the same), on the GTR tree by 1.1e-13
@pytest.mark.parametrize("pre,min_band,tol", [("tree", 500, 1e-12), ("aatree", 150, 5e-11)])
def test_tree_partials_through_band(oracle_mod, pre, min_band, tol):
    """Long-branch trees (GTR+G4 120 taxa, LG+G4 40 taxa): every internal partial vector of
    the oracle's traversal (numba rule) against the reference driver's (python engine),
    representation-free; hundreds of them sit unscaled in [2^-128, eps)."""
    c = band_tree(pre)
    res = oracle_mod.tree_lnl(_tips(c), c["ops"], c["lens"], tuple(c["root_edge"]),
                              float(c["root_len"]), c["evecs"], c["evals"], c["ivecs"],
                              c["freqs"], c["rates"], c["weights"], n_nodes=int(c["n_nodes"]),
                              return_all=True)
    par = c["ops"][:, 0]
    n_band = check_partials_repr(res["partials"][par], res["scale"][par], c["partials"],
                                 c["scale"], tol)
    assert n_band > min_band, n_band
    np.testing.assert_allclose(res["site_lnl"], c["site_lnl"], rtol=1e-12, atol=1e-10)


def test_lnl_node_matches_reference_engine(oracle_mod):
    g = load_golden("clv")
    for k in g["cases"]:
        k = str(k)
        sw = oracle_mod.lnl_node(g[k + "_pi"], g[k + "_out"], g[k + "_cml"])
        np.testing.assert_allclose(sw, g[k + "_lnl_node"], rtol=1e-14, atol=1e-12)


def test_clv_rescale_rule(oracle_mod):
    """numba_likelihood_engine.py:39-44: rescale only when 0 < max < 2^-128; zero stays."""
    K, C, S = 4, 2, 3
    p = np.stack([np.eye(K)] * C)
    a = np.ones((S, C, K))
    b = np.ones((S, C, K))
    a[0] *= 2.0 ** -70
    b[0] *= 2.0 ** -70        # product 2^-140 -> rescaled
    a[1] *= 2.0 ** -60
    b[1] *= 2.0 ** -60        # product 2^-120 -> not rescaled
    a[2] = 0.0                # product 0 -> not rescaled (m > 0 fails)
    sa = np.full((S, C), -1.0)
    sb = np.full((S, C), -2.0)
    for fn in (oracle_mod.clv, oracle_mod.clv_c):
        cml = np.zeros((S, C))
        out = fn(p, p, a, b, sa, sb, cml)
        np.testing.assert_allclose(out[0], 1.0)
        np.testing.assert_allclose(cml[0], -3.0 + np.log(2.0 ** -140))
        np.testing.assert_allclose(out[1], 2.0 ** -120)
        np.testing.assert_allclose(cml[1], -3.0)
        assert np.all(out[2] == 0) and np.all(cml[2] == -3.0)


def test_reference_gamma_known_answer(oracle_mod):
    g = load_golden("gamma")
    np.testing.assert_allclose(g["kat_0_5_5"],
                               [0.02121238, 0.15548577, 0.46708288, 1.10711735, 3.24910162],
                               atol=5e-9)  # src/discrete_gamma.pyx:41-42


def test_pulley_principle_golden():
    g = load_golden("pulley")
    assert abs(float(g["lnl_cherry"]) - float(g["lnl_edge"])) < 1e-14
    assert abs(float(g["lnl_cherry"]) + 4.122814335054628) < 1e-12


def _tips(case):
    alpha = "ACGT" if case["evecs"].shape[0] == 4 else "ARNDCQEGHILKMFPSTWYV"
    cm = golden_charmap("dna" if len(alpha) == 4 else "protein")
    tips = {}
    for idx, s in zip(case["tip_index"], case["seq_strings"]):
        tips[int(idx)] = np.array([cm[ch] for ch in s])
    return tips


@pytest.mark.parametrize("name", TREE_CASES)
def test_tree_lnl_matches_reference(oracle_mod, name):
    c = tree_case(name)
    lnl, site = oracle_mod.tree_lnl(_tips(c), c["ops"], c["lens"], tuple(c["root_edge"]),
                                    float(c["root_len"]), c["evecs"], c["evals"], c["ivecs"],
                                    c["freqs"], c["rates"], c["weights"],
                                    n_nodes=int(c["n_nodes"]))
    np.testing.assert_allclose(site, c["site_lnl"], rtol=1e-12, atol=1e-10)
    assert abs(lnl - float(c["lnl"])) <= 1e-11 * abs(float(c["lnl"]))


def test_deep_tree_exercises_rescaling(oracle_mod):
    c = tree_case("long_branches")
    res = oracle_mod.tree_lnl(_tips(c), c["ops"], c["lens"], tuple(c["root_edge"]),
                              float(c["root_len"]), c["evecs"], c["evals"], c["ivecs"],
                              c["freqs"], c["rates"], c["weights"], n_nodes=int(c["n_nodes"]),
                              return_all=True)
    assert np.count_nonzero(res["scale"]) > 0  # the 2^-128 branch is exercised


def test_oracle_threads_agree(oracle_mod):
    c = tree_case("cfg2_small")
    args = (_tips(c), c["ops"], c["lens"], tuple(c["root_edge"]), float(c["root_len"]),
            c["evecs"], c["evals"], c["ivecs"], c["freqs"], c["rates"], c["weights"])
    l1, s1 = oracle_mod.tree_lnl(*args, nthreads=1)
    l4, s4 = oracle_mod.tree_lnl(*args, nthreads=4)
    np.testing.assert_array_equal(s1, s4)
    assert abs(l1 - l4) < 1e-9 * abs(l1)
