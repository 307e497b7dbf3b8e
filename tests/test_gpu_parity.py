"""GPU parity: the HIP path (through the C ABI) against the reference's golden vectors
and the CPU oracle.  Tolerances (fp64): partial vectors 1e-12 relative to each vector's largest entry, sitewise lnL
absolute 1e-9, total lnL relative 1e-9 (the north-star bound) -- observed errors
are ~1e-14."""
import ctypes
import os

import numpy as np
import pytest

from conftest import band_tree, check_band_case, check_partials_repr, load_golden, tree_case

from phylo_utils_amd import TreeModel
from phylo_utils_amd import _native as N
from phylo_utils_amd import alignment as A
from phylo_utils_amd import substitution_models as SM
from phylo_utils_amd.likelihood import hip_likelihood_engine as E
from phylo_utils_amd.rate_models import GammaRateModel, InvariantSitesModel, UniformRateModel
from phylo_utils_amd.synthetic import CFG2_FREQS, CFG2_GTR_RATES, make_problem
from phylo_utils_amd.tree import Traversal, prepare_tree

pytestmark = pytest.mark.gpu

LNL_RTOL = 1e-9

CASE_MODELS = {
    "cfg1_jc": (lambda: SM.GTR(), A.DNA),
    "cfg2_small": (lambda: SM.GTR(CFG2_GTR_RATES, CFG2_FREQS), A.DNA),
    "cfg3_small": (lambda: SM.LG(), A.PROTEIN),
    "deep_scaling": (lambda: SM.GTR(CFG2_GTR_RATES, CFG2_FREQS), A.DNA),
    "ambig_dna": (lambda: SM.HKY85(2.0, [0.1, 0.2, 0.3, 0.4]), A.DNA),
    "ambig_prot": (lambda: SM.WAG(), A.PROTEIN),
    "k80_g1": (lambda: SM.K80(2.0), A.DNA),
    "long_branches": (lambda: SM.GTR(CFG2_GTR_RATES, CFG2_FREQS), A.DNA),
}


def assert_partials_close(got, ref, rtol=1e-12):
    """Per K-vector relative error: |got - ref| <= rtol * max_i |ref_i| for every
    (node, site, category) vector (small components of a partial vector carry the
    rounding of its large ones, so an elementwise rtol is the wrong yardstick)."""
    scale = np.abs(ref).max(axis=-1, keepdims=True)
    err = np.abs(got - ref)
    bad = err > rtol * scale
    assert not bad.any(), "max vector-relative error %.3e at %d entries" % (
        (err / np.where(scale > 0, scale, 1)).max(), bad.sum())


class _Rates:
    def __init__(self, rates, weights):
        self.rates = np.asarray(rates)
        self.weights = np.asarray(weights)
        self.ncat = len(self.rates)


def build_model(name, compress=False, **kw):
    c = tree_case(name)
    mk, alpha = CASE_MODELS[name]
    tm = TreeModel(**kw)
    tm.set_alignment([("t%d" % i, s) for i, s in enumerate(c["seq_strings"])], alpha,
                     compress=compress)
    tm.set_substitution_model(mk())
    tm.set_rate_model(_Rates(c["rates"], c["weights"]))
    tm.set_tree(c["newick"])
    tm.initialise()
    return tm, c


# ---------------------------------------------------------------- engine seam (per op)
def test_clv_matches_golden():
    g = load_golden("clv")
    for k in g["cases"]:
        k = str(k)
        cml = np.zeros_like(g[k + "_sa"])
        out = E.clv(g[k + "_p1"], g[k + "_p2"], g[k + "_clv1"], g[k + "_clv2"], g[k + "_sa"],
                    g[k + "_sb"], cml)
        np.testing.assert_allclose(out, g[k + "_out"], rtol=1e-13, err_msg=k)
        np.testing.assert_allclose(cml, g[k + "_cml"], rtol=1e-14, atol=1e-12, err_msg=k)
        sw = E.lnl_node(g[k + "_pi"], out, cml)
        np.testing.assert_allclose(sw, g[k + "_lnl_node"], rtol=1e-14, atol=1e-12)


def test_clv_band_between_thresholds():
    """The drop-in clv / lnl_node on vectors in [2^-128, eps) (numba: no rescale; the
    reference's python engine: rescaled) -- tests/golden/clv_band.npz via conftest."""
    g = load_golden("clv_band")
    for k in g["cases"]:
        k = str(k)
        cml = np.zeros_like(g[k + "_sa"])
        out = E.clv(g[k + "_p1"], g[k + "_p2"], g[k + "_clv1"], g[k + "_clv2"], g[k + "_sa"],
                    g[k + "_sb"], cml)
        sw = E.lnl_node(g[k + "_pi"], out, cml)
        with np.errstate(divide="ignore"):
            check_band_case(g, k, out, cml, sw)


@pytest.mark.parametrize("K,C", [(2, 1), (3, 2), (4, 3), (20, 5), (61, 2), (20, 40)])
def test_clv_shapes_vs_oracle(oracle_mod, K, C):
    rng = np.random.default_rng(K * 100 + C)
    S = 1000
    p1 = rng.dirichlet(np.ones(K), (C, K))
    p2 = rng.dirichlet(np.ones(K), (C, K))
    a = rng.random((S, C, K))
    b = rng.random((S, C, K))
    a[::7] *= 1e-30
    b[::7] *= 1e-20
    sa = rng.normal(size=(S, C))
    sb = rng.normal(size=(S, C))
    cml = np.zeros((S, C))
    ref_cml = np.zeros((S, C))
    out = E.clv(p1, p2, a, b, sa, sb, cml)
    ref = oracle_mod.clv(p1, p2, a, b, sa, sb, ref_cml)
    np.testing.assert_allclose(out, ref, rtol=1e-12)
    np.testing.assert_allclose(cml, ref_cml, rtol=1e-13, atol=1e-12)


def test_clv_out_argument_and_rescale_rule(oracle_mod):
    K, C, S = 4, 2, 3
    p = np.stack([np.eye(K)] * C)
    a = np.ones((S, C, K))
    b = np.ones((S, C, K))
    a[0] *= 2.0 ** -70
    b[0] *= 2.0 ** -70
    a[1] *= 2.0 ** -60
    b[1] *= 2.0 ** -60
    a[2] = 0.0
    sa = np.full((S, C), -1.0)
    sb = np.full((S, C), -2.0)
    cml = np.zeros((S, C))
    out = np.empty((S, C, K))
    r = E.clv(p, p, a, b, sa, sb, cml, out)
    assert r is out
    np.testing.assert_allclose(out[0], 1.0)
    np.testing.assert_allclose(cml[0], -3.0 + np.log(2.0 ** -140))
    np.testing.assert_allclose(out[1], 2.0 ** -120)
    assert np.all(cml[1] == -3.0) and np.all(out[2] == 0) and np.all(cml[2] == -3.0)
    sw = E.lnl_node(np.full(K, 0.25), out, cml)
    assert np.all(np.isneginf(sw[2]))


# ---------------------------------------------------------------- whole traversal
@pytest.mark.parametrize("name", sorted(CASE_MODELS))
def test_tree_lnl_matches_reference_golden(name):
    tm, c = build_model(name)
    site = tm.compute_likelihood_at_edge(*tm.traversal.root_edge)
    np.testing.assert_allclose(site, c["site_lnl"], rtol=1e-12, atol=1e-9)
    lnl = float(c["lnl"])
    assert abs(tm.likelihood() - lnl) <= LNL_RTOL * abs(lnl)
    assert abs(tm.likelihood() - lnl) <= 1e-12 * abs(lnl) * len(site)


@pytest.mark.parametrize("compact,keep,reorder", [(True, True, True), (False, True, True),
                                                  (True, False, True), (False, False, False),
                                                  (True, True, False)])
@pytest.mark.parametrize("name", ["cfg2_small", "cfg3_small", "long_branches", "ambig_prot",
                                  "ambig_dna"])
def test_engine_modes_agree(name, compact, keep, reorder):
    """dense vs coded tips, kept vs reused buffers, caller vs register-aware order:
    identical arithmetic per node => bitwise-equal sitewise lnL.  (ambig_dna, coded and
    lnL-only: the tip products PT over all 16 ambiguity codes, r06's per-row P kernel.)"""
    base, _ = build_model(name)
    tm, _ = build_model(name, compact_tips=compact, keep_partials=keep, reorder=reorder)
    np.testing.assert_array_equal(tm.sitewise_patterns(), base.sitewise_patterns())


@pytest.mark.parametrize("env", [{"PU_LDS_SLOTS": "0"}, {"PU_LDS_SLOTS": "1"},
                                 {"PU_FORCE_GENERIC": "1"}, {"PU_KEEP_OCC": "6"},
                                 {"PU_KEEP_OCC": "7"}, {"PU_CHUNK_USES": "3"},
                                 {"PU_SPLIT": "1"}, {"PU_SPLIT": "2"}, {"PU_SPLIT": "8"},
                                 {"PU_SPLIT": "4", "PU_LDS_SLOTS": "1", "PU_CHUNK_USES": "3"}])
@pytest.mark.parametrize("name", ["deep_scaling", "cfg3_small", "ambig_dna", "ambig_prot"])
def test_kernel_builds_and_plans_bitwise_equal(monkeypatch, name, env):
    """Every k_prune build / plan computes each node with identical arithmetic: HBM
    read-backs instead of the LDS stash (PU_LDS_SLOTS=0/1: PAT_MC), the general variant,
    6 workgroups per CU, the 7-wave build, tiny staging chunks, plans split into chain tasks + a top task
    (PU_SPLIT) -- bitwise-equal partials, scalers and lnL."""
    base, _ = build_model(name)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    tm, _ = build_model(name)
    np.testing.assert_array_equal(tm.sitewise_patterns(), base.sitewise_patterns())
    np.testing.assert_array_equal(tm.partials, base.partials)
    np.testing.assert_array_equal(tm.scale, base.scale)


def _height_order(ops):
    """A valid post-order that is not a DFS order: ops sorted by subtree height, so the
    children of an op are seldom the previous op's parent (PAT_MT / PAT_MM children)."""
    prod = {int(p): (int(a), int(b)) for p, a, b in ops}
    h = {}

    def height(v):
        stack = [v]
        while stack:
            x = stack[-1]
            if x not in prod:
                h[x] = 0
                stack.pop()
                continue
            a, b = prod[x]
            if a in h and b in h:
                h[x] = 1 + max(h[a], h[b])
                stack.pop()
            else:
                stack += [c for c in (a, b) if c not in h]
        return h[v]
    return np.array(sorted(ops.tolist(), key=lambda r: (height(r[0]), r[0])), dtype=np.int32)


@pytest.mark.parametrize("keep", [True, False])
def test_non_dfs_caller_order(oracle_mod, keep):
    base, c = build_model("cfg2_small", keep_partials=keep)
    tm = TreeModel(keep_partials=keep, reorder=False)
    tm.set_alignment([("t%d" % i, s) for i, s in enumerate(c["seq_strings"])], A.DNA,
                     compress=False)
    tm.set_substitution_model(SM.GTR(CFG2_GTR_RATES, CFG2_FREQS))
    tm.set_rate_model(_Rates(c["rates"], c["weights"]))
    tm.set_tree(c["newick"])
    tr = tm.traversal
    order = _height_order(tr.postorder_traversal)
    assert not np.array_equal(order, tr.postorder_traversal)
    tr.postorder_traversal = order
    tm.initialise()
    st = N.plan_stats(tr.n_nodes, order, tr.root_edge, 0, 2, N.PU_NO_REORDER)
    assert st["mem"] > 0  # HBM read-backs: the general kernel variant ran
    np.testing.assert_allclose(tm.sitewise_patterns(), base.sitewise_patterns(), rtol=1e-13)
    if keep:
        assert_partials_close(tm.partials, base.partials, rtol=1e-13)


def test_compressed_patterns_same_total():
    a, c = build_model("cfg2_small", compress=False)
    b, _ = build_model("cfg2_small", compress=True)
    assert b.alignment.shape[1] < a.alignment.shape[1]
    np.testing.assert_allclose(b.compute_likelihood_at_edge(*b.traversal.root_edge),
                               c["site_lnl"], rtol=1e-12, atol=1e-9)
    assert abs(a.likelihood() - b.likelihood()) <= 1e-11 * abs(a.likelihood())


# tol: the GPU / host model builds P from its own eigen-decomposition, which agrees with
# the reference's Model.p to rtol 1e-10 (test_host.py); on the 40-taxon LG tree with
# branches up to 1.2 that alone moves the normalised partials by 1.6e-11 (the oracle on the
# host model's eigen shows the same), on the GTR tree by 1.1e-13
@pytest.mark.parametrize("pre,min_band,tol", [("tree", 500, 1e-12), ("aatree", 150, 5e-11)])
def test_tree_partials_through_band(pre, min_band, tol):
    """k_prune (GTR+G4, 120 taxa) and k_prune_mfma (LG+G4, 40 taxa) on long-branch trees:
    every internal partial vector against the reference driver's (python engine,
    clv_band.npz), matched by clade and compared free of the rescaling representation;
    hundreds sit unscaled in [2^-128, eps) on the numba rule."""
    c = band_tree(pre)
    dna = pre == "tree"
    tm = TreeModel()
    tm.set_alignment([("t%d" % i, s) for i, s in enumerate(c["seq_strings"])],
                     A.DNA if dna else A.PROTEIN, compress=False)
    tm.set_substitution_model(SM.GTR(CFG2_GTR_RATES, CFG2_FREQS) if dna else SM.LG())
    tm.set_rate_model(_Rates(c["rates"], c["weights"]))
    tm.set_tree(c["newick"])
    tm.initialise()
    tr = tm.traversal
    clade = {idx: {nm} for nm, idx in tr.names.items()}
    for par, c1, c2 in tr.postorder_traversal:
        clade[int(par)] = clade[int(c1)] | clade[int(c2)]
    by_key = {",".join(sorted(v, key=lambda s: int(s[1:]))): k for k, v in clade.items()}
    rows = [(i, by_key[str(k)]) for i, k in enumerate(c["clades"]) if str(k) in by_key]
    assert len(rows) >= 0.9 * len(c["clades"])
    ref_i, ours = (np.array(x) for x in zip(*rows))
    parts, scale = tm.partials, tm.scale
    n_band = check_partials_repr(parts[ours], scale[ours], c["partials"][ref_i],
                                 c["scale"][ref_i], tol)
    assert n_band > min_band, n_band
    assert abs(tm.likelihood() - float(c["lnl"])) <= 1e-11 * abs(float(c["lnl"]))


@pytest.mark.parametrize("name", ["deep_scaling", "cfg3_small", "ambig_dna"])
def test_all_partials_and_root_vs_oracle(oracle_mod, name):
    tm, c = build_model(name)
    tr = tm.traversal
    K = tm.alignment.shape[2]
    tips = {tr.names[n]: tm.alignment[i] for n, i in tm.names.items()}
    ev, el, iv = tm.substitution_model.engine_eigen()
    ref = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                              tr.root_length(), ev, el, iv, tm.substitution_model.freqs,
                              c["rates"], c["weights"], n_nodes=tr.n_nodes, return_all=True)
    parts, scale = tm.partials, tm.scale
    assert parts.shape == (tr.n_nodes, tm.alignment.shape[1], len(c["rates"]), K)
    assert_partials_close(parts, ref["partials"])
    np.testing.assert_allclose(scale, ref["scale"], rtol=1e-13, atol=1e-10)
    rp, rs = tm.compute_partials_at_edge(*tr.root_edge)
    assert_partials_close(rp, ref["root_partials"])
    np.testing.assert_allclose(rs, ref["root_scale"], rtol=1e-13, atol=1e-10)
    if name == "deep_scaling":
        assert np.count_nonzero(scale) > 0
    # device P matrices vs Model.p restated on the CPU
    P = np.empty((len(tr.postorder_traversal) + 1, 2, len(c["rates"]), K, K))
    N.check(N.lib().pu_get_pmatrices(tm._ctx, N.ptr(P)))
    np.testing.assert_allclose(P[:-1], ref["P"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(P[-1], ref["Proot"], rtol=1e-12, atol=1e-15)


def test_pulley_principle_on_device():
    """tests/test_likelihood.py:35-49 on the live semantics: the a-b path is 0.3 in every
    rooting; c is a gap (all ones) and contributes a factor 1."""
    g = load_golden("pulley")
    tm = TreeModel()
    tm.set_alignment([("a", "A"), ("b", "C"), ("c", "-")], A.DNA)
    tm.set_substitution_model(SM.K80(2.0))
    tm.set_rate_model(UniformRateModel())
    lnls = []
    for nwk in ("((a:0.1,b:0.2):0.0,c:0.5);", "(a:0.05,(b:0.25,c:0.5):0.0);",
                "(b:0.2,(a:0.1,c:0.5):0.0);"):
        tm.set_tree(nwk)
        tm.initialise()
        lnls.append(tm.likelihood())
    np.testing.assert_allclose(lnls, float(g["lnl_cherry"]), rtol=1e-13)


def test_two_and_three_taxa_and_single_site(oracle_mod):
    for nwk, seqs in (("(a:0.3,b:0.2);", [("a", "ACGTA"), ("b", "ACGTT")]),
                      ("(a:0.3,b:0.2,c:0.1);", [("a", "A"), ("b", "C"), ("c", "G")])):
        tm = TreeModel()
        tm.set_alignment(seqs, A.DNA, compress=False)
        tm.set_substitution_model(SM.HKY85(2.0, [0.1, 0.2, 0.3, 0.4]))
        tm.set_rate_model(GammaRateModel(3, 0.7))
        tm.set_tree(nwk)
        tm.initialise()
        tr = tm.traversal
        tips = {tr.names[n]: tm.alignment[i] for n, i in tm.names.items()}
        ev, el, iv = tm.substitution_model.engine_eigen()
        lnl, site = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(),
                                        tr.root_edge, tr.root_length(), ev, el, iv,
                                        tm.substitution_model.freqs, tm.rate_model.rates,
                                        tm.rate_model.weights, n_nodes=tr.n_nodes)
        np.testing.assert_allclose(tm.sitewise_patterns(), site, rtol=1e-13)


@pytest.mark.parametrize("ncat", [1, 2, 3, 5, 6, 8, 16])
def test_category_counts(oracle_mod, ncat):
    model = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    rm = GammaRateModel(ncat, 0.4) if ncat > 1 else UniformRateModel()
    tree, names, states = make_problem(30, 777, model, rm.rates, seed=ncat)
    tm = TreeModel()
    tm.set_alignment_partials(np.eye(4)[states], names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    tr = tm.traversal
    tips = {tr.names[n]: tm.alignment[i] for n, i in tm.names.items()}
    ev, el, iv = model.engine_eigen()
    lnl, site = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                    tr.root_length(), ev, el, iv, model.freqs, rm.rates,
                                    rm.weights, n_nodes=tr.n_nodes)
    np.testing.assert_allclose(tm.sitewise_patterns(), site, rtol=1e-12)
    assert abs(tm.likelihood() - lnl) <= 1e-12 * abs(lnl)


def test_invariant_category_and_impossible_site(oracle_mod):
    model = SM.HKY85(3.0, [0.1, 0.2, 0.3, 0.4])
    tm = TreeModel(compact_tips=False)
    parts = np.eye(4)[np.array([[0, 1, 2, 3, 0], [0, 1, 2, 3, 1], [0, 2, 2, 3, 2]])]
    parts[0, 4] = 0.0  # no state possible: lnl_node gives -inf (numba :87)
    tm.set_alignment_partials(parts, ["a", "b", "c"])
    tm.set_substitution_model(model)
    tm.set_rate_model(InvariantSitesModel(0.3))
    tm.set_tree("((a:0.1,b:0.2):0.05,c:0.3);")
    tm.initialise()
    site = tm.sitewise_patterns()
    assert np.isneginf(site[4]) and np.all(np.isfinite(site[:4]))
    assert np.isneginf(tm.likelihood())


def test_branch_length_update_and_determinism(oracle_mod):
    tm, c = build_model("cfg2_small")
    l0 = tm.likelihood()
    tm.compute_partials()
    assert tm.likelihood() == l0  # fixed-order reduction: bitwise repeatable
    for k in list(tm.traversal.brlens):
        tm.traversal.brlens[k] *= 1.5
    tm.update_branch_lengths()
    tr = tm.traversal
    tips = {tr.names[n]: tm.alignment[i] for n, i in tm.names.items()}
    ev, el, iv = tm.substitution_model.engine_eigen()
    lnl, _ = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                 tr.root_length(), ev, el, iv, tm.substitution_model.freqs,
                                 c["rates"], c["weights"], n_nodes=tr.n_nodes)
    assert abs(tm.likelihood() - lnl) <= 1e-12 * abs(lnl)
    assert tm.likelihood() != l0


@pytest.mark.parametrize("name", ["cfg2_small", "deep_scaling", "ambig_dna"])
def test_fused_lnl_sum_equals_k_reduce(monkeypatch, name):
    """r06, opt-in (PU_RED_FUSED=1): DNA launches add the block sums in the traversal's last
    workgroup (flag-in-word slots, TraverseArgs::red_slots) instead of a k_reduce launch: the
    same lnL bit for bit,
    launch after launch (each launch's generation), and after the lengths change."""
    tm, _ = build_model(name)
    monkeypatch.setenv("PU_RED_FUSED", "1")
    fused = []
    for _ in range(5):
        tm.compute_partials()
        fused.append(tm.likelihood())
    monkeypatch.delenv("PU_RED_FUSED")
    tm.compute_partials()
    ref = tm.likelihood()
    assert all(f == ref for f in fused), (fused, ref)
    for k in list(tm.traversal.brlens):
        tm.traversal.brlens[k] *= 1.25
    tm.update_branch_lengths()
    ref2 = tm.likelihood()
    monkeypatch.setenv("PU_RED_FUSED", "1")
    tm.compute_partials()
    assert tm.likelihood() == ref2 != ref


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_baseline_config_full_size_vs_oracle(oracle_mod, cfg):
    """BASELINE configs 2 and 3 at full size against the oracle (OpenMP C)."""
    if cfg == "cfg2":
        model, ntax, S, alpha = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS), 50, 100_000, 0.5
    else:
        model, ntax, S, alpha = SM.LG(), 200, 10_000, 0.8
    rm = GammaRateModel(4, alpha)
    tree, names, states = make_problem(ntax, S, model, rm.rates, seed=7)
    K = len(model.freqs)
    tm = TreeModel()
    tm.set_alignment_partials(np.eye(K)[states], names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    tr = tm.traversal
    tips = {tr.names[n]: tm.alignment[i] for n, i in tm.names.items()}
    ev, el, iv = model.engine_eigen()
    lnl, site = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                    tr.root_length(), ev, el, iv, model.freqs, rm.rates,
                                    rm.weights, n_nodes=tr.n_nodes, nthreads=8)
    np.testing.assert_allclose(tm.sitewise_patterns(), site, rtol=1e-12, atol=1e-10)
    assert abs(tm.likelihood() - lnl) <= LNL_RTOL * abs(lnl)


@pytest.mark.parametrize("seed", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg5"])
def test_baseline_configs_seeds_0_to_4_vs_oracle(oracle_mod, cfg, seed):
    """seeds 0-4 of each single-GPU config's generator (topology, lengths
    U(0.01, 0.3), alignment simulated under the model) at reduced site counts, lnL and sitewise
    against the oracle (cfg2: 50 taxa x 5k sites; cfg3: 200 taxa x 1k AA sites; cfg5: 100 taxa
    x 2k sites, lnL-only)."""
    if cfg == "cfg3":
        model, ntax, S, alpha = SM.LG(), 200, 1_000, 0.8
    else:
        model = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
        ntax, S, alpha = (50, 5_000, 0.5) if cfg == "cfg2" else (100, 2_000, 0.5)
    rm = GammaRateModel(4, alpha)
    tree, names, states = make_problem(ntax, S, model, rm.rates, seed=seed)
    K = len(model.freqs)
    tm = TreeModel(keep_partials=cfg != "cfg5")
    tm.set_alignment_partials(np.eye(K)[states], names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    tr = tm.traversal
    tips = {tr.names[n]: tm.alignment[i] for n, i in tm.names.items()}
    ev, el, iv = model.engine_eigen()
    lnl, site = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                    tr.root_length(), ev, el, iv, model.freqs, rm.rates,
                                    rm.weights, n_nodes=tr.n_nodes, nthreads=8)
    np.testing.assert_allclose(tm.sitewise_patterns(), site, rtol=1e-12, atol=1e-10)
    assert abs(tm.likelihood() - lnl) <= LNL_RTOL * abs(lnl)


@pytest.mark.parametrize("env", [{}, {"PU_FORCE_GENERIC": "1"}, {"PU_LDS_SLOTS": "1"},
                                 {"PU_SPLIT": "3"}])
@pytest.mark.parametrize("keep", [True, False])
def test_protein_rescaling_vs_oracle(monkeypatch, oracle_mod, keep, env):
    """K = 20 (k_prune_mfma) on a deep tree with long branches: many sites rescale, so the
    cross-lane-group max and the rescale decision are exercised; every partial and scaler
    against the oracle, in the counted-wait modes and the wait-for-zero mode, with HBM
    read-backs (one stash slot)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    model = SM.LG()
    rm = GammaRateModel(4, 0.8)
    tree, names, states = make_problem(200, 150, model, rm.rates, seed=5, lo=0.4, hi=1.5)
    tm = TreeModel(keep_partials=keep)
    tm.set_alignment_codes(states.astype(np.uint8), np.eye(20), names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    tr = tm.traversal
    tips = {tr.names[n]: np.eye(20)[states[i]] for i, n in enumerate(names)}
    ev, el, iv = model.engine_eigen()
    ref = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                              tr.root_length(), ev, el, iv, model.freqs, rm.rates,
                              rm.weights, n_nodes=tr.n_nodes, return_all=True)
    assert np.count_nonzero(ref["scale"]) > 1000
    np.testing.assert_allclose(tm.sitewise_patterns(), ref["site_lnl"], rtol=1e-12)
    rp, rs = tm.compute_partials_at_edge(*tr.root_edge)
    assert_partials_close(rp, ref["root_partials"])
    np.testing.assert_allclose(rs, ref["root_scale"], rtol=1e-13, atol=1e-10)
    if keep:
        assert_partials_close(tm.partials, ref["partials"])
        np.testing.assert_allclose(tm.scale, ref["scale"], rtol=1e-13, atol=1e-10)


@pytest.mark.parametrize("keep", [True, False])
def test_scalers_stay_exact_across_runs(oracle_mod, keep):
    """Scaler tiles that were non-zero in one run and are zero in the next must be rewritten
    (the skip-zero-scaler protocol, TV_SKIP_ZERO_SCALE), and vice versa."""
    model = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    rm = GammaRateModel(4, 0.5)
    tree, names, states = make_problem(150, 300, model, rm.rates, seed=11, lo=0.4, hi=1.5)
    tm = TreeModel(keep_partials=keep)
    tm.set_alignment_codes(states.astype(np.uint8), np.eye(4), names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    tr = tm.traversal
    tips = {tr.names[n]: np.eye(4)[states[i]] for i, n in enumerate(names)}
    ev, el, iv = model.engine_eigen()
    orig = dict(tr.brlens)
    for factor in (1.0, 0.01, 1.0, 0.3):
        for k in orig:
            tr.brlens[k] = orig[k] * factor
        tm.update_branch_lengths()
        ref = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                  tr.root_length(), ev, el, iv, model.freqs, rm.rates,
                                  rm.weights, n_nodes=tr.n_nodes, return_all=True)
        np.testing.assert_allclose(tm.sitewise_patterns(), ref["site_lnl"], rtol=1e-12)
        rp, rs = tm.compute_partials_at_edge(*tr.root_edge)
        np.testing.assert_allclose(rs, ref["root_scale"], rtol=1e-13, atol=1e-10)
        if keep:
            np.testing.assert_allclose(tm.scale, ref["scale"], rtol=1e-13, atol=1e-10)
            if factor == 1.0:
                assert np.count_nonzero(ref["scale"]) > 0


# ---------------------------------------------------------------- C ABI
def _c_abi_problem():
    model = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    rm = GammaRateModel(4, 0.5)
    tree, names, states = make_problem(20, 1001, model, rm.rates, seed=21)
    tr = Traversal(prepare_tree(tree))
    nodes = np.array([tr.names[n] for n in names], dtype=np.int32)
    weights = np.arange(1, 1002, dtype=np.float64) % 3 + 1.0
    return model, rm, tr, nodes, np.ascontiguousarray(states.astype(np.uint8)), weights


def test_c_abi_set_tips_and_sitewise_run(oracle_mod):
    """pu_set_tips (codes and dense partials) + pu_run's sitewise output vs the oracle."""
    model, rm, tr, nodes, codes, w = _c_abi_problem()
    ev, el, iv = model.engine_eigen()
    ops = np.ascontiguousarray(tr.postorder_traversal, dtype=np.int32)
    bl = N.f64(tr.op_lengths())
    a, b = tr.root_edge
    tips = {int(nd): np.eye(4)[codes[i]] for i, nd in enumerate(nodes)}
    ref_lnl, ref_site = oracle_mod.tree_lnl(tips, ops, tr.op_lengths(), tr.root_edge,
                                            tr.root_length(), ev, el, iv, model.freqs,
                                            rm.rates, rm.weights, n_nodes=tr.n_nodes)
    for dense in (False, True):
        ctx = ctypes.c_void_p()
        N.check(N.lib().pu_ctx_create(ctypes.byref(ctx), 0, tr.n_nodes, len(nodes), 1001, 4,
                                      4, 0))
        try:
            part = np.ascontiguousarray(np.eye(4)[codes]) if dense else None
            N.check(N.lib().pu_set_tips(ctx, len(nodes), N.ptr(nodes), 4, N.ptr(np.eye(4)),
                                        None if dense else N.ptr(codes),
                                        N.ptr(part) if dense else None, N.ptr(w)), ctx)
            N.check(N.lib().pu_set_model(ctx, N.ptr(ev), N.ptr(el), N.ptr(iv),
                                         N.ptr(N.f64(model.freqs)), N.ptr(N.f64(rm.rates)),
                                         N.ptr(N.f64(rm.weights))), ctx)
            N.check(N.lib().pu_set_schedule(ctx, len(ops), N.ptr(ops), N.ptr(bl), a, b,
                                            tr.root_length()), ctx)
            lnl, site = ctypes.c_double(), np.zeros(1001)
            N.check(N.lib().pu_run(ctx, ctypes.byref(lnl), N.ptr(site)), ctx)
        finally:
            N.lib().pu_ctx_destroy(ctx)
        np.testing.assert_allclose(site, ref_site, rtol=1e-12)
        ref = float(np.dot(w, ref_site))
        assert abs(lnl.value - ref) <= LNL_RTOL * abs(ref)


def test_c_abi_group_one_device_matches_context():
    """pu_group_* on one device (the box has one GPU): the RCCL all-reduce path and the
    shard bookkeeping give exactly the single context's lnL and sitewise lnL."""
    model, rm, tr, nodes, codes, w = _c_abi_problem()
    ev, el, iv = model.engine_eigen()
    ops = np.ascontiguousarray(tr.postorder_traversal, dtype=np.int32)
    bl = N.f64(tr.op_lengths())
    a, b = tr.root_edge
    args = (N.ptr(ev), N.ptr(el), N.ptr(iv), N.ptr(N.f64(model.freqs)),
            N.ptr(N.f64(rm.rates)), N.ptr(N.f64(rm.weights)))
    ctx = ctypes.c_void_p()
    N.check(N.lib().pu_ctx_create(ctypes.byref(ctx), 0, tr.n_nodes, len(nodes), 1001, 4, 4, 0))
    try:
        N.check(N.lib().pu_set_tips(ctx, len(nodes), N.ptr(nodes), 4, N.ptr(np.eye(4)),
                                    N.ptr(codes), None, N.ptr(w)), ctx)
        N.check(N.lib().pu_set_model(ctx, *args), ctx)
        N.check(N.lib().pu_set_schedule(ctx, len(ops), N.ptr(ops), N.ptr(bl), a, b,
                                        tr.root_length()), ctx)
        lnl1, site1 = ctypes.c_double(), np.zeros(1001)
        N.check(N.lib().pu_run(ctx, ctypes.byref(lnl1), N.ptr(site1)), ctx)
    finally:
        N.lib().pu_ctx_destroy(ctx)
    g = ctypes.c_void_p()
    dev = np.zeros(1, dtype=np.int32)
    rc = N.lib().pu_group_create(ctypes.byref(g), 1, N.ptr(dev), tr.n_nodes, len(nodes), 1001,
                                 4, 4, 0)
    try:
        assert rc == 0, N.lib().pu_group_last_error(g)
        assert N.lib().pu_group_size(g) == 1
        first, count = ctypes.c_int64(), ctypes.c_int64()
        assert N.lib().pu_group_shard(g, 0, ctypes.byref(first), ctypes.byref(count)) == 0
        assert (first.value, count.value) == (0, 1001)
        for rc in (N.lib().pu_group_set_tips(g, len(nodes), N.ptr(nodes), 4, N.ptr(np.eye(4)),
                                             N.ptr(codes), None, N.ptr(w)),
                   N.lib().pu_group_set_model(g, *args),
                   N.lib().pu_group_set_schedule(g, len(ops), N.ptr(ops), N.ptr(bl), a, b,
                                                 tr.root_length())):
            assert rc == 0, N.lib().pu_group_last_error(g)
        lnl2, site2 = ctypes.c_double(), np.zeros(1001)
        assert N.lib().pu_group_run(g, ctypes.byref(lnl2), N.ptr(site2)) == 0, \
            N.lib().pu_group_last_error(g)
    finally:
        N.lib().pu_group_destroy(g)
    np.testing.assert_array_equal(site2, site1)
    assert lnl2.value == lnl1.value


def test_new_topology_reuses_resident_tips():
    """TreeModel.set_tree + initialise on the same taxa keeps the device context: the tips
    are re-bound to the new node numbering (pu_set_tip_nodes), nothing is uploaded again,
    and every number equals a fresh TreeModel's on that tree."""
    from phylo_utils_amd.synthetic import random_tree
    model = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    rm = GammaRateModel(4, 0.5)
    tree_a, names, states = make_problem(30, 517, model, rm.rates, seed=31)
    tree_b = random_tree(np.random.default_rng(32), 30)

    def fresh(tree):
        t = TreeModel()
        t.set_alignment_codes(states.astype(np.uint8), np.eye(4), names)
        t.set_substitution_model(model)
        t.set_rate_model(rm)
        t.set_tree(tree)
        t.initialise()
        return t

    tm = fresh(tree_a)
    lnl_a, parts_a = tm.likelihood(), tm.partials
    ctx = tm._ctx.value
    for tree, ref in ((tree_b, fresh(tree_b)), (tree_a, None)):
        tm.set_tree(tree)
        tm.initialise()
        assert tm._ctx.value == ctx  # reused, tips resident
        if ref is None:
            assert tm.likelihood() == lnl_a
            np.testing.assert_array_equal(tm.partials, parts_a)
        else:
            assert tm.likelihood() == ref.likelihood()
            np.testing.assert_array_equal(tm.sitewise_patterns(), ref.sitewise_patterns())
            np.testing.assert_array_equal(tm.partials, ref.partials)
            np.testing.assert_array_equal(tm.scale, ref.scale)


def _gtr_problem(ntax, S, seed):
    model = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    rm = GammaRateModel(4, 0.5)
    tree, names, states = make_problem(ntax, S, model, rm.rates, seed=seed)
    return model, rm, tree, names, states.astype(np.uint8)


def test_cfg4_tree_vs_oracle(oracle_mod):
    """BASELINE cfg4's 1000-taxon tree (the stash overflows: HBM read-backs, TV_GENERIC)
    against the oracle on 4096 sites; sitewise 1e-12, lnL 1e-9 relative."""
    model, rm, tree, names, codes = _gtr_problem(1000, 4096, 41)
    tm = TreeModel()
    tm.set_alignment_codes(codes, np.eye(4), names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    tr = tm.traversal
    tips = {tr.names[n]: np.eye(4)[codes[i]] for n, i in tm.names.items()}
    ev, el, iv = model.engine_eigen()
    lnl, site = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                    tr.root_length(), ev, el, iv, model.freqs, rm.rates,
                                    rm.weights, n_nodes=tr.n_nodes, nthreads=8)
    np.testing.assert_allclose(tm.sitewise_patterns(), site, rtol=1e-12, atol=1e-10)
    assert abs(tm.likelihood() - lnl) <= LNL_RTOL * abs(lnl)


def test_cfg4_full_shard_site_additivity():
    """BASELINE cfg4 per-GPU shard at full size (1000 taxa x 125k sites), through a size-
    independent property: every site's lnL is the same whether the site is evaluated in the
    whole shard or in either half (bit for bit: a site's arithmetic does not depend on S),
    and the totals add up (1e-12 relative)."""
    model, rm, tree, names, codes = _gtr_problem(1000, 125_000, 43)
    half = 62_500
    res = []
    for lo, hi in ((0, 125_000), (0, half), (half, 125_000)):
        tm = TreeModel(keep_partials=False)
        tm.set_alignment_codes(np.ascontiguousarray(codes[:, lo:hi]), np.eye(4), names)
        tm.set_substitution_model(model)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        res.append((tm.likelihood(), tm.sitewise_patterns().copy()))
        del tm
    (l_all, s_all), (l_a, s_a), (l_b, s_b) = res
    np.testing.assert_array_equal(s_all, np.concatenate([s_a, s_b]))
    assert abs(l_all - (l_a + l_b)) <= 1e-12 * abs(l_all)
    assert np.isfinite(l_all)


def test_cfg5_trees_vs_oracle(oracle_mod):
    """BASELINE cfg5 shape (100-taxon trees, 50k-site alignment): several independent
    topologies on one resident alignment (TreeShardedLikelihoods, tips uploaded once)
    against the oracle, tree by tree."""
    from phylo_utils_amd.parallel import TreeShardedLikelihoods
    from phylo_utils_amd.synthetic import random_tree
    model, rm, tree, names, codes = _gtr_problem(100, 50_000, 47)
    trees = [random_tree(np.random.default_rng(100 + i), 100) for i in range(3)]
    got = TreeShardedLikelihoods(trees, codes, np.eye(4), names, model, rm,
                                 device=0).local_likelihoods()
    ev, el, iv = model.engine_eigen()
    for t, g in zip(trees, got):
        tr = Traversal(prepare_tree(t))
        tips = {tr.names[n]: np.eye(4)[codes[i]] for i, n in enumerate(names)}
        lnl, _ = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(),
                                     tr.root_edge, tr.root_length(), ev, el, iv, model.freqs,
                                     rm.rates, rm.weights, n_nodes=tr.n_nodes, nthreads=8)
        assert abs(g - lnl) <= LNL_RTOL * abs(lnl), (g, lnl)


@pytest.mark.parametrize("split", ["0", "2"])
def test_protein_repeated_evaluations_vs_oracle(monkeypatch, oracle_mod, split):
    """K = 20 evaluations one after another on one context with different branch lengths:
    the fused P kernel (k_pmatrix_aa: P and the MFMA operands in one launch) gives the
    oracle's lnL every time, and the same lnL bitwise when a length set comes back.  (The
    PU_PMAT_BLOCK A/B switch is read once per process; the bench A/B runs it in a process of
    its own and compares lnL.)  split "2": the chain-task + top-task plan."""
    monkeypatch.setenv("PU_SPLIT", split)
    model = SM.LG()
    rm = GammaRateModel(4, 0.8)
    tree, names, states = make_problem(60, 700, model, rm.rates, seed=21)
    tm = TreeModel(keep_partials=True)
    tm.set_alignment_codes(states.astype(np.uint8), np.eye(20), names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    tr = tm.traversal
    tips = {tr.names[n]: np.eye(20)[states[i]] for i, n in enumerate(names)}
    ev, el, iv = model.engine_eigen()
    base = {e: tr.brlens[e] for e in list(tr.brlens.keys())}
    seen = {}
    for f in (1.0, 1.7, 0.6, 1.0, 1.7):
        for e, v in base.items():
            tr.brlens[e] = v * f
        tm.update_branch_lengths()
        got = tm.likelihood()
        lnl, _ = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                     tr.root_length(), ev, el, iv, model.freqs, rm.rates,
                                     rm.weights, n_nodes=tr.n_nodes, nthreads=8)
        assert abs(got - lnl) <= LNL_RTOL * abs(lnl), (f, got, lnl)
        if f in seen:
            assert got == seen[f]
        seen[f] = got


@pytest.mark.parametrize("name", ["cfg2_small", "cfg3_small"])
def test_store_mode_variable_is_ignored(monkeypatch, name):
    """PU_STORE_MODE=48 once made every op read side 0's P and drop the
    parent stores; the shipped library ignores it -- bitwise-equal lnL, sitewise and
    partials."""
    base, _ = build_model(name)
    monkeypatch.setenv("PU_STORE_MODE", "48")
    tm, _ = build_model(name)
    assert tm.likelihood() == base.likelihood()
    np.testing.assert_array_equal(tm.sitewise_patterns(), base.sitewise_patterns())
    np.testing.assert_array_equal(tm.partials, base.partials)


@pytest.mark.parametrize("dna,keep", [(False, True), (False, False), (True, True), (True, False)])
def test_split_handoff_under_changing_lengths(monkeypatch, dna, keep):
    """A split traversal hands each chain root to the workgroup that runs the top task within
    one launch (write-through stores, a ticket per (tile, category) / workgroup, one acquire).
    A stale hand-off would show the previous evaluation's values: 12 evaluations (protein at
    cfg3 size; DNA 300 taxa x 20k sites) with the branch lengths changing every time, lnL,
    sitewise and root partials bitwise equal to the unsplit plan each time (also lnL-only:
    every chain task colours its HBM slots apart)."""
    model = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS) if dna else SM.LG()
    K = len(model.freqs)
    rm = GammaRateModel(4, 0.5 if dna else 0.8)
    tree, names, states = make_problem(300 if dna else 200, 20_000 if dna else 10_000, model,
                                       rm.rates, seed=3)

    def build(split):
        monkeypatch.setenv("PU_SPLIT", split)
        tm = TreeModel(keep_partials=keep)
        tm.set_alignment_codes(states.astype(np.uint8), np.eye(K), names)
        tm.set_substitution_model(model)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        return tm

    split, whole = build("3"), build("0")
    assert N.plan_stats(split.traversal.n_nodes, split.traversal.postorder_traversal,
                        split.traversal.root_edge, 3, 3)["chains"] >= 2
    base = {e: v for e, v in split.traversal.brlens.items()}
    rng = np.random.default_rng(9)
    for it in range(12):
        f = rng.uniform(0.3, 2.0, size=len(base))
        for tm in (split, whole):
            for (e, v), fe in zip(base.items(), f):
                tm.traversal.brlens[e] = v * fe
            tm.update_branch_lengths()
        assert split.likelihood() == whole.likelihood(), it
        np.testing.assert_array_equal(split.sitewise_patterns(), whole.sitewise_patterns())
        if not keep:
            continue
        rs, ws = split.compute_partials_at_edge(*split.traversal.root_edge)
        rw, ww = whole.compute_partials_at_edge(*whole.traversal.root_edge)
        np.testing.assert_array_equal(rs, rw)
        np.testing.assert_array_equal(ws, ww)


@pytest.mark.parametrize("name", ["cfg2_small", "deep_scaling", "ambig_dna", "k80_g1"])
def test_lnl_only_tip_products_bitwise(monkeypatch, name):
    """lnL-only coded DNA traversals take a tip child's product from PT = P * table rows built
    in the P launch (TV_PTIP) with matvec_s's operation order: lnL and sitewise bitwise equal
    to the in-kernel products (PU_NO_PTIP), ambiguity codes included."""
    monkeypatch.delenv("PU_NO_PTIP", raising=False)
    base, _ = build_model(name, keep_partials=False)
    l0, s0 = base.likelihood(), base.sitewise_patterns().copy()
    monkeypatch.setenv("PU_NO_PTIP", "1")
    tm, _ = build_model(name, keep_partials=False)
    assert tm.likelihood() == l0
    np.testing.assert_array_equal(tm.sitewise_patterns(), s0)



@pytest.mark.parametrize("env", [{"PU_LDS_SLOTS": "3"}, {"PU_LDS_SLOTS": "5"},
                                 {"PU_KEEP_OCC": "6"}])
def test_register_stash_slots_bitwise(monkeypatch, env):
    """A 500-taxon KEEP plan at 4 workgroups per CU overflows its 3 LDS stash slots; the
    occupancy plan keeps two more waiting parents in registers (TV_RSLOTS) instead of reading
    them back from HBM.  Partials, scalers and lnL are bitwise those of the plans without
    register slots: 3 LDS slots with HBM read-backs, 5 LDS slots, 6 workgroups per CU."""
    rm = GammaRateModel(4, 0.5)
    model = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    tree, names, states = make_problem(500, 3000, model, rm.rates, seed=17)

    def build():
        tm = TreeModel(keep_partials=True)
        tm.set_alignment_codes(states.astype(np.uint8), np.eye(4), names)
        tm.set_substitution_model(model)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        return tm

    monkeypatch.delenv("PU_LDS_SLOTS", raising=False)
    monkeypatch.delenv("PU_KEEP_OCC", raising=False)
    base = build()
    assert N.plan_stats(base.traversal.n_nodes, base.traversal.postorder_traversal,
                        base.traversal.root_edge, 0, 3)["mem"] > 0  # 3 LDS slots overflow
    l0, s0, p0, c0 = base.likelihood(), base.sitewise_patterns(), base.partials, base.scale
    del base
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    tm = build()
    assert tm.likelihood() == l0
    np.testing.assert_array_equal(tm.sitewise_patterns(), s0)
    np.testing.assert_array_equal(tm.partials, p0)
    np.testing.assert_array_equal(tm.scale, c0)


@pytest.mark.parametrize("name", ["deep_scaling", "cfg3_small", "long_branches"])
def test_split_plans_with_dense_tips(monkeypatch, name):
    """Split plans (chain tasks + top task) with dense tip partials (compact_tips=False: the
    traversal reads tip vectors from HBM instead of codes): bitwise the unsplit plan."""
    monkeypatch.setenv("PU_SPLIT", "0")
    base, _ = build_model(name, compact_tips=False)
    l0, s0, p0 = base.likelihood(), base.sitewise_patterns().copy(), base.partials.copy()
    for split in ("2", "8"):
        monkeypatch.setenv("PU_SPLIT", split)
        tm, _ = build_model(name, compact_tips=False)
        assert tm.likelihood() == l0
        np.testing.assert_array_equal(tm.sitewise_patterns(), s0)
        np.testing.assert_array_equal(tm.partials, p0)


@pytest.mark.parametrize("env", [{"PU_KEEP_OCC": "3"}, {"PU_KEEP_OCC": "5"},
                                 {"PU_KEEP_OCC": "6"}, {"PU_KEEP_OCC": "7"},
                                 {"PU_LDS_PAD": "17408"}, {"PU_SPLIT": "9"}])
def test_keep_occupancy_rule_bitwise(monkeypatch, env):
    """DNA KEEP plans are occupancy plans (pu_set_schedule / keep_occupancy): k
    workgroups per CU, the most stash slots that fit, the build that allows k.  Every forced
    k (3..7: 1-5 stash slots, the 7-wave build), an explicit pad and a split plan compute the
    same partials, scalers and lnL bit for bit as the chosen plan (84k sites: 1313
    workgroups).  The streamed stores are written through the L2 (sc1 nt)."""
    rm = GammaRateModel(4, 0.5)
    model = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    tree, names, states = make_problem(50, 84000, model, rm.rates, seed=3)

    def build():
        tm = TreeModel(keep_partials=True)
        tm.set_alignment_codes(states.astype(np.uint8), np.eye(4), names)
        tm.set_substitution_model(model)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        return tm

    base = build()
    l0, s0 = base.likelihood(), base.sitewise_patterns()
    p0, c0 = base.partials, base.scale
    del base
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    tm = build()
    assert tm.likelihood() == l0
    np.testing.assert_array_equal(tm.sitewise_patterns(), s0)
    np.testing.assert_array_equal(tm.partials, p0)
    np.testing.assert_array_equal(tm.scale, c0)


@pytest.mark.parametrize("dna", [True, False])
def test_padded_tile_pitch_vs_oracle(oracle_mod, dna):
    """tile_pitch (pu_internal.h): 16384 sites are 256 tiles, and a slot spans C x 257 blocks
    (protein: 257 per category row; DNA: tile-major rows, layout_row), so every layout reader
    (traversal, read-backs, untile, edges, root) must use the pitch and layout_row and every
    loop the tile count.  Coded tips, KEEP and lnL-only: lnL,
    sitewise, all partials and scalers, and the partials at the root edge against the oracle."""
    if dna:
        model, ntax, alpha = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS), 24, 0.5
    else:
        model, ntax, alpha = SM.LG(), 6, 0.8
    S = 16384
    rm = GammaRateModel(4, alpha)
    tree, names, states = make_problem(ntax, S, model, rm.rates, seed=11)
    K = len(model.freqs)
    for keep in (True, False):
        tm = TreeModel(keep_partials=keep)
        tm.set_alignment_codes(np.asarray(states, dtype=np.uint8), np.eye(K), names)
        tm.set_substitution_model(model)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        tr = tm.traversal
        tips = {tr.names[n]: np.eye(K)[states[i]] for n, i in tm.names.items()}
        ev, el, iv = model.engine_eigen()
        ref = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                  tr.root_length(), ev, el, iv, model.freqs, rm.rates,
                                  rm.weights, n_nodes=tr.n_nodes, return_all=True)
        np.testing.assert_allclose(tm.sitewise_patterns(), ref["site_lnl"], rtol=1e-12, atol=1e-10)
        assert abs(tm.likelihood() - ref["lnl"]) <= LNL_RTOL * abs(ref["lnl"])
        if keep:
            if not dna:
                # protein: against the oracle on the device's own P (the partials' 2e-12
                # deviation on the oracle's P is P's rounding, test_protein_partials_deviation_
                # is_the_pmatrix); the layout is what this test is about
                P = np.empty((len(tr.postorder_traversal) + 1, 2, 4, K, K))
                N.check(N.lib().pu_get_pmatrices(tm._ctx, N.ptr(P)))
                ref = oracle_mod.tree_lnl_p(tips, tr.postorder_traversal, P[:-1], P[-1],
                                            tr.root_edge, model.freqs, rm.weights,
                                            n_nodes=tr.n_nodes, return_all=True)
            assert_partials_close(tm.partials, ref["partials"], rtol=1e-12)
            np.testing.assert_allclose(tm.scale, ref["scale"], rtol=1e-13, atol=1e-10)
            rp, rs = tm.compute_partials_at_edge(*tr.root_edge)
            assert_partials_close(rp, ref["root_partials"], rtol=1e-12)
            np.testing.assert_allclose(rs, ref["root_scale"], rtol=1e-13, atol=1e-10)


def _max_vec_err(got, ref):
    scale = np.abs(ref).max(axis=-1, keepdims=True)
    return float((np.abs(got - ref) / np.where(scale > 0, scale, 1)).max())


def test_protein_partials_deviation_is_the_pmatrix(oracle_mod):
    """the protein partials of the 16384-site pitch tree deviated from the
    oracle by up to 2.1e-12 of a vector's largest entry (1e-12 elsewhere).  The cause is P, not
    the traversal: k_pmatrix_aa forms each entry as fma(evecs[i][k] e^(l_k t r), ivecs[k][j],
    acc) (the fused form every P builder here shares) and the C oracle as a separate multiply
    and add; LG's eigenvectors mix signs, so the small entries of a short branch's P are sums
    that cancel, and their last-bit differences, relative to the entry, are far above 1e-16.
    Pinned here: with the device's own P the oracle's partials agree to 1e-13 (the MFMA
    products and the oracle's sequential ones), while the two P differ by at most a few ulp
    of 1 -- and the full deviation on the oracle's P stays below 5e-12."""
    model, ntax, alpha, S = SM.LG(), 6, 0.8, 16384
    rm = GammaRateModel(4, alpha)
    tree, names, states = make_problem(ntax, S, model, rm.rates, seed=11)
    tm = TreeModel(keep_partials=True)
    tm.set_alignment_codes(np.asarray(states, dtype=np.uint8), np.eye(20), names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    tr = tm.traversal
    tips = {tr.names[n]: np.eye(20)[states[i]] for n, i in tm.names.items()}
    ev, el, iv = model.engine_eigen()
    own = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                              tr.root_length(), ev, el, iv, model.freqs, rm.rates, rm.weights,
                              n_nodes=tr.n_nodes, return_all=True)
    P = np.empty((len(tr.postorder_traversal) + 1, 2, 4, 20, 20))
    N.check(N.lib().pu_get_pmatrices(tm._ctx, N.ptr(P)))
    dev = oracle_mod.tree_lnl_p(tips, tr.postorder_traversal, P[:-1], P[-1], tr.root_edge,
                                model.freqs, rm.weights, n_nodes=tr.n_nodes, return_all=True)
    parts = tm.partials
    e_dev = _max_vec_err(parts, dev["partials"])
    e_own = _max_vec_err(parts, own["partials"])
    dP = float(np.abs(P[:-1] - own["P"]).max())
    print("partials vs oracle on device P %.2e, on its own P %.2e; max |dP| %.2e"
          % (e_dev, e_own, dP))
    assert e_dev <= 1e-13, e_dev
    assert dP <= 1e-15, dP
    assert e_own <= 5e-12, e_own


# ---------------------------------------------------------------- layout pitch (r05)
@pytest.mark.parametrize("env", [{"PU_PITCH_EXTRA": "1"}, {"PU_PITCH_EXTRA": "3"},
                                 {"PU_PITCH_EXTRA": "7"}])
def test_layout_pitch_bitwise(monkeypatch, env):
    """Unused tiles added to every layout row (PU_PITCH_EXTRA, the r05 pitch A/B knob) are
    layout only: lnL, sitewise lnL, every partial and scaler, the root, an edge lnL and
    derivatives, and the values after new branch lengths are bitwise those of tile_pitch(S)."""
    rm = GammaRateModel(4, 0.5)
    model = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    tree, names, states = make_problem(40, 20000, model, rm.rates, seed=23)

    def build():
        tm = TreeModel(keep_partials=True)
        tm.set_alignment_codes(states.astype(np.uint8), np.eye(4), names)
        tm.set_substitution_model(model)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        return tm

    def snapshot(tm):
        a, b = tm.traversal.postorder_traversal[3][:2]  # (parent, first child)
        return (tm.likelihood(), tm.sitewise_patterns().copy(), tm.partials, tm.scale,
                tm.root_partials.copy(), tm.root_scale.copy(),
                tm.compute_likelihood_at_edge(a, b), tm.edge_derivatives(a, b))

    base = build()
    plan0 = N.ctx_plan(base._ctx)
    assert plan0["pitch_extra"] == 0
    ref = snapshot(base)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    tm = build()
    plan = N.ctx_plan(tm._ctx)
    assert plan["pitch_extra"] == int(env["PU_PITCH_EXTRA"])
    assert plan["pitch"] == plan0["pitch"] + plan["pitch_extra"]
    got = snapshot(tm)
    assert got[0] == ref[0]
    for g, r in zip(got[1:], ref[1:]):
        np.testing.assert_array_equal(g, r)
    b0 = dict(tm.traversal.brlens)
    for m in (base, tm):
        for e, v in b0.items():
            m.traversal.brlens[e] = v * 1.3
        m.update_branch_lengths()
    assert tm.likelihood() == base.likelihood()
    np.testing.assert_array_equal(tm.partials, base.partials)
    np.testing.assert_array_equal(tm.scale, base.scale)
