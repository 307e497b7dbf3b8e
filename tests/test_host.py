"""Host-side mirror of the reference interface (no GPU): substitution models, data
tables, charmaps, discrete gamma, newick/traversal, alignment encoding."""
import numpy as np
import pytest

from conftest import load_golden, tree_case, golden_charmap

from phylo_utils_amd import alignment as A
from phylo_utils_amd import substitution_models as SM
from phylo_utils_amd import tree as T
from phylo_utils_amd.discrete_gamma import discrete_gamma
from phylo_utils_amd.rate_models import (GammaRateModel, InvariantGammaModel,
                                         InvariantSitesModel, UniformRateModel)

F = [0.1, 0.2, 0.3, 0.4]
CFG2 = ([1.2, 3.5, 0.8, 1.1, 4.2, 1.0], [0.30, 0.20, 0.25, 0.25])
ZOO = {
    "gtr_default": lambda: SM.GTR(),
    "gtr_cfg2": lambda: SM.GTR(*CFG2),
    "gtr_test": lambda: SM.GTR([6., 5., 4., 3., 2., 1.], F),
    "k80_2": lambda: SM.K80(2.0),
    "k80_1_5": lambda: SM.K80(1.5),
    "f81": lambda: SM.F81(F),
    "f84": lambda: SM.F84(1.5, F),
    "hky85": lambda: SM.HKY85(1.5, F),
    "tn93": lambda: SM.TN93(2.5, 2.4, freqs=F),
    "lg": lambda: SM.LG(),
    "wag": lambda: SM.WAG(),
    "jtt": lambda: SM.JTT(),
    "dayhoff": lambda: SM.Dayhoff(),
}


@pytest.mark.parametrize("name", sorted(ZOO))
def test_model_q_and_p_match_reference(name):
    g = load_golden("models")
    m = ZOO[name]()
    np.testing.assert_allclose(m.q(), g[name + "_q"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(m.freqs, g[name + "_freqs"], rtol=0, atol=0)
    for t, pref in zip(g["ts"], g[name + "_p"]):
        np.testing.assert_allclose(m.p(t, g["rates"]), pref, rtol=1e-10, atol=2e-14)
    assert m.detailed_balance()
    assert abs(np.dot(m.freqs, -np.diag(m.q())) - 1.0) < 1e-12


def test_jc69_closed_form_and_rates():
    g = load_golden("models")
    jc = SM.JC69()
    for t, pref in zip(g["ts"], g["jc69_p"]):
        np.testing.assert_allclose(jc.p(t), pref, rtol=1e-13, atol=1e-15)
    # JC69 == GTR() through the engine path
    np.testing.assert_allclose(jc.p(0.3, [0.5, 2.0]), SM.GTR().p(0.3, [0.5, 2.0]), atol=1e-14)
    np.testing.assert_allclose(jc.q(), g["jc69_q"], atol=1e-15)


def test_nonreversible_models_are_not_reversible():
    s = SM.Strsym([1., 2., 3., 4., 5., 6.])
    u = SM.Unrest([[0., 1., 2., 3.], [4., 0., 5., 6.], [7., 8., 0., 9.], [10., 11., 12., 0.]])
    assert not s.detailed_balance() and not u.detailed_balance()
    assert abs(s.freqs[0] - s.freqs[3]) < 1e-12 and abs(s.freqs[1] - s.freqs[2]) < 1e-12
    np.testing.assert_allclose(s.p(0.3).sum(1), 1.0)
    with pytest.raises(NotImplementedError):
        u.engine_eigen()


def test_input_validation_like_reference():
    with pytest.raises(ValueError):
        SM.check_frequencies(np.array([0.25] * 4), 5)
    with pytest.raises(ValueError):
        SM.check_frequencies(np.array([0.250001, 0.25, 0.25, 0.25]), 4)
    with pytest.raises(ValueError):
        SM.check_rates(-np.ones((4, 4)), 4)
    with pytest.raises(ValueError):
        SM.GTR([1, 2, 3, 4, 5, 6], [0.5, 0.5, 0.1, 0.1])


def test_protein_tables_match_reference():
    from phylo_utils_amd import data
    g = load_golden("models")
    for nm in ("lg", "wag", "jtt", "dayhoff"):
        np.testing.assert_array_equal(getattr(data, nm + "_rates"), g[nm + "_rates_table"])
        np.testing.assert_array_equal(getattr(data, nm + "_freqs"), g[nm + "_freqs_table"])


def test_discrete_gamma_bitwise_equal_to_paml():
    """Host C++ (libphylo_hip.so, no device call) vs the reference's PAML C."""
    g = load_golden("gamma")
    for i, a in enumerate(g["alphas"]):
        for j, c in enumerate(g["ncats"]):
            c = int(c)
            np.testing.assert_array_equal(discrete_gamma(a, c), g["mean"][i, j, :c])
            np.testing.assert_array_equal(discrete_gamma(a, c, True), g["median"][i, j, :c])
    np.testing.assert_allclose(discrete_gamma(0.5, 5),
                               [0.02121238, 0.15548577, 0.46708288, 1.10711735, 3.24910162],
                               atol=5e-9)
    np.testing.assert_array_equal(discrete_gamma(0.7, 1), [1.0])
    with pytest.raises(RuntimeError):
        discrete_gamma(-1.0, 4)


def test_rate_models():
    g = GammaRateModel(4, 0.5)
    np.testing.assert_allclose(g.weights, 0.25)
    np.testing.assert_allclose(np.mean(g.rates), 1.0, rtol=1e-6)
    g.alpha = 2.0
    np.testing.assert_array_equal(g.rates, discrete_gamma(2.0, 4))
    u = UniformRateModel()
    assert u.ncat == 1 and u.rates[0] == 1.0
    i = InvariantSitesModel(0.2)
    np.testing.assert_allclose(i.rates, [0, 1.25])
    ig = InvariantGammaModel(0.2, 4, 0.5)
    assert ig.ncat == 5
    np.testing.assert_allclose(ig.weights.sum(), 1.0)
    with pytest.raises(ValueError):
        InvariantSitesModel(1.0)


@pytest.mark.parametrize("kind,alpha", [("dna", A.DNA), ("protein", A.PROTEIN),
                                        ("binary", A.BINARY)])
def test_charmaps_match_reference(kind, alpha):
    ref = golden_charmap(kind)
    assert set(ref) == set(A.CHARMAPS[alpha])
    for ch, v in ref.items():
        np.testing.assert_array_equal(A.CHARMAPS[alpha][ch], v, err_msg=ch)
    s = "".join(sorted(ref))
    np.testing.assert_array_equal(A.seq_to_partials(s, alpha), [ref[c] for c in s])
    np.testing.assert_array_equal(A.seq_to_partials(s, kind), [ref[c] for c in s])


def test_pattern_compression_like_reference():
    aln = [("a", "AACGTA-"), ("b", "AACGTAN"), ("c", "ATCGTAA")]
    parts, w, inv, names = A.alignment_to_numpy(aln, A.DNA)
    full = np.stack([A.seq_to_partials(s, A.DNA) for _, s in aln])
    ref, rinv, rw = np.unique(full, return_inverse=True, return_counts=True, axis=1)
    np.testing.assert_array_equal(parts, ref)
    np.testing.assert_array_equal(w, rw)
    np.testing.assert_array_equal(parts[:, inv], full)
    assert names == {"a": 0, "b": 1, "c": 2}
    codes, table = A.partials_to_codes(parts)
    np.testing.assert_array_equal(table[codes], parts)
    assert A.invariant_sites(parts)[0]


def test_fasta_reader(tmp_path):
    p = tmp_path / "x.fa"
    p.write_text(">s1 desc\nACGT\nAC\n>s2\nAAGTTT\n")
    assert A.read_fasta(str(p)) == [("s1", "ACGTAC"), ("s2", "AAGTTT")]


def test_newick_and_traversal_shapes():
    tr = T.Traversal(T.prepare_tree("((a:0.1,b:0.2):0.3,(c:0.1,d:0.4):0.2,e:1);"))
    assert tr.n_nodes == 2 * 5 - 2
    assert tr.postorder_traversal.shape == (3, 3)
    assert tr.root_length() == 0.3
    assert sorted(tr.names) == list("abcde")
    # every internal node appears once as parent; children before parents
    seen = set(tr.names.values())
    for p, a, b in tr.postorder_traversal:
        assert a in seen and b in seen
        seen.add(p)
    assert set(tr.root_edge) <= seen


def test_deroot_moves_length_to_sister():
    t = T.parse_newick("((a:1,b:2):0.5,(c:1,d:1):0.25);").deroot()
    lens = sorted(c.edge_length for c in t.seed_node.children)
    assert len(t.seed_node.children) == 3 and lens == [0.75, 1.0, 1.0]


def test_newick_roundtrip_quoted_and_comments():
    t = T.parse_newick("('x y':1[&c],(b:2,'c''d':3)n1:4)r;")
    t2 = T.parse_newick(t.as_newick())
    assert sorted(n.label for n in t2.leaf_nodes()) == ["b", "c'd", "x y"]
    assert [n.edge_length for n in t2.leaf_nodes()] == [1.0, 2.0, 3.0]


def test_deep_caterpillar_no_recursion_limit():
    n = 3000
    s = "t0:0.1"
    for i in range(1, n):
        s = "(%s,t%d:0.1):0.1" % (s, i)
    tr = T.Traversal(T.prepare_tree(s + ";"))
    assert tr.postorder_traversal.shape == (n - 2, 3)


@pytest.mark.parametrize("name", ["cfg1_jc", "cfg2_small", "deep_scaling", "ambig_dna"])
def test_newick_schedule_reproduces_golden_lnl(oracle_mod, name):
    """Our newick -> deroot/resolve -> Traversal schedule, evaluated by the oracle, gives the
    reference's lnL (reversible model: root placement invariant)."""
    c = tree_case(name)
    tr = T.Traversal(T.prepare_tree(c["newick"]))
    cm = golden_charmap("dna")
    tips = {tr.names["t%d" % i]: np.array([cm[ch] for ch in s])
            for i, s in enumerate(c["seq_strings"])}
    lnl, site = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                    tr.root_length(), c["evecs"], c["evals"], c["ivecs"],
                                    c["freqs"], c["rates"], c["weights"], n_nodes=tr.n_nodes)
    np.testing.assert_allclose(site, c["site_lnl"], rtol=1e-10, atol=1e-9)


def test_code_columns_sort_like_partial_columns():
    """alignment.char_codes numbers characters so that np.unique over code columns gives the
    reference's np.unique over float partial columns (alignment.py:40-57): same unique
    patterns (through the table), inverse index and counts -- the property the GPU pattern
    compression (pu_compress_patterns) relies on."""
    rng = np.random.default_rng(11)
    for alpha, chars in ((A.DNA, "ACGTRYMKWSBDHVN-acgtn"), (A.PROTEIN, "ACDEFGHIKLMNPQRSTVWY-?Xx")):
        for nt, S in ((1, 5), (3, 40), (9, 300)):
            pool = np.array(list(chars))
            cols = pool[rng.integers(0, len(pool), size=(nt, S // 2 + 1))]
            seqs = cols[:, rng.integers(0, cols.shape[1], size=S)]  # duplicated columns
            recs = [("t%d" % i, "".join(r)) for i, r in enumerate(seqs)]
            parts, w, inv, names = A.alignment_to_numpy(recs, alpha)
            codes, table, names2 = A.char_codes(recs, alpha)
            assert names2 == names
            u, inv2, cnt = np.unique(codes, axis=1, return_inverse=True, return_counts=True)
            np.testing.assert_array_equal(table[u], parts)
            np.testing.assert_array_equal(np.asarray(inv2).reshape(-1), inv)
            np.testing.assert_array_equal(cnt, w)
    with pytest.raises(ValueError, match="not in the alphabet"):
        A.char_codes([("a", "AC!")], A.DNA)
