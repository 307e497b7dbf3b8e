"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run only in the survey container, where /root/reference exists:

    python tests/golden/make_golden.py            # rewrites tests/golden/*.npz
    python tests/golden/make_golden.py nonrev     # only nonrev.npz
    python tests/golden/make_golden.py edges      # only edges.npz and cfg5_small.npz
    python tests/golden/make_golden.py band       # only clv_band.npz

What runs, and why this is the reference and not a re-implementation
---------------------------------------------------------------------
* ``phylo_utils.substitution_models`` (Q, eigen, ``Model.p``) and
  ``phylo_utils.data`` (LG/WAG/JTT/Dayhoff tables) are imported unmodified from
  /root/reference.  ``phylo_utils/__init__.py`` eagerly imports compiled
  extensions and numba (absent here), so a bare package object is registered
  instead of executing that initialiser; the submodules themselves are the
  reference's files.
* ``phylo_utils.likelihood.python_likelihood_engine`` -- the reference's own
  pure-numpy engine (``clv``, ``lnl_node``; same math as the live numba engine,
  layout ``probs[K,K,C]`` / ``clv[S,K,C]``; rescale threshold eps instead of
  2^-128).  The live numba engine cannot be imported (numba is not installed),
  and no stand-in for numba is used.  Fixtures are built so both thresholds
  agree: CLV magnitudes either >= eps (no rescale in either engine) or < 2^-128
  (rescale in both); whole-tree lnL is independent of the rescaling
  representation.
* Discrete-gamma rates come from the reference's PAML C
  (``src/c_discrete_gamma.c``) compiled in place by oracle/Makefile into
  oracle/_ref/ (``src/discrete_gamma.pyx:30-47`` calls it with alpha == beta).
* The TreeModel loop (``tree_model.py:160-217``) is a dozen lines of driver;
  it is restated here around the reference's own clv / lnl_node / Model.p.
  Trees are stored as the schedule they were evaluated with *and* as newick.
"""
from __future__ import annotations

import importlib
import os
import sys
import types

import numpy as np
from scipy.special import logsumexp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("PHYLO_REF", "/root/reference")
sys.path.insert(0, ROOT)

from oracle import oracle as orc  # noqa: E402  (reference PAML C via oracle/_ref)


def load_reference():
    pkg = types.ModuleType("phylo_utils")
    pkg.__path__ = [os.path.join(REF, "phylo_utils")]
    sys.modules["phylo_utils"] = pkg
    sm = importlib.import_module("phylo_utils.substitution_models")
    pe = importlib.import_module("phylo_utils.likelihood.python_likelihood_engine")
    data = importlib.import_module("phylo_utils.data")
    charmaps = importlib.import_module("phylo_utils.alignment.charmaps")
    return sm, pe, data, charmaps


SM, PE, DATA, CHARMAPS = load_reference()

CFG2_RATES = [1.2, 3.5, 0.8, 1.1, 4.2, 1.0]  # SURVEY 8(d) M2, order AC AG AT CG CT GT
CFG2_FREQS = [0.30, 0.20, 0.25, 0.25]
DNA = "ACGT"
PROT = "ARNDCQEGHILKMFPSTWYV"


# ------------------------------------------------------------------ reference engine glue
def ref_p(model, t, rates):
    """Model.p stacked [C,K,K] -> the python engine's probs layout [K,K,C]."""
    return np.ascontiguousarray(np.moveaxis(model.p(t, rates), 0, -1))


def ref_clv(p1, p2, clv1, clv2, sa, sb):
    """Reference python-engine clv on our [S][C][K] layout; returns (out, cml)."""
    a = np.ascontiguousarray(np.moveaxis(clv1, 2, 1))
    b = np.ascontiguousarray(np.moveaxis(clv2, 2, 1))
    cml = np.zeros_like(sa)
    out = PE.clv(np.ascontiguousarray(np.moveaxis(p1, 0, -1)),
                 np.ascontiguousarray(np.moveaxis(p2, 0, -1)), a, b, sa, sb, cml)
    return np.ascontiguousarray(np.moveaxis(out, 1, 2)), cml


class Node:
    __slots__ = ("children", "length", "name", "idx")

    def __init__(self, children=(), length=0.0, name=None):
        self.children = list(children)
        self.length = length
        self.name = name
        self.idx = -1


def random_tree(rng, n, lo=0.01, hi=0.3):
    """Random pairwise joining -> seed node with two children."""
    active = [Node(length=rng.uniform(lo, hi), name="t%d" % i) for i in range(n)]
    while len(active) > 2:
        i, j = sorted(rng.choice(len(active), 2, replace=False))
        b, a = active.pop(j), active.pop(i)
        active.append(Node([a, b], rng.uniform(lo, hi)))
    return Node(active, 0.0)


def postorder(node):
    for c in node.children:
        yield from postorder(c)
    yield node


def schedule(seed):
    """traversal.py:16-29 semantics on our own tree: post-order index of non-seed nodes,
    ops (par, ch1, ch2) over non-seed internal nodes, root edge = seed's two children."""
    i = 0
    for nd in postorder(seed):
        if nd is seed:
            continue
        nd.idx = i
        i += 1
    ops, lens = [], []
    for nd in postorder(seed):
        if nd is seed or not nd.children:
            continue
        c1, c2 = nd.children
        ops.append((nd.idx, c1.idx, c2.idx))
        lens.append((c1.length, c2.length))
    a, b = seed.children
    return (np.array(ops, dtype=np.int32), np.array(lens), (a.idx, b.idx),
            a.length + b.length, i)


def newick(node, root=True):
    if node.children:
        s = "(" + ",".join(newick(c, False) for c in node.children) + ")"
    else:
        s = node.name
    if not root:
        s += ":" + repr(float(node.length))
    return s + (";" if root else "")


def simulate(rng, seed, model, rates, n_sites, alphabet):
    """Root ~ pi, category ~ U(C), child ~ row of P(t*r)."""
    K = len(alphabet)
    C = len(rates)
    cats = rng.integers(0, C, n_sites)
    states = {}
    root = rng.choice(K, n_sites, p=np.asarray(model.freqs) / np.sum(model.freqs))

    def evolve(node, parent_states):
        P = model.p(node.length, rates)  # [C,K,K]
        cum = np.cumsum(P[cats, parent_states, :], axis=1)
        u = rng.random(n_sites)[:, None] * cum[:, -1:]
        st = np.minimum((u > cum).sum(axis=1), K - 1)
        if node.children:
            for c in node.children:
                evolve(c, st)
        else:
            states[node.name] = st

    for c in seed.children:
        evolve(c, root)
    return {k: "".join(alphabet[i] for i in v) for k, v in states.items()}


def charmap_partials(seq, charmap):
    return np.array([charmap[ch] for ch in seq], dtype=np.float64)


def ref_tree_lnl(model, rates, weights, tips, ops, lens, root_edge, root_len, n_nodes,
                 return_partials=False):
    """tree_model.py:101-217 driver around the reference's python-engine clv/lnl_node
    (return_partials: also the post-order partials [n][S][K][C] and scalers [n][S][C])."""
    S, K = next(iter(tips.values())).shape
    C = len(rates)
    partials = np.zeros((n_nodes, S, K, C))
    scale = np.zeros((n_nodes, S, C))
    for n, t in tips.items():
        partials[n] = t[:, :, None]
    for (par, c1, c2), (l1, l2) in zip(ops, lens):
        partials[par] = PE.clv(ref_p(model, l1, rates), ref_p(model, l2, rates),
                               partials[c1], partials[c2], scale[c1], scale[c2], scale[par])
    a, b = root_edge
    root_partials = np.zeros((S, K, C))
    root_scale = np.zeros((S, C))
    PE.clv(ref_p(model, 0, rates), ref_p(model, root_len, rates), partials[a], partials[b],
           scale[a], scale[b], root_scale, root_partials)
    sw = PE.lnl_node(np.asarray(model.freqs), root_partials, root_scale)
    site = logsumexp(sw + np.log(weights), axis=1)
    if return_partials:
        return site, sw, partials, scale
    return site, sw


# ------------------------------------------------------------------ fixtures
def make_gamma():
    alphas = np.array([0.05, 0.1, 0.2, 0.5, 0.8, 1.0, 2.0, 5.0, 10.0, 50.0, 100.0, 200.0])
    ncats = np.array([2, 3, 4, 5, 6, 8, 10, 16])
    mean = np.zeros((len(alphas), len(ncats), 16))
    median = np.zeros_like(mean)
    for i, a in enumerate(alphas):
        for j, c in enumerate(ncats):
            mean[i, j, :c] = orc.ref_discrete_gamma(a, c, False)
            median[i, j, :c] = orc.ref_discrete_gamma(a, c, True)
    # docstring known answer, src/discrete_gamma.pyx:41-42
    kat = orc.ref_discrete_gamma(0.5, 5)
    assert np.allclose(kat, [0.02121238, 0.15548577, 0.46708288, 1.10711735, 3.24910162])
    np.savez_compressed(os.path.join(HERE, "gamma.npz"), alphas=alphas, ncats=ncats,
                        mean=mean, median=median, kat_0_5_5=kat)


def model_zoo():
    f = [0.1, 0.2, 0.3, 0.4]
    return [
        ("gtr_default", SM.GTR()),
        ("gtr_cfg2", SM.GTR(list(CFG2_RATES), list(CFG2_FREQS))),
        ("gtr_test", SM.GTR([6., 5., 4., 3., 2., 1.], f)),
        ("k80_2", SM.K80(2.0)),
        ("k80_1_5", SM.K80(1.5)),
        ("f81", SM.F81(f)),
        ("f84", SM.F84(1.5, f)),
        ("hky85", SM.HKY85(1.5, f)),
        ("tn93", SM.TN93(2.5, 2.4, freqs=f)),
        ("lg", SM.LG()),
        ("wag", SM.WAG()),
        ("jtt", SM.JTT()),
        ("dayhoff", SM.Dayhoff()),
    ]


def make_models():
    ts = np.array([0.0, 1e-6, 0.01, 0.1, 0.5, 2.5, 10.0])
    rates = orc.ref_discrete_gamma(0.5, 4)
    out = {"ts": ts, "rates": rates}
    for name, m in model_zoo():
        out[name + "_q"] = np.asarray(m.q())
        out[name + "_freqs"] = np.asarray(m.freqs)
        out[name + "_p"] = np.stack([m.p(t, rates) for t in ts])
    jc = SM.JC69()
    out["jc69_p"] = np.stack([jc.p(t) for t in ts])
    out["jc69_q"] = np.asarray(jc.q())
    for nm in ("lg", "wag", "jtt", "dayhoff"):
        out[nm + "_rates_table"] = np.asarray(getattr(DATA, nm + "_rates"))
        out[nm + "_freqs_table"] = np.asarray(getattr(DATA, nm + "_freqs"))
    np.savez_compressed(os.path.join(HERE, "models.npz"), **out)


def make_clv(rng):
    out = {}
    names = []
    for K, model in ((4, SM.GTR(list(CFG2_RATES), list(CFG2_FREQS))), (20, SM.LG())):
        for C in (1, 4):
            rates = orc.ref_discrete_gamma(0.5, C) if C > 1 else np.array([1.0])
            for regime in ("normal", "tiny"):
                S = 64
                p1 = model.p(rng.uniform(0.01, 0.5), rates)
                p2 = model.p(rng.uniform(0.01, 0.5), rates)
                clv1 = rng.uniform(0.05, 1.0, (S, C, K))
                clv2 = rng.uniform(0.05, 1.0, (S, C, K))
                if regime == "tiny":
                    clv1 *= 1e-25
                    clv2 *= 10.0 ** rng.uniform(-40, -25, (S, C, 1))
                sa = rng.uniform(-50, 0, (S, C))
                sb = rng.uniform(-50, 0, (S, C))
                res, cml = ref_clv(p1, p2, clv1, clv2, sa, sb)
                m = np.einsum("cij,scj->sci", p1, clv1) * np.einsum("cij,scj->sci", p2, clv2)
                mx = m.max(-1)
                # both engines agree only outside [2^-128, eps): assert the construction
                assert np.all((mx >= np.finfo(float).eps) | (mx < 2.0 ** -128))
                key = "k%d_c%d_%s" % (K, C, regime)
                names.append(key)
                for nm, arr in (("p1", p1), ("p2", p2), ("clv1", clv1), ("clv2", clv2),
                                ("sa", sa), ("sb", sb), ("out", res), ("cml", cml)):
                    out[key + "_" + nm] = arr
                # lnl_node on the produced partials
                pi = np.asarray(model.freqs)
                sw = PE.lnl_node(pi, np.ascontiguousarray(np.moveaxis(res, 2, 1)), cml)
                out[key + "_pi"] = pi
                out[key + "_lnl_node"] = sw
    out["cases"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "clv.npz"), **out)


def make_clv_band():
    """clv_band.npz: partial products whose largest entry lies in [2^-128, eps), the band
    where the reference's two engines part: the python engine rescales there (max < eps,
    python_likelihood_engine.py), the live numba engine does not (0 < max < 2^-128,
    numba_likelihood_engine.py:7,37-44).  The fixture holds the python engine's output; the
    tests compare representation-free quantities (each vector over its largest entry, the
    log of that entry plus the scaler, and lnl_node) and check that the numba rule left the
    band unscaled."""
    rng = np.random.default_rng(20261016)
    eps = np.finfo(float).eps
    out, names = {}, []
    for K, model in ((4, SM.GTR(list(CFG2_RATES), list(CFG2_FREQS))), (20, SM.LG())):
        for C in (1, 4):
            rates = orc.ref_discrete_gamma(0.5, C) if C > 1 else np.array([1.0])
            S = 256
            p1 = model.p(rng.uniform(0.01, 0.5), rates)
            p2 = model.p(rng.uniform(0.01, 0.5), rates)
            clv1 = rng.uniform(0.05, 1.0, (S, C, K)) * 10.0 ** rng.uniform(-20, -8, (S, C, 1))
            clv2 = rng.uniform(0.05, 1.0, (S, C, K)) * 10.0 ** rng.uniform(-20, -8, (S, C, 1))
            # a few vectors on either side of the band, and exact zeros
            clv1[::17] *= 1e-30
            clv2[5::19] *= 1e12
            clv1[3::31] = 0.0
            sa = rng.uniform(-50, 0, (S, C))
            sb = rng.uniform(-50, 0, (S, C))
            res, cml = ref_clv(p1, p2, clv1, clv2, sa, sb)
            m = np.einsum("cij,scj->sci", p1, clv1) * np.einsum("cij,scj->sci", p2, clv2)
            mx = m.max(-1)
            band = (mx >= 2.0 ** -128) & (mx < eps)
            assert band.mean() > 0.8 and (mx < 2.0 ** -128).any() and (mx >= eps).any()
            key = "k%d_c%d" % (K, C)
            names.append(key)
            pi = np.asarray(model.freqs)
            sw = PE.lnl_node(pi, np.ascontiguousarray(np.moveaxis(res, 2, 1)), cml)
            for nm, arr in (("p1", p1), ("p2", p2), ("clv1", clv1), ("clv2", clv2), ("sa", sa),
                            ("sb", sb), ("out", res), ("cml", cml), ("pi", pi),
                            ("lnl_node", sw), ("band", band)):
                out[key + "_" + nm] = arr
    out["cases"] = np.array(names)
    # a whole tree through the band: the reference driver's post-order partials of every
    # internal node, keyed by clade (the set of tip names below it)
    gtr2 = SM.GTR(list(CFG2_RATES), list(CFG2_FREQS))
    tc = tree_case(rng, "tree", 120, 32, gtr2, 0.5, 4, DNA, CHARMAPS.dna_charmap, 0.0,
                   lo=0.3, hi=1.2)
    out.update(tc)
    return_tree_partials(out, "tree", gtr2, CHARMAPS.dna_charmap)
    # protein (k_prune_mfma): LG+G4, fewer tips reach the band (1/20 per tip)
    lg = SM.LG()
    out.update(tree_case(rng, "aatree", 40, 32, lg, 0.5, 4, PROT, CHARMAPS.protein_charmap,
                         0.0, lo=0.3, hi=1.2))
    return_tree_partials(out, "aatree", lg, CHARMAPS.protein_charmap, min_band=300)
    np.savez_compressed(os.path.join(HERE, "clv_band.npz"), **out)


def return_tree_partials(out, pre, model, charmap, min_band=500):
    """Re-run the reference driver on the stored tree case `pre` with return_partials and
    store the internal nodes' partials [n][S][C][K], scalers [n][S][C] and clades."""
    g = {k[len(pre) + 1:]: v for k, v in out.items() if k.startswith(pre + "_")}
    ops, lens = g["ops"], g["lens"]
    names = ["t%d" % i for i in range(len(g["seqs"]))]
    seqs = ["".join(map(chr, r)) for r in g["seqs"]]
    tips = {int(i): charmap_partials(sq, charmap) for i, sq in zip(g["tip_index"], seqs)}
    site, sw, partials, scale = ref_tree_lnl(
        model, g["rates"], g["weights"], tips, ops, lens, tuple(g["root_edge"]),
        float(g["root_len"]), int(g["n_nodes"]), return_partials=True)
    assert np.allclose(site, g["site_lnl"], rtol=0, atol=0)
    clade = {int(i): {nm} for i, nm in zip(g["tip_index"], names)}
    keys, P, Sc = [], [], []
    for par, c1, c2 in ops:
        clade[int(par)] = clade[int(c1)] | clade[int(c2)]
        keys.append(",".join(sorted(clade[int(par)], key=lambda s: int(s[1:]))))
        P.append(np.moveaxis(partials[par], 2, 1))  # [S][K][C] -> [S][C][K]
        Sc.append(scale[par])
    P, Sc = np.stack(P), np.stack(Sc)
    # the python engine rescaled wherever max < eps; on the numba rule the vectors whose
    # unscaled max lies in [2^-128, eps) keep it: count them through the represented value
    lm = np.log(P.max(-1)) + Sc  # log of the represented max, representation-free
    band = (lm >= -128 * np.log(2.0)) & (lm < np.log(np.finfo(float).eps))
    assert band.sum() > min_band, band.sum()
    out[pre + "_clades"] = np.array(keys)
    out[pre + "_partials"] = P
    out[pre + "_scale"] = Sc


def make_charmaps():
    out = {}
    for nm in ("dna", "protein", "binary"):
        cm = getattr(CHARMAPS, nm + "_charmap")
        keys = sorted(cm)
        out[nm + "_chars"] = np.frombuffer("".join(keys).encode(), dtype=np.uint8)
        out[nm + "_vectors"] = np.array([cm[k] for k in keys], dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "charmaps.npz"), **out)


def tree_case(rng, name, n_taxa, n_sites, model, alpha, ncat, alphabet, charmap,
              ambiguity=0.0, lo=0.01, hi=0.3):
    rates = orc.ref_discrete_gamma(alpha, ncat) if ncat > 1 else np.array([1.0])
    weights = np.full(ncat, 1.0 / ncat)
    seed = random_tree(rng, n_taxa, lo, hi)
    ops, lens, root_edge, root_len, n_nodes = schedule(seed)
    seqs = simulate(rng, seed, model, rates, n_sites, alphabet)
    if ambiguity > 0:
        amb = [k for k in charmap if k not in alphabet]
        for k in list(seqs):
            s = list(seqs[k])
            for i in np.nonzero(rng.random(n_sites) < ambiguity)[0]:
                s[i] = amb[rng.integers(len(amb))]
            seqs[k] = "".join(s)
    leaves = [nd for nd in postorder(seed) if not nd.children]
    tips = {nd.idx: charmap_partials(seqs[nd.name], charmap) for nd in leaves}
    site, sw = ref_tree_lnl(model, rates, weights, tips, ops, lens, root_edge, root_len,
                            n_nodes)
    names = sorted(seqs, key=lambda s: int(s[1:]))
    seq_codes = np.stack([np.frombuffer(seqs[k].encode(), dtype=np.uint8) for k in names])
    tip_index = np.array([next(nd.idx for nd in leaves if nd.name == k) for k in names])
    return {
        name + "_newick": np.frombuffer(newick(seed).encode(), dtype=np.uint8),
        name + "_seqs": seq_codes,
        name + "_tip_index": tip_index,
        name + "_ops": ops, name + "_lens": lens,
        name + "_root_edge": np.array(root_edge), name + "_root_len": np.array(root_len),
        name + "_n_nodes": np.array(n_nodes),
        name + "_rates": rates, name + "_weights": weights, name + "_alpha": np.array(alpha),
        name + "_site_lnl": site, name + "_sw": sw, name + "_lnl": np.array(site.sum()),
        name + "_model": np.frombuffer(model._name.encode(), dtype=np.uint8),
        name + "_evecs": np.asarray(model.eigen.evecs), name + "_evals": np.asarray(model.eigen.evals),
        name + "_ivecs": np.ascontiguousarray(model.eigen.ivecs), name + "_freqs": np.asarray(model.freqs),
    }


def make_trees(rng):
    dna = CHARMAPS.dna_charmap
    prot = CHARMAPS.protein_charmap
    gtr2 = SM.GTR(list(CFG2_RATES), list(CFG2_FREQS))
    out = {}
    cases = [
        # cfg1: JC69 == GTR() defaults (JC69.p has no rates argument, jc69.py:39)
        ("cfg1_jc", 4, 100, SM.GTR(), 1.0, 1, DNA, dna, 0.0),
        ("cfg2_small", 50, 2000, gtr2, 0.5, 4, DNA, dna, 0.0),
        ("cfg3_small", 40, 300, SM.LG(), 0.8, 4, PROT, prot, 0.0),
        ("deep_scaling", 300, 64, gtr2, 0.5, 4, DNA, dna, 0.0),
        ("ambig_dna", 20, 500, SM.HKY85(2.0, [0.1, 0.2, 0.3, 0.4]), 1.0, 3, DNA, dna, 0.1),
        ("ambig_prot", 12, 200, SM.WAG(), 0.3, 6, PROT, prot, 0.05),
        ("k80_g1", 30, 400, SM.K80(2.0), 1.0, 1, DNA, dna, 0.0),
    ]
    for c in cases:
        out.update(tree_case(rng, *c))
    out["cases"] = np.array([c[0] for c in cases])
    # deep tree with long branches: forces rescaling on many nodes
    out.update(tree_case(rng, "long_branches", 120, 80, gtr2, 0.5, 4, DNA, dna, 0.0,
                         lo=0.5, hi=2.0))
    out["cases"] = np.append(out["cases"], "long_branches")
    np.savez_compressed(os.path.join(HERE, "trees.npz"), **out)


def make_pulley():
    """tests/test_likelihood.py:35-49 pulley principle on the live semantics: K80(2),
    tips A|C, root at the cherry (0.1, 0.2) vs on the edge (0.0, 0.3)."""
    m = SM.K80(2.0)
    a = np.array([[1.0, 0, 0, 0]])
    c = np.array([[0, 1.0, 0, 0]])
    res = {}
    for nm, (t1, t2) in (("cherry", (0.1, 0.2)), ("edge", (0.0, 0.3))):
        root = np.zeros((1, 4, 1))
        sc = np.zeros((1, 1))
        PE.clv(ref_p(m, t1, [1.0]), ref_p(m, t2, [1.0]), a[:, :, None], c[:, :, None],
               np.zeros((1, 1)), np.zeros((1, 1)), sc, root)
        res[nm] = float(np.log((np.asarray(m.freqs) * root[0, :, 0]).sum()))
    assert abs(res["cherry"] - res["edge"]) < 1e-14
    assert abs(res["cherry"] - (-4.122814335054628)) < 1e-12  # SURVEY 0.3 probe value
    np.savez_compressed(os.path.join(HERE, "pulley.npz"), lnl_cherry=res["cherry"],
                        lnl_edge=res["edge"])


def make_nonrev():
    """Non-reversible DNA models (Strsym, Unrest; abstract.py:163-180): Q, freqs
    (q_to_freqs) and P = expm(Q r t) from the reference, plus whole-tree cases evaluated by
    the reference's engine on those P (tree_model.py:160-217 has no eigen step)."""
    rng = np.random.default_rng(20261016)
    ts = np.array([0.0, 1e-6, 0.01, 0.1, 0.5, 2.5])
    rates = orc.ref_discrete_gamma(0.5, 4)
    unrest_rates = np.array([[0, 1.5, 3.0, 0.7], [1.1, 0, 0.9, 4.1],
                             [2.6, 1.3, 0, 1.0], [0.6, 3.7, 1.2, 0]])
    strsym_rates = [1.4, 3.2, 0.8, 1.1, 0.9, 2.7]
    models = [("unrest", SM.Unrest(unrest_rates)), ("strsym", SM.Strsym(strsym_rates))]
    out = {"ts": ts, "rates": rates, "unrest_rates": unrest_rates,
           "strsym_rates": np.array(strsym_rates)}
    for nm, m in models:
        out[nm + "_q"] = np.asarray(m.q())
        out[nm + "_freqs"] = np.asarray(m.freqs)
        out[nm + "_p"] = np.stack([m.p(t, rates) for t in ts])
    dna = CHARMAPS.dna_charmap
    cases = [("unrest_g4", 24, 400, models[0][1], 0.5, 4, DNA, dna, 0.05),
             ("strsym_g1", 16, 300, models[1][1], 1.0, 1, DNA, dna, 0.0),
             ("unrest_deep", 200, 64, models[0][1], 0.5, 4, DNA, dna, 0.0)]
    for c in cases:
        d = tree_case(rng, *c)
        for k in ("_evecs", "_evals", "_ivecs"):  # np.linalg.eig of a non-symmetric Q
            d.pop(c[0] + k)
        out.update(d)
    out["cases"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(HERE, "nonrev.npz"), **out)


def ref_branch_derivs(probs3, pi, clv_a, clv_b, sa, sb):
    """The reference's lnl_branch_derivs (python_likelihood_engine.py:40-46, the body of
    numba_likelihood_engine.py:49-57) applied per (site, category): probs3 [C][3][K][K],
    clv_* [S][C][K], s* [S][C] -> [S][C][3]."""
    S, C, K = clv_a.shape
    out = np.zeros((S, C, 3))
    for s in range(S):
        for c in range(C):
            PE.lnl_branch_derivs(probs3[c], pi, clv_a[s, c], clv_b[s, c], sa[s, c:c + 1],
                                 sb[s, c:c + 1], out[s, c])
    return out


def mixture_derivs(per_cat, weights):
    """Per-site lnL, dlnL/dt, d2lnL/dt2 of the rate mixture sum_c w_c f_c e^(s_c) from the
    reference's per-category [log f + s, f'/f, (f''f - f'^2)/f^2] (driver arithmetic)."""
    o0, o1, o2 = per_cat[..., 0], per_cat[..., 1], per_cat[..., 2]
    a = o0 + np.log(weights)
    m = a.max(axis=1, keepdims=True)
    e = np.exp(a - m)
    L = e.sum(axis=1)
    L1 = (e * o1).sum(axis=1) / L
    L2 = (e * (o2 + o1 * o1)).sum(axis=1) / L - L1 * L1
    return np.stack([np.log(L) + m[:, 0], L1, L2], axis=1)


def make_edges():
    """SURVEY 8(f) N1 pinned on the reference: Model.dp_dt / d2p_dt2 (abstract.py:61-77,
    180-192), lnl_branch / lnl_branch_derivs of the python engine on random end vectors, and
    the root-edge derivatives of whole trees -- the reference's clv driver for the post-order
    partials, its lnl_branch_derivs per category with probs (P(t r), r dP(t r), r^2 d2P(t r))
    built from its dp_dt / d2p_dt2 at rate 1 (the chain-rule factor r that dp_dt(t, rates)
    omits, abstract.py:61-68), mixed over the categories."""
    rng = np.random.default_rng(20261017)
    ts = np.array([1e-6, 0.01, 0.1, 0.5, 2.5])
    rates = orc.ref_discrete_gamma(0.5, 4)
    unrest = SM.Unrest(np.array([[0, 1.5, 3.0, 0.7], [1.1, 0, 0.9, 4.1],
                                 [2.6, 1.3, 0, 1.0], [0.6, 3.7, 1.2, 0]]))
    models = [("gtr", SM.GTR(list(CFG2_RATES), list(CFG2_FREQS))), ("lg", SM.LG()),
              ("unrest", unrest)]
    out = {"ts": ts, "rates": rates}
    for nm, m in models:
        out[nm + "_dp"] = np.stack([m.dp_dt(t, rates) for t in ts])
        out[nm + "_d2p"] = np.stack([m.d2p_dt2(t, rates) for t in ts])
        out[nm + "_dp1"] = np.stack([m.dp_dt(t) for t in ts])      # rates=None form
        out[nm + "_d2p1"] = np.stack([m.d2p_dt2(t) for t in ts])
    # the seam functions on random end vectors (S = 48 sites, C = 4)
    for nm, m in models[:2]:
        K = len(m.freqs)
        S, C = 48, 4
        t = 0.37
        probs3 = np.stack([np.stack([m.p(t * r), r * m.dp_dt(t * r), r * r * m.d2p_dt2(t * r)])
                           for r in rates])                         # [C][3][K][K]
        ca = rng.uniform(0.01, 1.0, (S, C, K))
        cb = rng.uniform(0.01, 1.0, (S, C, K))
        sa = rng.uniform(-30, 0, (S, C))
        sb = rng.uniform(-30, 0, (S, C))
        pi = np.asarray(m.freqs)
        der = ref_branch_derivs(probs3, pi, ca, cb, sa, sb)
        # lnl_branch = out[0] of lnl_branch_derivs (the numba bodies are the same expression,
        # numba_likelihood_engine.py:55 and :79); the python engine's own lnl_branch cannot run:
        # it calls an unimported `log` (python_likelihood_engine.py:65, NameError)
        lnl = der[..., 0].copy()
        for k, v in (("probs3", probs3), ("clv_a", ca), ("clv_b", cb), ("sa", sa), ("sb", sb),
                     ("pi", pi), ("derivs", der), ("lnl", lnl)):
            out["seam_%s_%s" % (nm, k)] = v
    # whole trees: root-edge derivatives of the mixture at several lengths
    dna, prot = CHARMAPS.dna_charmap, CHARMAPS.protein_charmap
    for nm, m, n_taxa, n_sites, alphabet, charmap in (
            ("tree_gtr", models[0][1], 30, 400, DNA, dna),
            ("tree_lg", models[1][1], 12, 150, PROT, prot)):
        weights = np.full(len(rates), 1.0 / len(rates))
        seed = random_tree(rng, n_taxa)
        ops, lens, root_edge, root_len, n_nodes = schedule(seed)
        seqs = simulate(rng, seed, m, rates, n_sites, alphabet)
        leaves = [nd for nd in postorder(seed) if not nd.children]
        tips = {nd.idx: charmap_partials(seqs[nd.name], charmap) for nd in leaves}
        site, _, part, scale = ref_tree_lnl(m, rates, weights, tips, ops, lens, root_edge,
                                            root_len, n_nodes, return_partials=True)
        a, b = root_edge
        pa = np.moveaxis(part[a], 2, 1)   # [S][C][K]
        pb = np.moveaxis(part[b], 2, 1)
        pi = np.asarray(m.freqs)
        tl = np.array([root_len, 0.5 * root_len, 2.0 * root_len, 1e-4, 1.5])
        res = []
        for t in tl:
            probs3 = np.stack([np.stack([m.p(t * r), r * m.dp_dt(t * r),
                                         r * r * m.d2p_dt2(t * r)]) for r in rates])
            # f = sum_i pi_i a_i (P(t) b)_i: the root on a (P(0)) as tree_model.py:189-197
            per = ref_branch_derivs(probs3, pi, pb, pa, scale[b], scale[a])
            res.append(mixture_derivs(per, weights))
        res = np.stack(res)               # [n_t][S][3]
        assert np.allclose(res[0, :, 0], site, rtol=1e-12, atol=1e-10)
        names = sorted(seqs, key=lambda s: int(s[1:]))
        out.update({
            nm + "_seqs": np.stack([np.frombuffer(seqs[k].encode(), dtype=np.uint8)
                                    for k in names]),
            nm + "_tip_index": np.array([next(nd.idx for nd in leaves if nd.name == k)
                                         for k in names]),
            nm + "_ops": ops, nm + "_lens": lens, nm + "_root_edge": np.array(root_edge),
            nm + "_root_len": np.array(root_len), nm + "_n_nodes": np.array(n_nodes),
            nm + "_weights": weights, nm + "_t": tl, nm + "_site_derivs": res,
            nm + "_totals": res.sum(axis=1)})
    np.savez_compressed(os.path.join(HERE, "edges.npz"), **out)


def make_cfg5_small():
    """a reduced cfg5 -- several 100-taxon random trees evaluated on ONE
    alignment (2k DNA sites simulated on another tree), cfg2's GTR+G4, by the reference's
    engine through the tree_model.py driver."""
    rng = np.random.default_rng(20261018)
    m = SM.GTR(list(CFG2_RATES), list(CFG2_FREQS))
    rates = orc.ref_discrete_gamma(0.5, 4)
    weights = np.full(4, 0.25)
    true = random_tree(rng, 100)
    seqs = simulate(rng, true, m, rates, 2000, DNA)
    names = sorted(seqs, key=lambda s: int(s[1:]))
    out = {"seqs": np.stack([np.frombuffer(seqs[k].encode(), dtype=np.uint8) for k in names]),
           "rates": rates, "weights": weights}
    lnls = []
    for i in range(4):
        seed = random_tree(rng, 100)
        ops, lens, root_edge, root_len, n_nodes = schedule(seed)
        leaves = [nd for nd in postorder(seed) if not nd.children]
        tips = {nd.idx: charmap_partials(seqs[nd.name], CHARMAPS.dna_charmap) for nd in leaves}
        site, _ = ref_tree_lnl(m, rates, weights, tips, ops, lens, root_edge, root_len,
                               n_nodes)
        lnls.append(site.sum())
        out.update({"t%d_newick" % i: np.frombuffer(newick(seed).encode(), dtype=np.uint8),
                    "t%d_site_lnl" % i: site, "t%d_lnl" % i: np.array(site.sum())})
    out["lnl"] = np.array(lnls)
    np.savez_compressed(os.path.join(HERE, "cfg5_small.npz"), **out)


def main():
    if sys.argv[1:] == ["nonrev"]:  # python tests/golden/make_golden.py nonrev
        make_nonrev()
        return
    if sys.argv[1:] == ["band"]:  # python tests/golden/make_golden.py band
        make_clv_band()
        return
    if sys.argv[1:] == ["edges"]:  # python tests/golden/make_golden.py edges
        make_edges()
        make_cfg5_small()
        return
    rng = np.random.default_rng(20261015)
    make_gamma()
    make_models()
    make_clv(rng)
    make_clv_band()
    make_charmaps()
    make_pulley()
    make_trees(rng)
    make_nonrev()
    make_edges()
    make_cfg5_small()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
