"""Shared loaders of tests/golden/edges.npz and cfg5_small.npz (generated from the reference by
tests/golden/make_golden.py: Model.dp_dt / d2p_dt2, python_likelihood_engine.lnl_branch_derivs
and its tree_model.py driver)."""
import numpy as np

from conftest import load_golden

from phylo_utils_amd import alignment as A
from phylo_utils_amd import substitution_models as SM
from phylo_utils_amd.synthetic import CFG2_FREQS, CFG2_GTR_RATES

UNREST = np.array([[0, 1.5, 3.0, 0.7], [1.1, 0, 0.9, 4.1], [2.6, 1.3, 0, 1.0],
                   [0.6, 3.7, 1.2, 0]])
MODELS = {"gtr": lambda: SM.GTR(CFG2_GTR_RATES, CFG2_FREQS), "lg": lambda: SM.LG(),
          "unrest": lambda: SM.Unrest(UNREST)}
TREES = {"tree_gtr": ("gtr", A.DNA), "tree_lg": ("lg", A.PROTEIN)}


def edges():
    return load_golden("edges")


def tree_problem(g, name):
    """(model, alphabet, tips {node: [S][K]}, ops, lens, root_edge, root_len, n_nodes, t,
    totals [n_t][3], site_derivs [n_t][S][3], rates, weights) of an edges.npz tree case."""
    mname, alpha = TREES[name]
    m = MODELS[mname]()
    seqs = ["".join(map(chr, r)) for r in g[name + "_seqs"]]
    tips = {int(n): A.seq_to_partials(s, alpha) for n, s in zip(g[name + "_tip_index"], seqs)}
    return dict(model=m, alpha=alpha, tips=tips, ops=g[name + "_ops"], lens=g[name + "_lens"],
                root_edge=tuple(int(x) for x in g[name + "_root_edge"]),
                root_len=float(g[name + "_root_len"]), n_nodes=int(g[name + "_n_nodes"]),
                t=g[name + "_t"], totals=g[name + "_totals"], site=g[name + "_site_derivs"],
                rates=g["rates"], weights=g[name + "_weights"], seqs=seqs)


def cfg5_small():
    g = load_golden("cfg5_small")
    seqs = ["".join(map(chr, r)) for r in g["seqs"]]
    trees = [bytes(g["t%d_newick" % i]).decode() for i in range(len(g["lnl"]))]
    return seqs, trees, g["lnl"], g["rates"], g["weights"]
