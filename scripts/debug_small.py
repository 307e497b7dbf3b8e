#!/usr/bin/env python
"""Small-tree GPU debugging: per-node partials of the device vs the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from phylo_utils_amd import TreeModel  # noqa: E402
from phylo_utils_amd import alignment as A  # noqa: E402
from phylo_utils_amd import substitution_models as SM  # noqa: E402
from phylo_utils_amd.rate_models import GammaRateModel  # noqa: E402
from phylo_utils_amd.synthetic import make_problem  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    ntax = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    nsites = int(sys.argv[2]) if len(sys.argv) > 2 else 70
    model = SM.K80(2.0)
    rm = GammaRateModel(4, 0.5)
    tree, names, states = make_problem(ntax, nsites, model, rm.rates, seed=3)
    tm = TreeModel()
    tm.set_alignment_codes(states.astype(np.uint8), np.eye(4), names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    lnl = tm.likelihood()
    tr = tm.traversal
    tips = {tr.names[n]: tm.alignment[i] for n, i in tm.names.items()}
    ev, el, iv = model.engine_eigen()
    ref = O.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                     tr.root_length(), ev, el, iv, model.freqs, rm.rates, rm.weights,
                     n_nodes=tr.n_nodes, return_all=True)
    print("lnl gpu %.10f oracle %.10f" % (lnl, ref["lnl"]))
    parts = tm.partials
    for (p, a, b) in tr.postorder_traversal:
        d = np.abs(parts[p] - ref["partials"][p]).max()
        print("node %3d <- (%3d, %3d)  max|diff| %.3e" % (p, a, b, d))


if __name__ == "__main__":
    main()


def hypotheses():
    """Which wrong combination did node 7 (CT op) compute?"""
    model = SM.K80(2.0)
    rm = GammaRateModel(4, 0.5)
    tree, names, states = make_problem(5, 70, model, rm.rates, seed=3)
    tm = TreeModel()
    tm.set_alignment_codes(states.astype(np.uint8), np.eye(4), names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(tree)
    tm.initialise()
    tm.likelihood()
    tr = tm.traversal
    tips = {tr.names[n]: tm.alignment[i] for n, i in tm.names.items()}
    ev, el, iv = model.engine_eigen()
    ref = O.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                     tr.root_length(), ev, el, iv, model.freqs, rm.rates, rm.weights,
                     n_nodes=tr.n_nodes, return_all=True)
    parts = tm.partials
    P = ref["P"]  # [op][2][C][K][K]
    ops = tr.postorder_traversal
    k = len(ops) - 1
    p, a, b = ops[k]
    va, vb = parts[a], parts[b]
    got = parts[p]

    def mv(Pm, v):  # [C][K][K] x [S][C][K]
        return np.einsum("cij,scj->sci", Pm, v)
    cands = {
        "correct": mv(P[k, 0], va) * mv(P[k, 1], vb),
        "b<-a": mv(P[k, 0], va) * mv(P[k, 1], va),
        "a<-b": mv(P[k, 0], vb) * mv(P[k, 1], vb),
        "P swapped": mv(P[k, 1], va) * mv(P[k, 0], vb),
        "b=0 vec": mv(P[k, 0], va) * 0,
    }
    for n, cnd in cands.items():
        print("%-10s %.3e" % (n, np.abs(cnd - got).max()))
    print("a", a, "b", b, "tip?", a in tm.names.values(), b in tm.names.values())


if __name__ == "__main__" and os.environ.get("HYP"):
    hypotheses()
