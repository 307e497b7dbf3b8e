"""Synthetic workloads: random topologies and alignments simulated
under the configured model.  Used by bench.py and the GPU tests -- there is no
dataset download; every input is generated from a seeded numpy Generator.

* topology: random pairwise joining of N labelled tips, branch lengths
  ~ U(lo, hi); the final two subtrees hang from the seed.
* alignment: root state ~ pi, category ~ U{0..C-1} per site, each child drawn
  from the row of P(t * r_c) of its parent's state.  No gaps; patterns are not
  compressed (S = sites).
"""
from __future__ import annotations

import numpy as np

from .tree import Node, Tree

CFG2_GTR_RATES = [1.2, 3.5, 0.8, 1.1, 4.2, 1.0]  # AC AG AT CG CT GT
CFG2_FREQS = [0.30, 0.20, 0.25, 0.25]


def random_tree(rng, n_taxa, lo=0.01, hi=0.3):
    active = [Node("t%d" % i, rng.uniform(lo, hi)) for i in range(n_taxa)]
    while len(active) > 2:
        i, j = sorted(rng.choice(len(active), 2, replace=False))
        b, a = active.pop(j), active.pop(i)
        parent = Node(None, rng.uniform(lo, hi))
        parent.add(a)
        parent.add(b)
        active.append(parent)
    seed = Node()
    for n in active:
        seed.add(n)
    return Tree(seed)


def simulate_states(rng, tree, model, rates, n_sites):
    """{leaf label: int8 states [S]} simulated down `tree`."""
    K = len(model.freqs)
    C = len(rates)
    cats = rng.integers(0, C, n_sites)
    freqs = np.asarray(model.freqs, dtype=np.float64)
    root = rng.choice(K, n_sites, p=freqs / freqs.sum())
    out = {}
    stack = [(c, root) for c in tree.seed_node.children]
    while stack:
        node, parent_states = stack.pop()
        P = model.p(node.edge_length, rates)  # [C][K][K]
        # the row of (category, parent state) of every site, cumulated once per row -- the same
        # sums as cumulating the gathered rows, so the alignment is unchanged (r04: 3x faster)
        cum_rows = np.cumsum(P, axis=2).reshape(C * K, K)
        cum = np.take(cum_rows, cats * K + parent_states, axis=0)
        u = rng.random(n_sites)[:, None] * cum[:, -1:]
        st = np.minimum((u > cum).sum(axis=1), K - 1).astype(np.int8)
        if node.children:
            stack.extend((c, st) for c in node.children)
        else:
            out[node.label] = st
    return out


def make_problem(n_taxa, n_sites, model, rates, seed=0, lo=0.01, hi=0.3):
    """(tree, names [ntaxa], states int8 [ntaxa][S])."""
    rng = np.random.default_rng(seed)
    tree = random_tree(rng, n_taxa, lo, hi)
    st = simulate_states(rng, tree, model, rates, n_sites)
    names = sorted(st, key=lambda s: int(s[1:]))
    return tree, names, np.stack([st[n] for n in names])
