"""Trees and the flattened post-order schedule (no dendropy).

Mirrors the parts of ``phylo_utils/traversal.py`` and ``phylo_utils/utils.py``
the likelihood path uses:

* ``parse_newick`` -- a small Newick reader (labels, ``:lengths``, quoted labels,
  comments ``[...]`` skipped).
* ``deroot`` / ``resolve_polytomies`` -- ``deepcopy_tree`` (``utils.py:114-118``):
  a bifurcating seed loses one internal child (the second child if it is
  internal, else the first), whose edge length moves to its sister; nodes with
  more than two children keep the first child and hang the rest below new
  zero-length nodes.
* ``Traversal`` (``traversal.py:6-35``): non-seed nodes indexed in post-order
  (leaves included), ``names`` {leaf label: index}, ``root_edge`` = the seed's
  two children, ``brlens`` keyed by the sorted index pair with the seed's
  children joined by ``max`` of their lengths (``utils.py:202-213``), and
  ``postorder_traversal`` int32 [N-2][3] of (parent, child1, child2)
  (``utils.py:127-134``), and ``optimising_traversal`` int32 [3N-5][5]
  (``utils.py:137-188``, ``traversal.py:29,34-35``).
"""
from __future__ import annotations

import numpy as np


class Node(object):
    __slots__ = ("children", "parent", "length", "label")

    def __init__(self, label=None, length=None):
        self.children = []
        self.parent = None
        self.length = length
        self.label = label

    def add(self, child):
        child.parent = self
        self.children.append(child)
        return child

    def is_leaf(self):
        return not self.children

    @property
    def edge_length(self):
        return 0.0 if self.length is None else self.length

    def postorder(self):
        """Iterative post-order (deep caterpillars exceed Python's recursion limit)."""
        out, stack = [], [(self, False)]
        while stack:
            n, done = stack.pop()
            if done or not n.children:
                out.append(n)
                continue
            stack.append((n, True))
            for c in reversed(n.children):
                stack.append((c, False))
        return out

    def leaves(self):
        return [n for n in self.postorder() if n.is_leaf()]


class Tree(object):
    def __init__(self, seed):
        self.seed_node = seed

    def postorder_node_iter(self):
        return iter(self.seed_node.postorder())

    def leaf_nodes(self):
        return self.seed_node.leaves()

    def copy(self):
        return Tree(_copy(self.seed_node))

    def as_newick(self):
        return _write(self.seed_node) + ";"

    def deroot(self):
        """Collapse a basal bifurcation into a trifurcation (dendropy deroot semantics)."""
        seed = self.seed_node
        if len(seed.children) != 2:
            return self
        a, b = seed.children
        if len(b.children) >= 2:
            keep, drop = a, b
        elif len(a.children) >= 2:
            keep, drop = b, a
        else:
            return self
        keep.length = keep.edge_length + drop.edge_length
        pos = seed.children.index(drop)
        for c in drop.children:
            c.parent = seed
        seed.children[pos:pos + 1] = drop.children
        return self

    def resolve_polytomies(self):
        """Binary everywhere: first child stays, the others go below new 0-length nodes."""
        for n in self.seed_node.postorder():
            while len(n.children) > 2:
                rest = n.children[1:]
                n.children = n.children[:1]
                new = n.add(Node(length=0.0))
                for c in rest:
                    new.add(c)
                n = new
        return self


def _copy(node):
    new = Node(node.label, node.length)
    stack = [(node, new)]
    while stack:
        src, dst = stack.pop()
        for c in src.children:
            d = dst.add(Node(c.label, c.length))
            stack.append((c, d))
    return new


def _write(node):
    def lab(n):
        s = ""
        if n.label is not None:
            s = n.label if all(ch not in n.label for ch in " (),:;[]'") else \
                "'" + n.label.replace("'", "''") + "'"
        if n.length is not None and n is not node:
            s += ":" + repr(float(n.length))
        return s

    # iterative writer
    parts = {}
    for n in node.postorder():
        if n.children:
            parts[id(n)] = "(" + ",".join(parts.pop(id(c)) for c in n.children) + ")" + lab(n)
        else:
            parts[id(n)] = lab(n)
    return parts[id(node)]


def parse_newick(text):
    """Newick string -> Tree (rooted as written)."""
    s = text.strip()
    i, n = 0, len(s)
    root = Node()
    cur = root
    stack = []
    expect_child = True

    def read_label(i):
        if i < n and s[i] == "'":
            j = i + 1
            buf = []
            while j < n:
                if s[j] == "'":
                    if j + 1 < n and s[j + 1] == "'":
                        buf.append("'")
                        j += 2
                        continue
                    break
                buf.append(s[j])
                j += 1
            return "".join(buf), j + 1
        j = i
        while j < n and s[j] not in "(),:;[":
            j += 1
        lab = s[i:j].strip()
        return (lab if lab else None), j

    def read_length(i):
        j = i
        while j < n and s[j] not in "(),;[":
            j += 1
        return float(s[i:j]), j

    started = False
    while i < n:
        ch = s[i]
        if ch.isspace():
            i += 1
        elif ch == "[":
            j = s.find("]", i)
            if j < 0:
                raise ValueError("unterminated comment in newick")
            i = j + 1
        elif ch == "(":
            if not started:
                started = True
                stack.append(root)
                cur = root
            else:
                child = cur.add(Node())
                stack.append(child)
                cur = child
            expect_child = True
            i += 1
        elif ch == ",":
            if not stack:
                raise ValueError("unbalanced ',' in newick")
            cur = stack[-1]
            expect_child = True
            i += 1
        elif ch == ")":
            if not stack:
                raise ValueError("unbalanced ')' in newick")
            cur = stack.pop()
            expect_child = False
            i += 1
            lab, i = read_label(i)
            cur.label = lab if lab is not None else cur.label
        elif ch == ":":
            i += 1
            cur.length, i = read_length(i)
        elif ch == ";":
            break
        else:
            if not started:  # single leaf tree
                started = True
            lab, i = read_label(i)
            if expect_child and stack:
                cur = stack[-1].add(Node(lab))
            else:
                cur.label = lab
            expect_child = False
    if stack:
        raise ValueError("unbalanced parentheses in newick")
    return Tree(root)


def prepare_tree(tree):
    """deepcopy_tree (utils.py:114-118): copy, deroot, resolve polytomies."""
    if isinstance(tree, str):
        tree = parse_newick(tree)
    return tree.copy().deroot().resolve_polytomies()


class BranchLengths(dict):
    """Length lookup by unordered node-index pair (utils.py:191-199)."""

    def __getitem__(self, key):
        val = self.get(key)
        if val is None:
            val = self.get(tuple(key)[::-1])
        if val is None:
            raise KeyError(key)
        return val


def optimising_traversal(seed, node_dict):
    """get_optimising_traversal (utils.py:137-188): 3N-5 rows of 5 node indices.

    Row 0 is (-1, -1, -1, LEFT, RIGHT): optimise the root edge.  Then, depth first from
    LEFT and from RIGHT, every other node NOD with parent PAR, sibling SIB and
    grandparent GPA (the other root-edge end when PAR is LEFT or RIGHT) adds
    (PAR, SIB, GPA, NOD, PAR) -- re-orient PAR's partials towards NOD from SIB and GPA,
    then optimise edge (NOD, PAR) -- and, after its children, an internal NOD adds
    (NOD, CH1, CH2, -1, -1), restoring its post-order partials.  Iterative (a
    1000-taxon caterpillar is deeper than Python's recursion limit).
    """
    left, right = seed.children
    rows = [(-1, -1, -1, node_dict[left], node_dict[right])]
    for start in (left, right):
        stack = [(start, False)]
        while stack:
            node, done = stack.pop()
            nod = node_dict[node]
            if done:
                ch1, ch2 = node.children
                rows.append((nod, node_dict[ch1], node_dict[ch2], -1, -1))
                continue
            if node is not left and node is not right:
                par = node.parent
                gpa = right if par is left else (left if par is right else par.parent)
                sib = next(c for c in par.children if c is not node)  # utils.get_sibling
                rows.append((node_dict[par], node_dict[sib], node_dict[gpa], nod,
                             node_dict[par]))
            if node.children:
                ch1, ch2 = node.children
                stack.append((node, True))
                stack.append((ch2, False))
                stack.append((ch1, False))
    return np.array(rows, dtype=np.int32).reshape(-1, 5)


class Traversal(object):
    """Node indexing + post-order schedule for the engine (traversal.py:6-35)."""

    def __init__(self, tree):
        seed = tree.seed_node
        order = [n for n in seed.postorder() if n is not seed]
        self.node_dict = {n: i for i, n in enumerate(order)}
        self.names = {}
        for n in order:
            if n.is_leaf():
                if n.label is None:
                    raise ValueError("unlabelled leaf in tree")
                if n.label in self.names:
                    raise ValueError("duplicate leaf label %r" % n.label)
                self.names[n.label] = self.node_dict[n]
        if len(seed.children) != 2:
            raise ValueError("seed node must have two children after resolution")
        self.n_nodes = len(order)
        self.root_edge = tuple(self.node_dict[c] for c in seed.children)
        self.brlens = BranchLengths()
        for n in order:
            if n.parent is seed:
                nb = [c for c in seed.children if c is not n][0]
                length = max(c.edge_length for c in seed.children)
            else:
                nb = n.parent
                length = n.edge_length
            self.brlens[tuple(sorted((self.node_dict[n], self.node_dict[nb])))] = length
        ops = [(self.node_dict[n], self.node_dict[n.children[0]], self.node_dict[n.children[1]])
               for n in order if n.children]
        self.postorder_traversal = np.array(ops, dtype=np.int32).reshape(-1, 3)
        self.optimising_traversal = optimising_traversal(seed, self.node_dict)

    def op_lengths(self):
        """[n_ops][2] lengths of (parent, child1), (parent, child2) for pu_set_schedule."""
        return np.array([[self.brlens[(p, a)], self.brlens[(p, b)]]
                         for p, a, b in self.postorder_traversal], dtype=np.float64).reshape(-1, 2)

    def root_length(self):
        return float(self.brlens[self.root_edge])
