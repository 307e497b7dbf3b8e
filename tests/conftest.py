"""Test configuration.

Markers: ``gpu`` -- needs a real MI355X (run with ``-m gpu``); everything else runs
on the CPU container.  The oracle (``oracle/``) is test infrastructure and is
imported only here, in tests, in ``__graft_entry__.smoke`` and in bench.py's
cpu_baseline leg.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def golden_charmap(kind):
    g = load_golden("charmaps")
    return {chr(c): v for c, v in zip(g[kind + "_chars"], g[kind + "_vectors"])}


def tree_case(name):
    """Decoded golden tree case: dict with tips {node: [S][K]}, schedule, model params."""
    g = load_golden("trees")
    d = {k[len(name) + 1:]: g[k] for k in g.files if k.startswith(name + "_")}
    d["newick"] = bytes(d["newick"]).decode()
    seqs = ["".join(map(chr, row)) for row in d["seqs"]]
    d["seq_strings"] = seqs
    return d


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as orc
    orc.build()
    return orc


def has_gpu():
    try:
        from phylo_utils_amd import _native as N
        return N.device_count() > 0
    except Exception:
        return False
