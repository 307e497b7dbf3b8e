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


def check_band_case(g, k, out, cml, sw):
    """Compare clv / lnl_node outputs on the numba rule against a clv_band.npz case (the
    reference's python engine, which rescales in [2^-128, eps) where numba does not):
    representation-free quantities only -- each vector over its largest entry (1e-13), the
    log of that entry plus the scaler (1e-12 relative), lnl_node -- plus the numba rule
    itself: the band is left unscaled and an all-zero vector stays zero with no log added
    (the python engine yields NaN / -inf there)."""
    sa, sb, ref, ref_cml, band = (g[k + "_" + n] for n in ("sa", "sb", "out", "cml", "band"))
    zero = ~np.isfinite(ref_cml)
    assert zero.any() and band.any()
    assert np.all(out[zero] == 0.0) and np.array_equal(cml[zero], (sa + sb)[zero])
    nz = ~zero
    mo, mr = out.max(-1), ref.max(-1)
    np.testing.assert_allclose((out / np.where(mo > 0, mo, 1)[..., None])[nz],
                               (ref / mr[..., None])[nz], rtol=0, atol=1e-13, err_msg=k)
    np.testing.assert_allclose((np.log(mo) + cml)[nz], (np.log(mr) + ref_cml)[nz],
                               rtol=1e-12, atol=1e-12, err_msg=k)
    # numba_likelihood_engine.py:37-44: no rescale in the band; python: rescaled there
    assert np.array_equal(cml[band], (sa + sb)[band]), k
    assert np.all(ref_cml[band] != (sa + sb)[band]), k
    np.testing.assert_allclose(sw[nz], g[k + "_lnl_node"][nz], rtol=1e-13, atol=1e-12,
                               err_msg=k)
    assert np.all(np.isneginf(sw[zero]))


def band_tree(pre="tree"):
    """A tree case of clv_band.npz ("tree": GTR+G4, 120 taxa; "aatree": LG+G4, 40 taxa) in
    tree_case's format plus the reference's internal partials [n][S][C][K], scalers [n][S][C]
    and clades (comma-joined tip names)."""
    g = load_golden("clv_band")
    d = {k[len(pre) + 1:]: g[k] for k in g.files if k.startswith(pre + "_")}
    d["newick"] = bytes(d["newick"]).decode()
    d["seq_strings"] = ["".join(map(chr, row)) for row in d["seqs"]]
    return d


def check_partials_repr(got_p, got_s, ref_p, ref_s, tol=1e-12):
    """Partials vs the python engine's, free of the rescaling representation: each vector
    over its largest entry (absolute `tol`) and the log of that entry plus the scaler
    (relative `tol`).  Returns the number of vectors whose unscaled largest entry lies in
    [2^-128, eps) on the numba rule (`got`)."""
    mo, mr = got_p.max(-1), ref_p.max(-1)
    np.testing.assert_allclose(got_p / mo[..., None], ref_p / mr[..., None], rtol=0, atol=tol)
    np.testing.assert_allclose(np.log(mo) + got_s, np.log(mr) + ref_s, rtol=tol, atol=1e-12)
    return int(((mo >= 2.0 ** -128) & (mo < np.finfo(float).eps)).sum())


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
