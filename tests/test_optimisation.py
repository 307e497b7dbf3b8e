"""phylo_utils_amd.optimisation (the phylo_utils.optimisation interface, reference
src/optimisation.pyx) against fixtures made by the reference's own compiled module
(tests/golden/make_golden_optim.py): the out triples, every abscissa the callables were
evaluated at, and the parameter transforms agree bit for bit."""
import os

import numpy as np
import pytest

from phylo_utils_amd import optimisation as opt

import optim_cases as oc

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "optimisation.npz"))


@pytest.mark.parametrize("i", range(len(oc.CASES)))
def test_brent_matches_reference(i):
    name, guess, lb, rb, tol = oc.CASES[i]
    f, _ = oc.FUNCS[name]
    g, xs = oc.traced(f)
    out = opt.brent_wrap(guess, lb, rb, g, tol)
    np.testing.assert_array_equal(np.array(xs), GOLD["brent_%d_fx" % i])
    np.testing.assert_array_equal(out, GOLD["brent_%d_out" % i])


@pytest.mark.parametrize("i", range(len(oc.CASES)))
def test_dbrent_matches_reference(i):
    name, guess, lb, rb, tol = oc.CASES[i]
    f, df = oc.FUNCS[name]
    g, xs = oc.traced(f)
    dg, dxs = oc.traced(df)
    out = opt.dbrent_wrap(guess, lb, rb, g, dg, tol)
    np.testing.assert_array_equal(np.array(xs), GOLD["dbrent_%d_fx" % i])
    np.testing.assert_array_equal(np.array(dxs), GOLD["dbrent_%d_dfx" % i])
    np.testing.assert_array_equal(out, GOLD["dbrent_%d_out" % i])


def test_minimisers_find_the_minimum():
    # (x - 2)^2 + 1; the reference argument order: brent_wrap(guess, lbracket, rbracket)
    # brackets [lbracket, guess] and starts at rbracket
    f, df = oc.FUNCS["quad"]
    out = opt.brent_wrap(5.0, 0.0, 1.0, f)
    assert abs(out[0] - 2.0) < 1e-7 and abs(out[1] - 1.0) < 1e-12
    out = opt.dbrent_wrap(5.0, 0.0, 1.0, f, df)
    assert abs(out[0] - 2.0) < 1e-7 and abs(out[1] - 1.0) < 1e-12


@pytest.mark.parametrize("i", range(len(oc.SIMPLEX)))
def test_simplex_transforms_match_reference(i):
    p = GOLD["simplex_%d_p" % i]
    th = opt.simplex_encode(p)
    np.testing.assert_array_equal(th, GOLD["simplex_%d_theta" % i])
    np.testing.assert_array_equal(opt.simplex_decode(th), GOLD["simplex_%d_back" % i])
    q = opt.transform_params(p)
    np.testing.assert_array_equal(q, GOLD["simplex_%d_q" % i])
    np.testing.assert_array_equal(opt.decode_params(q), GOLD["simplex_%d_decoded" % i])
    np.testing.assert_allclose(opt.decode_params(q), p, rtol=1e-12, atol=1e-15)


def test_quad_interp_matches_reference():
    got = np.array([opt.quad_interp(*a) for a in oc.QUAD])
    np.testing.assert_array_equal(got, GOLD["quad"])
    assert got[0] == 1.0
