"""Test functions and argument sets for the 1-D optimisers (phylo_utils_amd/optimisation.py
vs the reference's src/optimisation.pyx).  Shared by tests/golden/make_golden_optim.py
(which ran them through the reference's compiled module) and tests/test_optimisation.py."""
import math

import numpy as np


def _jc_pair(n_same, n_diff):
    """-lnL of a two-sequence JC69 distance: the shape of a branch-length problem."""
    def f(t):
        e = math.exp(-4.0 * t / 3.0)
        return -(n_same * math.log(0.25 + 0.75 * e) + n_diff * math.log(0.25 - 0.25 * e))

    def df(t):
        e = math.exp(-4.0 * t / 3.0)
        de = -4.0 / 3.0 * e
        return -(n_same * 0.75 * de / (0.25 + 0.75 * e) - n_diff * 0.25 * de / (0.25 - 0.25 * e))
    return f, df


FUNCS = {
    "quad": (lambda x: (x - 2.0) ** 2 + 1.0, lambda x: 2.0 * (x - 2.0)),
    "quartic": (lambda x: x ** 4 - 3.0 * x ** 3 + 2.0, lambda x: 4.0 * x ** 3 - 9.0 * x ** 2),
    "expx": (lambda x: math.exp(x) - 2.0 * x, lambda x: math.exp(x) - 2.0),
    "jc": _jc_pair(80, 20),
    "jc_close": _jc_pair(997, 3),
    "wavy": (lambda x: abs(x - 1.0) ** 1.5 + 0.1 * math.sin(5.0 * x),
             lambda x: 1.5 * math.copysign(abs(x - 1.0) ** 0.5, x - 1.0) + 0.5 * math.cos(5.0 * x)),
    "flat": (lambda x: 1.0, lambda x: 0.0),
}

# (function, guess, lbracket, rbracket, tol) -- the *_wrap argument order of the reference
CASES = [
    ("quad", 1.0, 0.0, 5.0, 1.5e-8),
    ("quad", 3.0, -1.0, 4.0, 1e-12),
    ("quad", 0.5, 0.0, 1.0, 1.5e-8),     # bracket [0, guess] excludes the minimum
    ("quartic", 2.0, 1.0, 4.0, 1.5e-8),
    ("quartic", 3.5, 0.5, 2.5, 1e-6),
    ("expx", 0.2, -2.0, 3.0, 1.5e-8),
    ("jc", 0.1, 1e-5, 10.0, 1.5e-8),
    ("jc", 5.0, 1e-5, 0.3, 1.5e-8),
    ("jc_close", 0.01, 1e-8, 2.0, 1.5e-8),
    ("jc_close", 1.0, 1e-8, 0.001, 1e-10),
    ("wavy", 0.7, -1.0, 3.0, 1.5e-8),
    ("wavy", 2.0, 0.0, 1.2, 1e-4),
    ("flat", 0.3, 0.0, 1.0, 1.5e-8),
]

SIMPLEX = [
    np.array([0.25, 0.25, 0.25, 0.25]),
    np.array([0.1, 0.2, 0.3, 0.4]),
    np.array([0.30, 0.20, 0.25, 0.25]),
    np.array([0.7, 0.3]),
    np.random.default_rng(7).dirichlet(np.ones(20)),
]

QUAD = [
    (0.0, 1.0, 2.0, 1.0, 0.0, 1.0),
    (0.1, 0.5, 0.9, 3.0, 1.0, 2.5),
    (1.0, 2.0, 3.0, 5.0, 5.0, 5.0),            # collinear: divisor clamped to TINY
    (-1.0, 0.5, 4.0, 2.0, -1.0, 7.0),
]


def traced(f):
    """f wrapped to record every abscissa it is called at."""
    xs = []

    def g(x):
        xs.append(float(x))
        return f(x)
    return g, xs
