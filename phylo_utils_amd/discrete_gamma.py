"""Discrete-gamma rate categories -- drop-in for ``phylo_utils.discrete_gamma``.

``discrete_gamma(alpha, ncat, median_rates=False)`` has the reference's signature
and meaning (``src/discrete_gamma.pyx:30-47``: mean rates of ``ncat`` equal-
probability categories of Gamma(alpha, alpha), or rescaled medians).  It runs
the host C++ routine ``pu_discrete_gamma`` in libphylo_hip.so, which follows the
same published algorithms as PAML's ``DiscreteGamma`` and reproduces the
reference's rates bit for bit (tests/test_host.py::test_discrete_gamma_bitwise_equal_to_paml).  Do not substitute scipy:
its rates differ from the reference's by up to 8.4e-9 relative.
"""
import numpy as np

from . import _native as N


def discrete_gamma(alpha, ncat, median_rates=False):
    """Rates for a ``ncat``-category discrete gamma with shape ``alpha`` (mean 1).

    >>> discrete_gamma(0.5, 5)  # doctest: +SKIP
    array([0.02121238, 0.15548577, 0.46708288, 1.10711735, 3.24910162])
    """
    ncat = int(ncat)
    if ncat < 1:
        raise ValueError("ncat must be >= 1")
    rates = np.zeros(ncat, dtype=np.float64)
    N.check(N.lib().pu_discrete_gamma(float(alpha), ncat, int(bool(median_rates)),
                                      N.ptr(rates)), what="pu_discrete_gamma")
    return rates
