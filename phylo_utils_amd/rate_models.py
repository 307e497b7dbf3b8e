"""Among-site rate variation: finite mixtures of rate categories.

The engine reads three things from a rate model -- ``rates`` (C multipliers of every
branch length), ``weights`` (the C mixture weights; ``log(weights)`` enters the per-site
logsumexp of ``tree_model.py:216``) and ``ncat`` -- and hands them to ``pu_set_model``.
Everything else here is parameter bookkeeping.

A model is described once, as a table of its parameters (name, validator) plus one
function from the parameter values to ``(rates, weights)``.  Assigning a parameter
validates it and recomputes the categories.  Observable behaviour follows
``phylo_utils/rate_models.py``: the class names and constructor arguments, the
``alpha`` / ``pinvar`` attributes, the ``ValueError`` messages, and equal-weight discrete
Gamma rates from the PAML routine (``rate_models.py:15-121``; the rates themselves come from
``pu_discrete_gamma``, bit-identical to ``src/c_discrete_gamma.c``).
"""
import numpy as np

from .discrete_gamma import discrete_gamma


def _pinvar_ok(p):
    if not 0 <= p < 1:
        raise ValueError("pinvar must be in the range [0, 1)")
    return p


def _alpha_ok(a):
    if not 0.001 <= a:
        raise ValueError("alpha must be greater than 0.001")
    return a


def _gamma(alpha, n):
    """n equal-weight discrete-Gamma(alpha, alpha) categories (mean rate 1)."""
    return discrete_gamma(alpha, n), np.full(n, 1.0 / n)


class RateModel(object):
    """Base: subclasses list their parameters in ``_PARAMS`` (name -> validator or None)
    and implement ``_categories(**params) -> (rates, weights)``."""

    _PARAMS = {}

    def __init__(self, **params):
        object.__setattr__(self, "_values", {})
        for name, value in params.items():
            self._values[name] = self._check(name, value)
        self._update()

    def _check(self, name, value):
        check = self._PARAMS[name]
        return check(value) if check else value

    def _update(self):
        r, w = self._categories(**self._values)
        object.__setattr__(self, "_cats", (np.asarray(r, dtype=np.float64),
                                           np.asarray(w, dtype=np.float64)))

    def __getattr__(self, name):
        values = self.__dict__.get("_values", {})
        if name in values:
            return values[name]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in self._PARAMS:
            self._values[name] = self._check(name, value)
            self._update()
        else:
            object.__setattr__(self, name, value)

    @property
    def rates(self):
        return self._cats[0]

    @property
    def weights(self):
        return self._cats[1]

    @property
    def ncat(self):
        return len(self._cats[0])

    def __repr__(self):
        args = ",".join("{}={}".format(k, v) for k, v in self._values.items())
        return "{}({})".format(type(self).__name__, args)

    def __str__(self):
        return "{}\nweights={}\nrates={}".format(repr(self), self.weights, self.rates)


class GammaRateModel(RateModel):
    """``ncat`` equal-weight discrete-Gamma categories (rate_models.py:15-37)."""

    _PARAMS = {"ncat_gamma": None, "alpha": float}

    def __init__(self, ncat, alpha=1.0):
        super().__init__(ncat_gamma=int(ncat), alpha=alpha)

    @staticmethod
    def _categories(ncat_gamma, alpha):
        return _gamma(alpha, ncat_gamma)

    def __repr__(self):
        return "GammaRateModel(ncat={},alpha={})".format(self.ncat, self.alpha)


class UniformRateModel(RateModel):
    """One category at rate 1 (rate_models.py:40-47)."""

    @staticmethod
    def _categories():
        return [1.0], [1.0]


class InvariantSitesModel(RateModel):
    """+I: an invariable class (rate 0, weight pinvar) and one variable class whose rate
    keeps the mean at 1 (rate_models.py:50-74)."""

    _PARAMS = {"pinvar": _pinvar_ok}

    def __init__(self, pinvar):
        super().__init__(pinvar=pinvar)

    @staticmethod
    def _categories(pinvar):
        return [0.0, 1.0 / (1.0 - pinvar)], [pinvar, 1.0 - pinvar]


class InvariantGammaModel(RateModel):
    """+I+G: the invariable class followed by ``n_gamma_cat`` Gamma classes sharing weight
    1 - pinvar, rates scaled by 1 / (1 - pinvar) (rate_models.py:77-121)."""

    _PARAMS = {"pinvar": _pinvar_ok, "n_gamma_cat": None, "alpha": _alpha_ok}

    def __init__(self, pinvar, n_gamma_cat, alpha=1.0):
        super().__init__(pinvar=pinvar, n_gamma_cat=int(n_gamma_cat), alpha=float(alpha))

    @staticmethod
    def _categories(pinvar, n_gamma_cat, alpha):
        g, gw = _gamma(alpha, n_gamma_cat)
        return (np.concatenate([[0.0], g / (1.0 - pinvar)]),
                np.concatenate([[pinvar], gw * (1.0 - pinvar)]))
