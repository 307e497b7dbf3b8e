"""Among-site rate variation models (mirror of ``phylo_utils/rate_models.py``).

The engine consumes only ``rates`` and ``weights`` (``pu_set_model``); P(t*r) is
built per category on the GPU and the per-category site likelihoods are
combined with ``log(weights)`` exactly as ``tree_model.py:216`` does.
"""
import numpy as np

from .discrete_gamma import discrete_gamma


class RateModel(object):
    @property
    def weights(self):
        return self._weights

    @property
    def rates(self):
        return self._rates


class GammaRateModel(RateModel):
    """Equal-weight discrete gamma (rate_models.py:15-37)."""

    def __init__(self, ncat, alpha=1.0):
        self.ncat = ncat
        self.alpha = float(alpha)
        self._weights = np.array([1.0 / ncat] * ncat)

    def __repr__(self):
        return "GammaRateModel(ncat={},alpha={})".format(self.ncat, self.alpha)

    def __str__(self):
        return "\n".join([self.__repr__(), "weights={}".format(self.weights),
                          "rates={}".format(self.rates)])

    @property
    def alpha(self):
        return self._alpha

    @alpha.setter
    def alpha(self, alpha):
        self._alpha = alpha
        self._rates = discrete_gamma(alpha, self.ncat)


class UniformRateModel(RateModel):
    """Single category, rate 1 (rate_models.py:40-47)."""

    def __init__(self):
        self.ncat = 1
        self._weights = np.array([1.0])
        self._rates = np.array([1.0])

    def __repr__(self):
        return "UniformRateModel()"


class InvariantSitesModel(RateModel):
    """Proportion of invariable sites (rate_models.py:50-74)."""

    def __init__(self, pinvar):
        self.pinvar = pinvar
        self.ncat = 2

    def __repr__(self):
        return "InvariantSitesModel(pinvar={})".format(self.pinvar)

    @property
    def pinvar(self):
        return self._pinvar

    @pinvar.setter
    def pinvar(self, pinvar):
        if not 0 <= pinvar < 1:
            raise ValueError("pinvar must be in the range [0, 1)")
        self._pinvar = pinvar
        self._weights = np.array([pinvar, 1 - pinvar])
        self._rates = np.array([0, 1 / (1 - pinvar)])


class InvariantGammaModel(RateModel):
    """+I+G (rate_models.py:77-121)."""

    def __init__(self, pinvar, n_gamma_cat, alpha=1.0):
        if not 0 <= pinvar < 1:
            raise ValueError("pinvar must be in the range [0, 1)")
        if not 0.001 <= alpha:
            raise ValueError("alpha must be greater than 0.001")
        self.ncat = n_gamma_cat + 1
        self._pinvar = pinvar
        self._alpha = float(alpha)
        self._rates, self._weights = self._compute(pinvar, n_gamma_cat, alpha)

    @staticmethod
    def _compute(pinvar, ncat, alpha):
        g = discrete_gamma(alpha, ncat)
        rates = np.hstack([0, g / (1 - pinvar)])
        weights = np.hstack([pinvar, np.ones(ncat) / ncat * (1 - pinvar)])
        return rates, weights

    @property
    def alpha(self):
        return self._alpha

    @alpha.setter
    def alpha(self, alpha):
        if not 0.001 <= alpha:
            raise ValueError("alpha must be greater than 0.001")
        self._alpha = alpha
        self._rates, self._weights = self._compute(self.pinvar, self.ncat - 1, alpha)

    @property
    def pinvar(self):
        return self._pinvar

    @pinvar.setter
    def pinvar(self, pinvar):
        if not 0 <= pinvar < 1:
            raise ValueError("pinvar must be in the range [0, 1)")
        self._pinvar = pinvar
        self._rates, self._weights = self._compute(pinvar, self.ncat - 1, self.alpha)
