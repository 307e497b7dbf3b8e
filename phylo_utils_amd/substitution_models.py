"""Substitution models: Q matrices, eigen-decompositions and P(t) (host, numpy).

Mirrors ``phylo_utils.substitution_models`` (``substitution_models/abstract.py``,
``utils.py`` and the per-model files): same class names, constructor arguments,
``p(t, rates)`` stacking (``abstract.py:49-59``), Q scaling to one expected
substitution per unit time (``utils.py:45-65``) and the symmetric ``B``-matrix
eigen-decomposition of reversible models (``utils.py:82-98``).  The engine only
consumes ``(evecs, evals, ivecs, freqs)`` -- P(t) for every branch and rate is
computed on the GPU from those (``pu_set_model`` / ``k_pmatrix``).

Differences from the reference, deliberate:
  * ``JC69.p(t, rates=None)`` also accepts ``rates`` (the reference's
    ``jc69.py:39`` takes only ``t``, so JC69 cannot drive its TreeModel -- SURVEY
    0.4); with ``rates=None`` it is the reference's closed form.
  * Every model carries an eigen-decomposition usable by the engine; the TN93
    family uses the generic B-matrix route (P agrees to ~1e-15 with the
    reference's closed-form eigenvectors, tests/test_models.py).
"""
from __future__ import annotations

import numpy as np

from . import data

MIN_BRANCH_LENGTH = 1 / 2 ** 16  # abstract.py:8 (unused by the likelihood path)
SMALL = 1 / 2 ** 128             # utils.py:3


# ----------------------------------------------------------------- helpers (utils.py)
def compute_b_matrix(q_matrix, sqrtfreqs):
    """B = diag(sqrt pi) Q diag(1/sqrt pi): symmetric when Q is reversible (utils.py:5-12)."""
    return (sqrtfreqs[:, None] * q_matrix) / sqrtfreqs[None, :]


def check_frequencies(freqs, length):
    """utils.py:15-23: right length, non-negative, sums to one (rtol 1e-16)."""
    freqs = np.ascontiguousarray(freqs, dtype=np.float64)
    if len(freqs) != length:
        raise ValueError("Frequencies vector is not the right length (length={})".format(len(freqs)))
    if np.min(freqs) < 0:
        raise ValueError("Frequencies vector contains negative values")
    if not np.allclose(sum(freqs), 1.0, rtol=1e-16):
        raise ValueError("Frequencies do not add to 1.0 within tolerance (sum={})".format(sum(freqs)))
    return freqs


def check_rates(rates, size, symmetry=True):
    """utils.py:26-34: square (size x size), non-negative, symmetric if reversible."""
    rates = np.ascontiguousarray(rates, dtype=np.float64)
    if rates.shape != (size, size):
        raise ValueError("Rate matrix is not the right shape (length={})".format(rates.shape))
    if np.min(rates) < 0:
        raise ValueError("Rate matrix contains negative values")
    if symmetry and not np.allclose(rates, rates.T):
        raise ValueError("Rate matrix is not symmetrical")
    return rates


def q_to_freqs(q_matrix):
    """Stationary distribution: solve Q^T pi = 0 with sum(pi) = 1 (utils.py:68-79)."""
    n = q_matrix.shape[0]
    a = np.vstack([np.ones(n), q_matrix.T])
    b = np.zeros(n + 1)
    b[0] = 1.0
    pi, _, _, _ = np.linalg.lstsq(a, b, rcond=None)
    return pi


def compute_q_matrix(rates, freqs, scale=True):
    """Q = R diag(pi), rows summing to zero, scaled so -sum_i pi_i q_ii = 1 (utils.py:45-65)."""
    q = np.array(rates, dtype=np.float64) if freqs is None else rates * np.asarray(freqs)[None, :]
    n = q.shape[0]
    q[np.diag_indices(n)] -= q.sum(axis=1)
    if scale:
        f = q_to_freqs(q) if freqs is None else freqs
        q = q / (-np.diag(q).dot(f))
    return q


def get_eigen(q_matrix, freqs=None):
    """(evecs, evals, ivecs) with Q = evecs diag(evals) ivecs (utils.py:82-98)."""
    if freqs is not None:
        rootf = np.sqrt(freqs)
        evals, r = np.linalg.eigh(compute_b_matrix(q_matrix, rootf))
        evecs = r / rootf[:, None]
        ivecs = r.T * rootf[None, :]
    else:
        evals, evecs = np.linalg.eig(q_matrix)
        order = np.argsort(evals)
        evals = evals[order]
        evecs = evecs[:, order]
        ivecs = np.linalg.inv(evecs)
    return (np.ascontiguousarray(evecs), np.ascontiguousarray(evals),
            np.ascontiguousarray(ivecs))


def expm(matrix, squarings=8):
    """Taylor(4) scaling-and-squaring exponential used for non-reversible Q (utils.py:101-116)."""
    p = matrix / 2 ** squarings
    p2 = p.dot(p)
    p3 = p.dot(p2)
    p4 = p.dot(p3)
    e = np.eye(p.shape[0]) + p + p2 / 2.0 + p3 / 6.0 + p4 / 24.0
    for _ in range(squarings):
        e = e.dot(e)
    return e


# ----------------------------------------------------------------- eigen / base classes
class Eigen(object):
    """evecs diag(f(evals)) ivecs (abstract.py:88-122)."""
    __slots__ = ("evecs", "evals", "ivecs")

    def __init__(self, evecs, evals, ivecs):
        self.evecs = evecs
        self.evals = evals
        self.ivecs = ivecs

    @property
    def values(self):
        return self.evecs, self.evals, self.ivecs

    def exp(self, t=1.0):
        return (self.evecs * np.exp(self.evals * t)).dot(self.ivecs)

    def reconstitute(self):
        return (self.evecs * self.evals).dot(self.ivecs)

    def fn_apply(self, fn):
        return (self.evecs * fn(self.evals)).dot(self.ivecs)


class Model(object):
    """Common interface (abstract.py:11-85)."""
    _name = None
    _rates = None
    _freqs = None
    _size = None
    _states = None
    reversible = True

    def __init__(self):
        self.eigen = None
        self._q_mtx = None

    name = property(lambda self: self._name)
    rates = property(lambda self: self._rates)
    freqs = property(lambda self: self._freqs)
    size = property(lambda self: self._size)
    states = property(lambda self: self._states)

    def q(self):
        return self._q_mtx

    def b(self):
        return compute_b_matrix(self.q(), np.sqrt(self.freqs))

    def p(self, t, rates=None):
        """P(t), or stacked [P(t*r) for r in rates] along axis 0 (abstract.py:49-59)."""
        if rates is None:
            return self.eigen.exp(t)
        return np.stack([self.eigen.exp(t * r) for r in rates], axis=0)

    def dp_dt(self, t, rates=None):
        if rates is None:
            return self.eigen.fn_apply(lambda x: x * np.exp(x * t))
        return np.stack([self.eigen.fn_apply(lambda x: x * np.exp(x * t * r)) for r in rates])

    def d2p_dt2(self, t, rates=None):
        if rates is None:
            return self.eigen.fn_apply(lambda x: x * x * np.exp(x * t))
        return np.stack([self.eigen.fn_apply(lambda x: x * x * np.exp(x * t * r))
                         for r in rates])

    def p_derivative(self, t, rates, order):
        """d^order/dt^order P(t r) for each rate r, stacked [C][K][K] (order 0, 1, 2).  The
        chain-rule factor r that dp_dt / d2p_dt2 (abstract.py:61-77, 180-192) leave out is
        applied here: this is what the engine's edge derivatives differentiate.  Order 0 is
        exactly p(t, rates)."""
        rates = np.asarray(rates, dtype=np.float64)
        if order == 0:
            return np.asarray(self.p(t, rates))
        if order == 1:
            return np.asarray(self.dp_dt(t, rates)) * rates[:, None, None]
        if order == 2:
            return np.asarray(self.d2p_dt2(t, rates)) * (rates * rates)[:, None, None]
        raise ValueError("order must be 0, 1 or 2")

    def detailed_balance(self):
        """pi_i q_ij == pi_j q_ji (abstract.py:79-85)."""
        m = self.q().T * self.freqs
        return np.allclose(m, m.T)

    def engine_eigen(self):
        """(evecs, evals, ivecs) as C-contiguous fp64 for pu_set_model."""
        if not self.reversible:
            raise NotImplementedError("%s is not reversible: its likelihood depends on the root "
                                      "placement and it has no real eigen-decomposition "
                                      "(out of scope, DESIGN.md)" % self._name)
        ev, el, iv = self.eigen.values
        return (np.ascontiguousarray(ev, dtype=np.float64),
                np.ascontiguousarray(el, dtype=np.float64),
                np.ascontiguousarray(iv, dtype=np.float64))


class ProteinModel(Model):
    _name = "GenericProtein"
    _size = 20
    _states = list(data.PROTEIN_STATES)

    def __init__(self, rates, freqs, default_freqs=None):
        Model.__init__(self)
        self._rates = check_rates(rates, self.size)
        # the published frequency vectors are used as stored, unchecked (lg.py:10-14);
        # Dayhoff's sum to 1.000001
        self._freqs = (np.array(default_freqs, dtype=np.float64) if freqs is None
                       else check_frequencies(freqs, self.size))
        self._q_mtx = compute_q_matrix(self._rates, self._freqs)
        self.eigen = Eigen(*get_eigen(self._q_mtx, self._freqs))

    def __repr__(self):
        return "Protein model: {}\nFreqs:        {}\n".format(self._name, self._freqs)


class DNAReversibleModel(Model):
    _name = "GenericReversibleDNA"
    _size = 4
    _states = list(data.DNA_STATES)

    def _build(self, rates, freqs, scale_q=True):
        Model.__init__(self)
        self._rates = check_rates(rates, 4)
        self._freqs = check_frequencies(freqs, 4)
        self._q_mtx = compute_q_matrix(self._rates, self._freqs, scale_q)
        self.eigen = Eigen(*get_eigen(self._q_mtx, self._freqs))

    def __repr__(self):
        iu = (np.array([0, 0, 0, 1, 1, 2]), np.array([1, 2, 3, 2, 3, 3]))
        return "DNA reversible model: {}\nRel. rates: {}\nFreqs:      {}\n".format(
            self._name, self._rates[iu], self._freqs)


class DNANonReversibleModel(Model):
    _name = "GenericNonReversibleDNA"
    _size = 4
    _states = list(data.DNA_STATES)
    reversible = False

    def p(self, t, rates=None):
        q = self.q()
        if rates is None:
            return expm(q * t)
        return np.stack([expm(q * r * t) for r in rates], axis=0)

    def dp_dt(self, t, rates=None):
        q = self.q()
        if rates is None:
            return q.dot(expm(q * t))
        return np.stack([q.dot(expm(q * r * t)) for r in rates], axis=0)

    def d2p_dt2(self, t, rates=None):
        q = self.q()
        if rates is None:
            return q.dot(q).dot(expm(q * t))
        return np.stack([q.dot(q).dot(expm(q * r * t)) for r in rates], axis=0)


# ----------------------------------------------------------------- DNA models
_UPPER = (np.array([0, 0, 0, 1, 1, 2]), np.array([1, 2, 3, 2, 3, 3]))


def _sym_from_upper(vals):
    m = np.zeros((4, 4))
    m[_UPPER] = vals
    m[_UPPER[::-1]] = vals
    return m


class GTR(DNAReversibleModel):
    """General time-reversible (gtr.py:9-46); rates as 5 or 6 values (AC AG AT CG CT [GT=1])
    or a symmetric 4x4 matrix."""
    _name = "GTR"

    def __init__(self, rates=None, freqs=None, scale_q=True):
        if rates is None:
            rates = data.fixed_equal_nucleotide_rates.copy()
        else:
            r = np.asarray(rates, dtype=np.float64)
            if r.ndim == 1:
                if len(r) == 5:
                    r = np.append(r, 1.0)
                if len(r) != 6:
                    raise ValueError("GTR needs 5 or 6 exchangeabilities or a 4x4 matrix")
                r = _sym_from_upper(r)
            rates = r
        if freqs is None:
            freqs = data.fixed_equal_nucleotide_frequencies.copy()
        self._build(rates, freqs, scale_q)

    @staticmethod
    def square_matrix(uppertri):
        return _sym_from_upper(np.asarray(uppertri, dtype=np.float64))


class TN93(DNAReversibleModel):
    """Tamura-Nei: transitions alpha_y (C<->T), alpha_r (A<->G), transversions beta (tn93.py:59-82)."""
    _name = "TN93"

    def __init__(self, alpha_y, alpha_r, beta=1.0, freqs=None, scale_q=True):
        if freqs is None:
            freqs = data.fixed_equal_nucleotide_frequencies.copy()
        ay, ar, b = float(alpha_y), float(alpha_r), float(beta)
        self._alpha_y, self._alpha_r, self._beta = ay, ar, b
        self._build(np.array([[0, b, ar, b], [b, 0, b, ay], [ar, b, 0, b], [b, ay, b, 0]]),
                    freqs, scale_q)


class K80(TN93):
    """Kimura 2-parameter, equal frequencies (k80.py)."""
    _name = "K80"

    def __init__(self, kappa, scale_q=True):
        TN93.__init__(self, kappa, kappa, 1, data.fixed_equal_nucleotide_frequencies.copy(),
                      scale_q=scale_q)


class F81(TN93):
    _name = "F81"

    def __init__(self, freqs, scale_q=True):
        TN93.__init__(self, 1, 1, 1, freqs, scale_q=scale_q)


class F84(TN93):
    _name = "F84"

    def __init__(self, kappa, freqs, scale_q=True):
        ay = 1 + kappa / (freqs[1] + freqs[3])
        ar = 1 + kappa / (freqs[0] + freqs[2])
        TN93.__init__(self, ay, ar, 1, freqs, scale_q=scale_q)


class HKY85(TN93):
    _name = "HKY85"

    def __init__(self, kappa, freqs, scale_q=True):
        TN93.__init__(self, kappa, kappa, 1, freqs, scale_q=scale_q)


class JC69(DNAReversibleModel):
    """Jukes-Cantor (jc69.py:26-45): equal rates and frequencies."""
    _name = "JC69"

    def __init__(self):
        self._build(data.fixed_equal_nucleotide_rates.copy(),
                    data.fixed_equal_nucleotide_frequencies.copy())

    def p(self, t, rates=None):
        if rates is not None:
            return DNAReversibleModel.p(self, t, rates)
        e1 = 0.25 + 0.75 * np.exp(-4 * t / 3.)
        e2 = 0.25 - 0.25 * np.exp(-4 * t / 3.)
        return np.where(np.eye(4, dtype=bool), e1, e2)


class Strsym(DNANonReversibleModel):
    """Strand-symmetric (strsym.py): 6 rates, A<->C == T<->G, etc."""
    _name = "STRSYM"

    def __init__(self, rates=None):
        Model.__init__(self)
        if rates is None:
            rates = [1.0] * 6
        if len(rates) != 6:
            raise ValueError("Provide a list of 6 rate parameters")
        a, b, c, d, e, f = [float(x) for x in rates]
        # rows/cols A C G T; X->Y and comp(X)->comp(Y) share a rate (strsym.py:34-35)
        m = np.array([[0, a, b, c],
                      [d, 0, e, f],
                      [f, e, 0, d],
                      [c, b, a, 0]], dtype=np.float64)
        self._rates = check_rates(m, 4, symmetry=False)
        self._q_mtx = compute_q_matrix(self._rates, None)

    @property
    def freqs(self):
        return q_to_freqs(self._q_mtx)


class Unrest(DNANonReversibleModel):
    """Unrestricted 12-rate model (unrest.py)."""
    _name = "UNREST"

    def __init__(self, rates=None):
        Model.__init__(self)
        if rates is None:
            rates = data.fixed_equal_nucleotide_rates.copy()
        self._rates = check_rates(rates, 4, symmetry=False)
        self._q_mtx = compute_q_matrix(self._rates, None)

    @property
    def freqs(self):
        return q_to_freqs(self._q_mtx)


# ----------------------------------------------------------------- protein models
class LG(ProteinModel):
    _name = "LG"

    def __init__(self, freqs=None):
        ProteinModel.__init__(self, data.lg_rates, freqs, data.lg_freqs)


class WAG(ProteinModel):
    _name = "WAG"

    def __init__(self, freqs=None):
        ProteinModel.__init__(self, data.wag_rates, freqs, data.wag_freqs)


class JTT(ProteinModel):
    _name = "JTT"

    def __init__(self, freqs=None):
        ProteinModel.__init__(self, data.jtt_rates, freqs, data.jtt_freqs)


class Dayhoff(ProteinModel):
    _name = "Dayhoff"

    def __init__(self, freqs=None):
        ProteinModel.__init__(self, data.dayhoff_rates, freqs, data.dayhoff_freqs)


__all__ = ["JC69", "K80", "F81", "F84", "HKY85", "TN93", "GTR", "Strsym", "Unrest", "LG",
           "WAG", "JTT", "Dayhoff", "Model", "Eigen"]
