"""One-dimensional optimisers and parameter transforms: the ``phylo_utils.optimisation``
interface (reference ``src/optimisation.pyx``), restated in Python.

These are host algorithms over Python callables; the callables this package hands them
evaluate on the GPU (``TreeModel.optimise_edge(method="brent" | "dbrent")``: one
``k_edge`` launch per evaluation).  The reference's behaviour is kept
exactly, including its quirks, so that a caller sees the same sequence of evaluations and
the same result:

* ``brent_wrap(guess, lbracket, rbracket, fn)`` calls ``brent(lbracket, rbracket, guess)``
  (``optimisation.pyx:308-314``): the *bracket* is [lbracket, guess] (ordered) and the
  search starts at ``rbracket``.
* ``brent`` runs at most ITMAX = 100 iterations, ``dbrent`` at most 99
  (``range(1, ITMAX)``, :196); on exhaustion both return f(x) re-evaluated and
  ITMAX + 1 as the iteration count (:175-177, 295-297).
* ``dbrent``'s minimum-step probe moves by ``tol``, not ``tol1`` (:262), and its last
  housekeeping test is ``fu < fv`` where ``brent`` has ``fu <= fv`` (:168 vs :292).

Parity: ``tests/test_optimisation.py`` replays fixtures made by the reference's own
compiled module (``tests/golden/make_golden_optim.py``): every evaluated abscissa and the
``out`` triple agree bit for bit.
"""
from __future__ import annotations

import numpy as np
from scipy.special import expit, logit

__all__ = ["simplex_encode", "simplex_decode", "transform_params", "decode_params",
           "quad_interp", "brent", "dbrent", "brent_wrap", "dbrent_wrap"]

ITMAX = 100
CGOLD = 0.3819660112501051   # 1 - 1/golden ratio
ZEPS = 1.0e-10
TINY = 1e-15


# ------------------------------------------------------------------ parameter transforms
def simplex_encode(p):
    """Frequencies p (length N, summing to 1) -> stick-breaking fractions theta (length
    N - 1), each in [0, 1] (optimisation.pyx:14-29)."""
    p = np.ascontiguousarray(p, dtype=np.float64)
    theta = np.zeros(p.size - 1)
    rest = 1.0
    for i in range(p.size - 1):
        theta[i] = p[i] / rest
        rest -= p[i]
    return theta


def simplex_decode(theta):
    """Inverse of simplex_encode (optimisation.pyx:31-43)."""
    theta = np.ascontiguousarray(theta, dtype=np.float64)
    p = np.zeros(theta.size + 1)
    left = 1.0
    for i in range(theta.size):
        p[i] = theta[i] * left
        left *= 1.0 - theta[i]
    p[theta.size] = left
    return p


def transform_params(p):
    """Simplex -> unconstrained reals: logit of the stick-breaking fractions (:45-46)."""
    return logit(simplex_encode(p))


def decode_params(q):
    """Unconstrained reals -> simplex (:48-49)."""
    return simplex_decode(expit(q))


# ------------------------------------------------------------------ 1-D minimisation
def quad_interp(p, q, r, fp, fq, fr):
    """Abscissa of the turning point of the parabola through (p, fp), (q, fq), (r, fr),
    the divisor clamped away from zero by TINY (optimisation.pyx:62-84)."""
    # products grouped as in the reference (r * (r * fp), not (r * r) * fp): same rounding
    num = (-r * (r * fp) + q * (q * fp) - p * (p * fq) + r * (r * fq) - q * (q * fr) +
           p * (p * fr))
    div = (q * fp - r * fp + r * fq - p * fq + p * fr - q * fr)
    if div < 0 and -div < TINY:
        div = -TINY
    elif 0 <= div < TINY:
        div = TINY
    return num / (2 * div)


def brent(ax, bx, cx, f, tol, out):
    """Brent's parabolic-interpolation / golden-section minimiser over the bracket spanned by
    ax and cx, starting at bx (optimisation.pyx:86-177).  Fills out[:3] with
    (x, f(x), iterations)."""
    lo, hi = (ax, cx) if ax < cx else (cx, ax)
    x = w = v = float(bx)
    fx = fw = fv = f(x)
    d = 0.0
    e = 0.0          # the step before last
    for it in range(1, ITMAX + 1):
        xm = 0.5 * (lo + hi)
        tol1 = tol * abs(x) + ZEPS
        tol2 = 2.0 * tol1
        if abs(x - xm) <= tol2 - 0.5 * (hi - lo):
            out[0], out[1], out[2] = x, fx, it
            return
        golden = True
        if abs(e) > tol1:
            # parabola through x, w, v
            r = (x - w) * (fx - fv)
            q = (x - v) * (fx - fw)
            p = (x - v) * q - (x - w) * r
            q = 2.0 * (q - r)
            if q > 0.0:
                p = -p
            q = abs(q)
            e_old, e = e, d
            if not (abs(p) >= abs(0.5 * q * e_old) or p <= q * (lo - x) or p >= q * (hi - x)):
                golden = False
                d = p / q
                if (x + d) - lo < tol2 or hi - (x + d) < tol2:
                    d = tol1 if xm - x >= 0 else -tol1
        if golden:
            e = (lo - x) if x >= xm else (hi - x)
            d = CGOLD * e
        u = x + d if abs(d) >= tol1 else x + (tol1 if d >= 0 else -tol1)
        fu = f(u)    # the one evaluation per iteration
        if fu <= fx:
            if u >= x:
                lo = x
            else:
                hi = x
            v, w, x = w, x, u
            fv, fw, fx = fw, fx, fu
        else:
            if u < x:
                lo = u
            else:
                hi = u
            if fu <= fw or w == x:
                v, w = w, u
                fv, fw = fw, fu
            elif fu <= fv or v == x or v == w:
                v, fv = u, fu
    out[0], out[1], out[2] = x, f(x), ITMAX + 1


def dbrent(ax, bx, cx, f, df, tol, out):
    """Brent's minimiser with derivatives: secant steps from the two previous points,
    bisection on the side the derivative points to (optimisation.pyx:179-297).  Fills
    out[:3] with (x, f(x), iterations)."""
    assert len(out) >= 3
    lo, hi = (ax, cx) if ax < cx else (cx, ax)
    x = w = v = float(bx)
    fx = fw = fv = f(x)
    dx = dw = dv = df(x)
    d = 0.0
    e = 0.0
    for it in range(1, ITMAX):
        xm = 0.5 * (lo + hi)
        tol1 = tol * abs(x) + ZEPS
        tol2 = 2.0 * tol1
        if abs(x - xm) <= tol2 - 0.5 * (hi - lo):
            out[0], out[1], out[2] = x, fx, it
            return
        bisect = True
        if abs(e) > tol1:
            s1 = s2 = 2.0 * (hi - lo)   # out-of-bracket defaults
            if dw != dx:
                s1 = (w - x) * dx / (dx - dw)   # secant through w
            if dv != dx:
                s2 = (v - x) * dx / (dx - dv)   # secant through v
            u1, u2 = x + s1, x + s2
            ok1 = (lo - u1) * (u1 - hi) > 0.0 and dx * s1 <= 0.0
            ok2 = (lo - u2) * (u2 - hi) > 0.0 and dx * s2 <= 0.0
            e_old, e = e, d
            if ok1 or ok2:
                if ok1 and ok2:
                    d = s1 if abs(s1) < abs(s2) else s2
                else:
                    d = s1 if ok1 else s2
                if abs(d) <= abs(0.5 * e_old):
                    bisect = False
                    if (x + d) - lo < tol2 or hi - (x + d) < tol2:
                        d = tol1 if xm - x >= 0 else -tol1
        if bisect:
            e = (lo - x) if dx >= 0.0 else (hi - x)
            d = 0.5 * e
        if abs(d) >= tol1:
            u = x + d
            fu = f(u)
        else:
            u = x + (tol if d >= 0 else -tol)
            fu = f(u)
            if fu > fx:   # the smallest downhill step goes uphill: done
                out[0], out[1], out[2] = x, fx, it
                return
        du = df(u)
        if fu <= fx:
            if u >= x:
                lo = x
            else:
                hi = x
            v, fv, dv = w, fw, dw
            w, fw, dw = x, fx, dx
            x, fx, dx = u, fu, du
        else:
            if u < x:
                lo = u
            else:
                hi = u
            if fu <= fw or w == x:
                v, fv, dv = w, fw, dw
                w, fw, dw = u, fu, du
            elif fu < fv or v == x or v == w:
                v, fv, dv = u, fu, du
    out[0], out[1], out[2] = x, f(x), ITMAX + 1


def dbrent_wrap(guess, lbracket, rbracket, fn, dfn, tol=1.5e-8):
    """out = [x, f(x), iterations] (optimisation.pyx:300-306; argument order as there:
    dbrent(lbracket, rbracket, guess))."""
    out = np.zeros(3, dtype=np.double)
    dbrent(float(lbracket), float(rbracket), float(guess), fn, dfn, float(tol), out)
    return out


def brent_wrap(guess, lbracket, rbracket, fn, tol=1.5e-8):
    """out = [x, f(x), iterations] (optimisation.pyx:308-314; argument order as there:
    brent(lbracket, rbracket, guess))."""
    out = np.zeros(3, dtype=np.double)
    brent(float(lbracket), float(rbracket), float(guess), fn, float(tol), out)
    return out
