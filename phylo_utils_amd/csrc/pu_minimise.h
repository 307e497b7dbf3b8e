// pu_minimise.h -- the reference's one-dimensional minimisers (src/optimisation.pyx: brent
// :86-177, dbrent :179-297; restated in phylo_utils_amd/optimisation.py, bit-identical to the
// compiled module) as a resumable state machine: min_start() names the first abscissa to
// evaluate, min_step() takes f and f' there and names the next one, until `done`.  One
// definition serves both drivers of pu_minimise_edge (pu_edge.cpp): the host loop (one k_edge
// launch per evaluation) and the combiner of the persistent k_edge_newton launch
// (pu_edge.hip), so both take exactly the reference's steps.  Arithmetic as in the reference:
// no contraction into fused multiply-adds, the reference's operand order.
#pragma once

#include <hip/hip_runtime.h>

namespace pu {

enum : int { PU_MIN_NEWTON = 0, PU_MIN_BRENT = 1, PU_MIN_DBRENT = 2 };

struct MinState {
    double x, w, v, fx, fw, fv, dx, dw, dv, d, e, lo, hi, u, tol;
    int method, it, phase, small, done;
    double res_x, res_f;  // out[0], out[1] of the reference (f = the minimised objective)
    int res_it;           // out[2]: iterations (ITMAX + 1 when exhausted)
};

constexpr int kMinItmax = 100;                     // optimisation.pyx ITMAX
constexpr double kMinCGold = 0.3819660112501051;   // CGOLD
constexpr double kMinZeps = 1.0e-10;               // ZEPS
enum : int { MS_INIT = 0, MS_EVAL = 1, MS_FINAL = 2 };

// brent(ax, bx, cx) / dbrent(ax, bx, cx): the bracket spanned by ax and cx, the search from bx
__host__ __device__ inline double min_start(MinState &s, int method, double ax, double bx,
                                            double cx, double tol) {
    s.method = method;
    s.lo = ax < cx ? ax : cx;
    s.hi = ax < cx ? cx : ax;
    s.x = s.w = s.v = bx;
    s.tol = tol;
    s.d = s.e = 0.0;
    s.it = 1;
    s.phase = MS_INIT;
    s.small = 0;
    s.done = 0;
    return bx;
}

__host__ __device__ inline void min_finish(MinState &s, double x, double f, int it) {
    s.res_x = x;
    s.res_f = f;
    s.res_it = it;
    s.done = 1;
}

// the loop head: convergence test, then the next abscissa (phase MS_EVAL), or the final
// re-evaluation of x when the iterations are spent (MS_FINAL)
__host__ __device__ inline double min_plan(MinState &s) {
#pragma clang fp contract(off)
    const bool db = s.method == PU_MIN_DBRENT;
    // brent: for it in range(1, ITMAX + 1); dbrent: for it in range(1, ITMAX)
    if (s.it > (db ? kMinItmax - 1 : kMinItmax)) {
        s.phase = MS_FINAL;
        return s.x;
    }
    const double x = s.x, lo = s.lo, hi = s.hi;
    const double xm = 0.5 * (lo + hi);
    const double tol1 = s.tol * fabs(x) + kMinZeps;
    const double tol2 = 2.0 * tol1;
    if (fabs(x - xm) <= tol2 - 0.5 * (hi - lo)) {
        min_finish(s, x, s.fx, s.it);
        return x;
    }
    double d = s.d, e = s.e;
    if (!db) {  // optimisation.pyx:105-137
        bool golden = true;
        if (fabs(e) > tol1) {  // the parabola through x, w, v
            const double r = (x - s.w) * (s.fx - s.fv);
            double q = (x - s.v) * (s.fx - s.fw);
            double p = (x - s.v) * q - (x - s.w) * r;
            q = 2.0 * (q - r);
            if (q > 0.0) p = -p;
            q = fabs(q);
            const double e_old = e;
            e = d;
            if (!(fabs(p) >= fabs(0.5 * q * e_old) || p <= q * (lo - x) || p >= q * (hi - x))) {
                golden = false;
                d = p / q;
                if ((x + d) - lo < tol2 || hi - (x + d) < tol2) d = xm - x >= 0 ? tol1 : -tol1;
            }
        }
        if (golden) {
            e = x >= xm ? (lo - x) : (hi - x);
            d = kMinCGold * e;
        }
        s.d = d;
        s.e = e;
        s.small = 0;
        s.u = fabs(d) >= tol1 ? x + d : x + (d >= 0 ? tol1 : -tol1);
    } else {  // optimisation.pyx:205-266
        bool bisect = true;
        if (fabs(e) > tol1) {
            double s1 = 2.0 * (hi - lo), s2 = s1;  // out-of-bracket defaults
            if (s.dw != s.dx) s1 = (s.w - x) * s.dx / (s.dx - s.dw);
            if (s.dv != s.dx) s2 = (s.v - x) * s.dx / (s.dx - s.dv);
            const double u1 = x + s1, u2 = x + s2;
            const bool ok1 = (lo - u1) * (u1 - hi) > 0.0 && s.dx * s1 <= 0.0;
            const bool ok2 = (lo - u2) * (u2 - hi) > 0.0 && s.dx * s2 <= 0.0;
            const double e_old = e;
            e = d;
            if (ok1 || ok2) {
                if (ok1 && ok2)
                    d = fabs(s1) < fabs(s2) ? s1 : s2;
                else
                    d = ok1 ? s1 : s2;
                if (fabs(d) <= fabs(0.5 * e_old)) {
                    bisect = false;
                    if ((x + d) - lo < tol2 || hi - (x + d) < tol2) d = xm - x >= 0 ? tol1 : -tol1;
                }
            }
        }
        if (bisect) {
            e = s.dx >= 0.0 ? (lo - x) : (hi - x);
            d = 0.5 * e;
        }
        s.d = d;
        s.e = e;
        if (fabs(d) >= tol1) {
            s.small = 0;
            s.u = x + d;
        } else {  // the smallest step (by tol, not tol1: optimisation.pyx:262)
            s.small = 1;
            s.u = x + (d >= 0 ? s.tol : -s.tol);
        }
    }
    s.phase = MS_EVAL;
    return s.u;
}

// f, df: the objective and its derivative at the abscissa the last call named
__host__ __device__ inline double min_step(MinState &s, double f, double df) {
#pragma clang fp contract(off)
    if (s.phase == MS_INIT) {
        s.fx = s.fw = s.fv = f;
        s.dx = s.dw = s.dv = df;
        return min_plan(s);
    }
    if (s.phase == MS_FINAL) {
        min_finish(s, s.x, f, kMinItmax + 1);
        return s.x;
    }
    const bool db = s.method == PU_MIN_DBRENT;
    const double u = s.u, fu = f, du = df, x = s.x;
    if (db && s.small && fu > s.fx) {  // the smallest downhill step goes uphill: done
        min_finish(s, x, s.fx, s.it);
        return x;
    }
    if (fu <= s.fx) {
        if (u >= x)
            s.lo = x;
        else
            s.hi = x;
        s.v = s.w, s.fv = s.fw, s.dv = s.dw;
        s.w = x, s.fw = s.fx, s.dw = s.dx;
        s.x = u, s.fx = fu, s.dx = du;
    } else {
        if (u < x)
            s.lo = u;
        else
            s.hi = u;
        if (fu <= s.fw || s.w == x) {
            s.v = s.w, s.fv = s.fw, s.dv = s.dw;
            s.w = u, s.fw = fu, s.dw = du;
        } else if ((db ? fu < s.fv : fu <= s.fv) || s.v == x || s.v == s.w) {
            // (dbrent's test is fu < fv where brent has fu <= fv: optimisation.pyx:168, 292)
            s.v = u, s.fv = fu, s.dv = du;
        }
    }
    ++s.it;
    return min_plan(s);
}

}  // namespace pu
