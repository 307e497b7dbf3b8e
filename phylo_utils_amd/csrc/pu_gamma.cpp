// pu_gamma.cpp -- discrete-gamma rate categories (host).
//
// Replaces phylo_utils.discrete_gamma.discrete_gamma (src/discrete_gamma.pyx:30-47),
// which calls PAML's DiscreteGamma (src/c_discrete_gamma.c:285-321) with
// alpha == beta.  Implemented here from the published algorithms the reference
// cites, evaluated in the same arithmetic order so the rates agree to the bit:
//   * ln Gamma        Pike & Hill (1966), CACM Algorithm 291 (Stirling series,
//                     argument shifted to >= 7); an exact-factorial shortcut for
//                     integer arguments 0..11 in the mean-rate path.
//   * normal quantile Odeh & Evans (1974), Applied Statistics AS 70.
//   * chi2 quantile   Best & Roberts (1975), Applied Statistics AS 91
//                     (tolerance 0.5e-6 relative).
//   * incomplete Gamma ratio  Bhattacharjee (1970), Applied Statistics AS 32
//                     (series for x <= 1 or x < alpha, else continued fraction;
//                     tolerance 1e-8).
//   * mean rates: Yang (1994) eq. 9-10: category boundaries from the gamma
//     quantiles, mean of each slice from I(b*beta, alpha+1).
#include <math.h>

#include "../../include/phylo_hip.h"

namespace {

constexpr double kLnSqrt2Pi = 0.918938533204673;
constexpr double kLn2 = 0.6931471805;  // AS 91 keeps this 10-digit constant

// head + Stirling series, summed left to right from `head` (the association
// matters for bitwise agreement with the reference's rates).
double stirling(double head, double x) {
    const double z = 1.0 / (x * x);
    return head + (x - 0.5) * log(x) - x + kLnSqrt2Pi +
           (((-0.000595238095238 * z + 0.000793650793651) * z - 0.002777777777778) * z +
            0.083333333333333) /
               x;
}

// Shift x up to >= 7 by the recurrence Gamma(x+1) = x Gamma(x); returns the
// log of the accumulated product's reciprocal and updates x.
double shift_to_seven(double &x) {
    if (!(x < 7.0)) return 0.0;
    double prod = 1.0, z = x - 1.0;
    while (++z < 7.0) prod *= z;
    x = z;
    return -log(prod);
}

// ln Gamma(x), x > 0, Algorithm 291 form used by the chi2 quantile.
double ln_gamma_291(double x) {
    const double f = shift_to_seven(x);
    return stirling(f, x);
}

// ln Gamma(x) with the exact small-integer branch (used for alpha + 1).
double ln_gamma_exact_int(double x) {
    const int n = (int)x;
    if ((double)n == x && n >= 0 && n <= 11) {
        long fact = 1;
        for (long i = 2; i <= (long)(n - 1); ++i) fact *= i;
        return log((double)fact);
    }
    double fneg = 0.0;
    if (x <= 0.0) {  // not reached for rate models (alpha > 0)
        if ((int)x - x == 0) return -1.0;
        double r = 1.0;
        for (; x < 0; x++) r /= x;
        if (r < 0) return -1.0;
        fneg = log(r);
    }
    const double f = shift_to_seven(x);
    return stirling(fneg + f, x);
}

double normal_quantile_as70(double prob) {
    const double a0 = -0.322232431088, a1 = -1.0, a2 = -0.342242088547,
                 a3 = -0.0204231210245, a4 = -0.453642210148e-4;
    const double b0 = 0.0993484626060, b1 = 0.588581570495, b2 = 0.531103462366,
                 b3 = 0.103537752850, b4 = 0.0038560700634;
    const double tail = prob < 0.5 ? prob : 1.0 - prob;
    double z;
    if (tail < 1e-20) {
        z = 999.0;
    } else {
        const double y = sqrt(log(1.0 / (tail * tail)));
        z = y + ((((y * a4 + a3) * y + a2) * y + a1) * y + a0) /
                    ((((y * b4 + b3) * y + b2) * y + b1) * y + b0);
    }
    return prob < 0.5 ? -z : z;
}

// AS 32: regularised lower incomplete gamma P(alpha, x); -1 on bad input.
double incomplete_gamma_as32(double x, double alpha, double ln_gamma_alpha) {
    const double accurate = 1e-8, overflow = 1e30;
    if (x == 0) return 0.0;
    if (x < 0 || alpha <= 0) return -1.0;
    const double factor = exp(alpha * log(x) - x - ln_gamma_alpha);
    if (!(x > 1 && x >= alpha)) {
        // series expansion
        double sum = 1.0, term = 1.0, rn = alpha;
        do {
            rn += 1.0;
            term *= x / rn;
            sum += term;
        } while (term > accurate);
        return sum * (factor / alpha);
    }
    // continued fraction (Legendre), two-term recurrences pn[0..5]
    double a = 1.0 - alpha, b = a + x + 1.0, term = 0.0;
    double pn[6] = {1.0, x, x + 1.0, x * b, 0.0, 0.0};
    double frac = pn[2] / pn[3];
    for (;;) {
        a += 1.0;
        b += 2.0;
        term += 1.0;
        const double an = a * term;
        pn[4] = b * pn[2] - an * pn[0];
        pn[5] = b * pn[3] - an * pn[1];
        if (pn[5] != 0) {
            const double rn = pn[4] / pn[5];
            const double dif = fabs(frac - rn);
            if (dif <= accurate && dif <= accurate * rn) break;  // keeps the previous convergent
            frac = rn;
        }
        for (int i = 0; i < 4; ++i) pn[i] = pn[i + 2];
        if (!(fabs(pn[4]) < overflow))
            for (int i = 0; i < 4; ++i) pn[i] /= overflow;
    }
    return 1.0 - factor * frac;
}

// AS 91: chi2 quantile with v degrees of freedom; -1 on bad input.
double chi2_quantile_as91(double prob, double v) {
    const double tol = 0.5e-6;
    if (prob < 0.000002 || prob > 0.999998 || v <= 0) return -1.0;
    const double g = ln_gamma_291(v / 2);
    const double xx = v / 2, c = xx - 1;
    double ch;
    if (v < -1.24 * log(prob)) {
        // small degrees of freedom relative to the tail
        ch = pow(prob * xx * exp(g + xx * kLn2), 1 / xx);
        if (ch - tol < 0) return ch;
    } else if (v <= 0.32) {
        ch = 0.4;
        const double la = log(1 - prob);
        double q;
        do {
            q = ch;
            const double p1 = 1 + ch * (4.67 + ch);
            const double p2 = ch * (6.73 + ch * (6.66 + ch));
            const double t = -0.5 + (4.67 + 2 * ch) / p1 - (6.73 + ch * (13.32 + 3 * ch)) / p2;
            ch -= (1 - exp(la + g + 0.5 * ch + c * kLn2) * p2 / p1) / t;
        } while (fabs(q / ch - 1) - 0.01 > 0);
    } else {
        // Wilson-Hilferty start
        const double x = normal_quantile_as70(prob);
        const double p1 = 0.222222 / v;
        ch = v * pow((x * sqrt(p1) + 1 - p1), 3.0);
        if (ch > 2.2 * v + 6) ch = -2 * (log(1 - prob) - c * log(0.5 * ch) + g);
    }
    // seven-term Taylor refinement until relative change <= tol
    double q;
    do {
        q = ch;
        const double p1 = 0.5 * ch;
        double t = incomplete_gamma_as32(p1, xx, g);
        if (t < 0) return -1.0;
        const double p2 = prob - t;
        t = p2 * exp(xx * kLn2 + g + p1 - c * log(ch));
        const double b = t / ch;
        const double a = 0.5 * t - b * c;
        const double s1 = (210 + a * (140 + a * (105 + a * (84 + a * (70 + 60 * a))))) / 420;
        const double s2 = (420 + a * (735 + a * (966 + a * (1141 + 1278 * a)))) / 2520;
        const double s3 = (210 + a * (462 + a * (707 + 932 * a))) / 2520;
        const double s4 =
            (252 + a * (672 + 1182 * a) + c * (294 + a * (889 + 1740 * a))) / 5040;
        const double s5 = (84 + 264 * a + c * (175 + 606 * a)) / 2520;
        const double s6 = (120 + c * (346 + 127 * c)) / 5040;
        ch += t * (1 + 0.5 * t * s1 -
                   b * c * (s1 - b * (s2 - b * (s3 - b * (s4 - b * (s5 - b * s6))))));
    } while (fabs(q / ch - 1) > tol);
    return ch;
}

double gamma_quantile(double prob, double alpha, double beta) {
    return chi2_quantile_as91(prob, 2.0 * alpha) / (2.0 * beta);
}

}  // namespace

extern "C" int pu_discrete_gamma(double alpha, int n_cat, int median_rates, double *rates) {
    if (!(alpha > 0) || n_cat < 1 || rates == nullptr) return PU_E_ARG;
    const double beta = alpha, mean = alpha / beta;
    const int K = n_cat;
    if (median_rates) {
        double t = 0.0;
        for (int i = 0; i < K; ++i) rates[i] = gamma_quantile((i * 2. + 1) / (2. * K), alpha, beta);
        for (int i = 0; i < K; ++i) t += rates[i];
        for (int i = 0; i < K; ++i) rates[i] *= mean * K / t;
        return PU_OK;
    }
    if (K == 1) {  // the reference reads freqK[-1] here (c_discrete_gamma.c:314); mean is 1
        rates[0] = mean;
        return PU_OK;
    }
    const double lnga1 = ln_gamma_exact_int(alpha + 1);
    double cut_prev = 0.0;
    for (int i = 0; i < K - 1; ++i) {
        const double q = gamma_quantile((i + 1.0) / K, alpha, beta);
        if (q < 0) return PU_E_ARG;
        const double cut = incomplete_gamma_as32(q * beta, alpha + 1, lnga1);
        rates[i] = (i == 0 ? cut * mean * K : (cut - cut_prev) * mean * K);
        cut_prev = cut;
    }
    rates[K - 1] = (1 - cut_prev) * mean * K;
    return PU_OK;
}
