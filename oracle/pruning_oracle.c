/*
 * pruning_oracle.c -- CPU restatement of phylo_utils' live likelihood path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the CPU
 * baseline ("port") for bench.py.  Nothing in phylo_utils_amd/ links, loads
 * or calls it; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it.
 *
 * What it restates (reference paths relative to /root/reference):
 *   or_clv        numba `clv`       phylo_utils/likelihood/numba_likelihood_engine.py:14-46
 *                 (rescale rule 0 < m < 2^-128, threshold :7; divide by m, add log m)
 *   or_lnl_node   numba `lnl_node`  numba_likelihood_engine.py:82-87  (-inf when f <= 0)
 *   or_pmatrix    Model.p / Eigen.exp   phylo_utils/substitution_models/abstract.py:49-59,99-105
 *                 P = (evecs * exp(evals * t * r)) . ivecs
 *   or_edge_derivs  edge lnL + d/dt, d2/dt2 over the rate mixture (SURVEY 8(f) N1;
 *                 lnl_branch_derivs numba_likelihood_engine.py:49-57)
 *   or_traverse   TreeModel.compute_partials + compute_likelihood_at_edge
 *                 phylo_utils/tree_model.py:160-176, 178-198, 200-217
 *                 (post-order ops, root combine with P(0)=I, lnl_node, logsumexp over
 *                 categories with log weights, pattern weights, sum).
 *
 * The arithmetic is deliberately plain: sequential dot products, separate
 * multiply and add (build with -ffp-contract=off), division by m.  The
 * oracle is pinned by tests/golden (generated from the reference's own
 * numpy engine, substitution models and PAML C) -- see DESIGN.md "Oracle".
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_SCALE_THRESHOLD (1.0 / 340282366920938463463374607431768211456.0) /* 2^-128 */

/* one (site, category) K-vector update; numba_likelihood_engine.py:36-44 */
static inline void clv_one(int K, const double *p1, const double *p2, const double *a,
                           const double *b, double sa, double sb, double *out,
                           double *cml) {
    double m;
    int i, j;
    for (i = 0; i < K; ++i) {
        double x = 0.0, y = 0.0;
        for (j = 0; j < K; ++j) x += p1[i * K + j] * a[j];
        for (j = 0; j < K; ++j) y += p2[i * K + j] * b[j];
        out[i] = x * y;
    }
    /* np.max: NaN propagates */
    m = out[0];
    for (i = 1; i < K; ++i)
        if (out[i] > m || out[i] != out[i]) m = out[i];
    if (m < OR_SCALE_THRESHOLD && m > 0) {
        *cml = sa + sb + log(m);
        for (i = 0; i < K; ++i) out[i] /= m;
    } else {
        *cml = sa + sb;
    }
}

/* clv over S sites: p1,p2 [C][K][K]; clv1,clv2,out [S][C][K]; sa,sb,cml [S][C] */
void or_clv(int K, int C, long S, const double *p1, const double *p2, const double *clv1,
            const double *clv2, const double *sa, const double *sb, double *cml,
            double *out) {
    long s;
    int c;
    for (s = 0; s < S; ++s)
        for (c = 0; c < C; ++c) {
            long v = (s * C + c) * K, e = s * C + c;
            clv_one(K, p1 + (long)c * K * K, p2 + (long)c * K * K, clv1 + v, clv2 + v,
                    sa[e], sb[e], out + v, cml + e);
        }
}

/* lnl_node: pi [K], partials [S][C][K], scale [S][C] -> out [S][C] */
void or_lnl_node(int K, int C, long S, const double *pi, const double *partials,
                 const double *scale, double *out) {
    long s;
    int c, i;
    for (s = 0; s < S; ++s)
        for (c = 0; c < C; ++c) {
            const double *v = partials + (s * C + c) * K;
            double f = 0.0;
            for (i = 0; i < K; ++i) f += v[i] * pi[i];
            out[s * C + c] = (f > 0) ? log(f) + scale[s * C + c] : -INFINITY;
        }
}

/* P for n_br branches x C rates: out [n_br][C][K][K] */
void or_pmatrix(int K, int C, int n_br, const double *evecs, const double *evals,
                const double *ivecs_rowmajor, const double *brlens, const double *rates,
                double *out) {
    int b, c, i, j, k;
    double *ex = (double *)malloc(sizeof(double) * K);
    for (b = 0; b < n_br; ++b)
        for (c = 0; c < C; ++c) {
            double *P = out + ((long)b * C + c) * K * K;
            for (k = 0; k < K; ++k) ex[k] = exp(evals[k] * (brlens[b] * rates[c]));
            for (i = 0; i < K; ++i)
                for (j = 0; j < K; ++j) {
                    double acc = 0.0;
                    for (k = 0; k < K; ++k) acc += (evecs[i * K + k] * ex[k]) * ivecs_rowmajor[k * K + j];
                    P[i * K + j] = acc;
                }
        }
    free(ex);
}

/* scipy.special.logsumexp over a length-C vector (tree_model.py:216), restating
 * scipy 1.15 `_logsumexp`: the maximal terms (count m) are taken out of the sum,
 * out = log1p(s/m) + log(m) + a_max with s the shifted sum of the others. */
static inline double lse(int C, const double *a) {
    double amax = -INFINITY, shift, s = 0.0, m = 0.0;
    int c;
    for (c = 0; c < C; ++c)
        if (a[c] > amax) amax = a[c];
    for (c = 0; c < C; ++c)
        if (a[c] == amax) m += 1.0;
    shift = isfinite(amax) ? amax : 0.0;
    for (c = 0; c < C; ++c)
        if (a[c] != amax) s += exp(a[c] - shift);
    if (s != 0.0) s /= m;
    return log1p(s) + log(m) + amax;
}

/*
 * Whole traversal.  partials/scale are [n_nodes][S][C][K] / [n_nodes][S][C]
 * with tip rows pre-filled by the caller (tree_model.py:142-148).
 * ops [n_ops][3] = (par, ch1, ch2); P [n_ops][2][C][K][K]; Proot [2][C][K][K]
 * (P(0) for root_a, P(len) for root_b; tree_model.py:189-197).
 * Returns sum_s site_weights[s] * site_lnl[s].
 */
double or_traverse(int K, int C, long S, int n_ops, const int32_t *ops, const double *P,
                   const double *Proot, int root_a, int root_b, double *partials,
                   double *scale, double *root_partials, double *root_scale,
                   const double *pi, const double *weights, const double *site_weights,
                   double *site_lnl, int nthreads) {
    const long nv = S * C * K, ns = S * C;
    double total = 0.0;
    long blk = 256;
    long nblk = (S + blk - 1) / blk;
    long bi;
    double *logw = (double *)malloc(sizeof(double) * C);
    int c;
    if (C > 64) {
        free(logw);
        return NAN;
    }
    for (c = 0; c < C; ++c) logw[c] = log(weights[c]);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static) reduction(+ : total)
#endif
    for (bi = 0; bi < nblk; ++bi) {
        long s0 = bi * blk, s1 = s0 + blk < S ? s0 + blk : S, s;
        int o, cc;
        double sw[64];
        for (o = 0; o < n_ops; ++o) {
            int par = ops[3 * o], c1 = ops[3 * o + 1], c2 = ops[3 * o + 2];
            const double *p1 = P + (long)o * 2 * C * K * K, *p2 = p1 + (long)C * K * K;
            for (s = s0; s < s1; ++s)
                for (cc = 0; cc < C; ++cc) {
                    long v = (s * C + cc) * K, e = s * C + cc;
                    clv_one(K, p1 + (long)cc * K * K, p2 + (long)cc * K * K,
                            partials + c1 * nv + v, partials + c2 * nv + v,
                            scale[c1 * ns + e], scale[c2 * ns + e], partials + par * nv + v,
                            scale + par * ns + e);
                }
        }
        for (s = s0; s < s1; ++s) {
            double f;
            int i;
            for (cc = 0; cc < C; ++cc) {
                long v = (s * C + cc) * K, e = s * C + cc;
                clv_one(K, Proot + (long)cc * K * K, Proot + (long)(C + cc) * K * K,
                        partials + root_a * nv + v, partials + root_b * nv + v,
                        scale[root_a * ns + e], scale[root_b * ns + e], root_partials + v,
                        root_scale + e);
                f = 0.0;
                for (i = 0; i < K; ++i) f += root_partials[v + i] * pi[i];
                sw[cc] = ((f > 0) ? log(f) + root_scale[e] : -INFINITY) + logw[cc];
            }
            site_lnl[s] = lse(C, sw);
            total += site_weights[s] * site_lnl[s];
        }
    }
    free(logw);
    return total;
}

/*
 * Edge lnL and its first and second derivatives w.r.t. the edge length t.
 * The root sits on edge (a, b) as in compute_partials_at_edge (tree_model.py:178-198):
 * P(0) on a; on b P(t r_c) and its t-derivatives dP, d2P (evecs diag((l r)^k e^{l t r})
 * ivecs).  Per category f_c = sum_i pi_i (P0 a)_i (P b)_i as in lnl_branch_derivs
 * (numba_likelihood_engine.py:49-57); per site the rate mixture
 * L_s = sum_c w_c f_c e^{sa_c + sb_c}, and out3 = {sum_s sw_s log L_s, sum_s sw_s L'_s/L_s,
 * sum_s sw_s (L''_s/L_s - (L'_s/L_s)^2)}.  a, b [S][C][K]; sa, sb [S][C]; P* [C][K][K].
 */
void or_edge_derivs(int K, int C, long S, const double *a, const double *sa, const double *b,
                    const double *sb, const double *P0, const double *P, const double *dP,
                    const double *d2P, const double *pi, const double *weights,
                    const double *site_weights, double *out3, double *site_lnl) {
    double t0 = 0.0, t1 = 0.0, t2 = 0.0;
    long s;
    int c, i, j;
    double lc[64], g1[64], g2[64];
    if (C > 64) {
        out3[0] = out3[1] = out3[2] = NAN;
        return;
    }
    for (s = 0; s < S; ++s) {
        double mx = -INFINITY, L = 0.0, N1 = 0.0, N2 = 0.0;
        for (c = 0; c < C; ++c) {
            const double *va = a + (s * C + c) * K, *vb = b + (s * C + c) * K;
            const long m0 = (long)c * K * K;
            double f = 0.0, f1 = 0.0, f2 = 0.0;
            for (i = 0; i < K; ++i) {
                double x = 0.0, y = 0.0, yd = 0.0, yd2 = 0.0;
                for (j = 0; j < K; ++j) {
                    x += P0[m0 + i * K + j] * va[j];
                    y += P[m0 + i * K + j] * vb[j];
                    yd += dP[m0 + i * K + j] * vb[j];
                    yd2 += d2P[m0 + i * K + j] * vb[j];
                }
                f += pi[i] * x * y;
                f1 += pi[i] * x * yd;
                f2 += pi[i] * x * yd2;
            }
            if (f > 0) {
                lc[c] = log(f) + sa[s * C + c] + sb[s * C + c] + log(weights[c]);
                g1[c] = f1 / f;
                g2[c] = f2 / f;
                if (lc[c] > mx) mx = lc[c];
            } else {
                lc[c] = -INFINITY;
                g1[c] = g2[c] = 0.0;
            }
        }
        for (c = 0; c < C; ++c) {
            if (lc[c] == -INFINITY) continue;
            double e = exp(lc[c] - mx);
            L += e;
            N1 += e * g1[c];
            N2 += e * g2[c];
        }
        if (L > 0) {
            double d1 = N1 / L;
            double sl = mx + log(L);
            if (site_lnl) site_lnl[s] = sl;
            t0 += site_weights[s] * sl;
            t1 += site_weights[s] * d1;
            t2 += site_weights[s] * (N2 / L - d1 * d1);
        } else {
            if (site_lnl) site_lnl[s] = -INFINITY;
            if (site_weights[s] != 0) t0 = -INFINITY;
        }
    }
    out3[0] = t0;
    out3[1] = t1;
    out3[2] = t2;
}
