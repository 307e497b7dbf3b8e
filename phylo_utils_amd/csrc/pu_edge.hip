// pu_edge.hip -- gfx950 kernels for edge operations on the device-resident CLVs of a
// context: the root placed on any edge, the branch-length derivatives of the
// lnL, and in-place partials updates (the re-orientation rows of the optimising traversal).
//
// Reference behaviour (paths relative to the reference repository root):
//   EDGE_UPDATE  partials[par] = clv(P(t1), P(t2), partials[c1], partials[c2])
//                phylo_utils/likelihood/numba_likelihood_engine.py:35-44, as driven by the
//                rows of phylo_utils/utils.py:137-188 (get_optimising_traversal)
//   EDGE_LNL     compute_partials_at_edge + compute_likelihood_at_edge + sum
//                phylo_utils/tree_model.py:178-217, bin/phy.py:146 -- P(0) on node a,
//                P(length) on node b, on the nodes' CURRENT partials ("the values are only
//                valid if the CLVs at a and b are valid", tree_model.py:181-182)
//   EDGE_DERIV   lnL and its first and second derivatives w.r.t. the edge length of the
//                rate mixture sum_c w_c f_c (f_c as in lnl_branch_derivs,
//                numba_likelihood_engine.py:49-57, with d/dt P(t r) = evecs diag(l r e^{l t r})
//                ivecs -- the chain-rule factor r that Model.dp_dt, abstract.py:61-77, omits)
//
// Mapping: a workgroup is one wave and one 64-site tile; a lane is a site and walks the
// rate categories (any C), reading the tiled slot layout of pu_kernels.hip (coalesced: the
// 64 sites of a category row are contiguous).  The P matrices an edge needs are computed
// once per workgroup into LDS from the eigen-decomposition, with the arithmetic of
// k_pmatrix (so P(0) and P(t) are bit-identical to the traversal's), and read as LDS
// broadcasts.  The lnL / derivative sums are reduced in one launch: every workgroup writes
// its partial sums, and the last workgroup to finish (atomic ticket) adds them in a fixed
// order -- bitwise repeatable, no second launch, no spinning.
#include "pu_internal.h"

#include <math.h>

namespace pu {

namespace {

constexpr double kScaleThreshold = 0x1p-128;  // numba_likelihood_engine.py:7
constexpr int kLanes = 64;

typedef double dbl2 __attribute__((ext_vector_type(2)));

// ---- site vectors in the tiled slot layout (pu_kernels.hip k_untile / k_untile_aa) ----
template <int K>
__device__ __forceinline__ int tiled_index(int i, int l) {
    if constexpr (K == 20) {  // [wave 4][row 5][64]: lane (g, s16) of wave w, rows g, g+4..
        const int w = l >> 4, s16 = l & 15;
        const int g = i < 16 ? (i & 3) : i - 16, r = i < 16 ? (i >> 2) : 4;
        return (w * 5 + r) * 64 + g * 16 + s16;
    } else {  // [K/2][64][2]
        return (i >> 1) * 128 + 2 * l + (i & 1);
    }
}

template <int K>
__device__ __forceinline__ void load_site(const double *row, int l, double (&v)[K]) {
    if constexpr (K == 20) {
#pragma unroll
        for (int i = 0; i < K; ++i) v[i] = row[tiled_index<K>(i, l)];
    } else {
        const dbl2 *q = reinterpret_cast<const dbl2 *>(row) + l;
#pragma unroll
        for (int i = 0; i < K / 2; ++i) {
            const dbl2 t = q[i * kLanes];
            v[2 * i] = t.x;
            v[2 * i + 1] = t.y;
        }
    }
}

template <int K>
__device__ __forceinline__ void store_site(double *row, int l, const double (&v)[K]) {
    if constexpr (K == 20) {
#pragma unroll
        for (int i = 0; i < K; ++i) row[tiled_index<K>(i, l)] = v[i];
    } else {
        dbl2 *q = reinterpret_cast<dbl2 *>(row) + l;
#pragma unroll
        for (int i = 0; i < K / 2; ++i) q[i * kLanes] = dbl2{v[2 * i], v[2 * i + 1]};
    }
}

// the K-vector and scaler of one node at (site, category)
template <int K>
__device__ __forceinline__ void node_vec(const EdgeArgs &a, NodeSrc n, int cat, int tile, int l,
                                         int64_t site_c, double (&v)[K], double &s) {
    if (n.kind == SRC_SLOT) {
        const size_t row = (size_t)cat * a.n_tiles + tile;
        load_site<K>(a.clv + (size_t)n.idx * a.slot_stride + row * K * kLanes, l, v);
        s = a.scale[(size_t)n.idx * a.sstride + row * kLanes + l];
        return;
    }
    const double *src = n.kind == SRC_CODED
                            ? a.table + (size_t)a.codes[(size_t)n.idx * a.code_stride + site_c] * K
                            : a.tips + ((size_t)n.idx * a.S + site_c) * K;
#pragma unroll
    for (int i = 0; i < K; ++i) v[i] = src[i];
    s = 0.0;
}

// x = P v, P a [K][K] matrix in LDS; the fma chain of matvec_s / k_clv (bitwise equal)
template <int K>
__device__ __forceinline__ void matvec_l(const double *P, const double (&v)[K], double (&x)[K]) {
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) acc = fma(P[i * K + j], v[j], acc);
        x[i] = acc;
    }
}

template <int K>
__device__ __forceinline__ void rescale(double (&out)[K], double sa, double sb, double &cml) {
    double m = out[0];  // np.max: NaN propagates
#pragma unroll
    for (int i = 1; i < K; ++i) m = (out[i] > m || out[i] != out[i]) ? out[i] : m;
    const double base = sa + sb;
    if (m < kScaleThreshold && m > 0.0) {
        cml = base + log(m);
#pragma unroll
        for (int i = 0; i < K; ++i) out[i] = out[i] / m;
    } else {
        cml = base;
    }
}

// scipy 1.15 logsumexp over C values strided by 64 (tree_model.py:216; = lse_strided of
// pu_kernels.hip, so the root edge reproduces the traversal's sitewise lnL bit for bit)
__device__ __forceinline__ double lse64(const double *a, int n) {
    double amax = -INFINITY;
    for (int c = 0; c < n; ++c) amax = (a[c * kLanes] > amax) ? a[c * kLanes] : amax;
    double m = 0.0, s = 0.0;
    const double shift = isfinite(amax) ? amax : 0.0;
    for (int c = 0; c < n; ++c) {
        const double x = a[c * kLanes];
        if (x == amax)
            m += 1.0;
        else
            s += exp(x - shift);
    }
    if (s != 0.0) s /= m;
    return log1p(s) + log(m) + amax;
}

// P matrices into LDS: n_mat matrices per category, matrix m of category c at
// lds[(m * C + c) * K * K].  Matrix m uses length t[m] and derivative order ord[m]:
// evecs diag(x^ord e^{l t r}) ivecs with x = l r (k_pmatrix's arithmetic for ord 0).
template <int K>
__device__ void build_p(const EdgeArgs &a, double *lds, double *ex, int n_mat,
                        const double (&t)[4], const int (&ord)[4]) {
    const int C = a.C;
    for (int idx = threadIdx.x; idx < n_mat * C * K; idx += kLanes) {
        const int k = idx % K, mc = idx / K, c = mc % C, m = mc / C;
        const double r = a.rates[c];
        const double tt = t[m] * r;
        double e = exp(a.evals[k] * tt);
        if (ord[m] > 0) {
            const double x = a.evals[k] * r;
            e = ord[m] == 1 ? x * e : (x * x) * e;
        }
        ex[idx] = e;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < n_mat * C * K * K; idx += kLanes) {
        const int ij = idx % (K * K), mc = idx / (K * K);
        const int i = ij / K, j = ij - i * K;
        const double *e = ex + mc * K;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) acc = fma(a.evecs[i * K + k] * e[k], a.ivecs[k * K + j], acc);
        lds[idx] = acc;
    }
    __syncthreads();
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Sum the per-workgroup partials: the last workgroup to arrive adds all of them in a fixed
// order (block i's values by lane i % 64, then a fixed butterfly), so the result does not
// depend on which workgroup finished last.
__device__ void grid_reduce3(const EdgeArgs &a, double v0, double v1, double v2) {
    v0 = wave_sum(v0);
    v1 = wave_sum(v1);
    v2 = wave_sum(v2);
    __shared__ unsigned int ticket;
    if (threadIdx.x == 0) {
        double *p = a.block_part + 3 * (size_t)blockIdx.x;
        p[0] = v0;
        p[1] = v1;
        p[2] = v2;
        __threadfence();  // agent scope: the partials reach the coherent level first
        ticket = atomicAdd(a.counter, 1u);
    }
    __syncthreads();
    if (ticket != gridDim.x - 1) return;
    __threadfence();
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += kLanes) {
        const double *p = a.block_part + 3 * (size_t)b;
        s0 += __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s1 += __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s2 += __hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (threadIdx.x == 0) {
        a.result[0] = s0;
        a.result[1] = s1;
        a.result[2] = s2;
        *a.counter = 0u;  // ready for the next launch on this stream
    }
}

// LDS layout: [P matrices: n_mat * C * K * K][exp workspace: n_mat * C * K][per-category
// site values: C * 64 (EDGE_LNL)]
__host__ __device__ inline int edge_mats(int mode) { return mode == EDGE_DERIV ? 4 : 2; }

template <int K, int MODE>
__global__ void __launch_bounds__(kLanes) k_edge(EdgeArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int C = a.C;
    const int nm = edge_mats(MODE);
    double *Pl = lds;
    double *ex = Pl + (size_t)nm * C * K * K;
    double *swl = ex + (size_t)nm * C * K;
    const int tile = blockIdx.x, l = threadIdx.x;
    const int64_t site = (int64_t)tile * kLanes + l;
    const int64_t site_c = site < a.S ? site : a.S - 1;
    const int nwt = a.n_tiles * C;

    if constexpr (MODE == EDGE_UPDATE) {
        for (int o = 0; o < a.n_ops; ++o) {
            const EdgeOp op = a.op[o];
            const double t[4] = {op.t_a, op.t_b, 0.0, 0.0};
            const int ord[4] = {0, 0, 0, 0};
            __syncthreads();  // the previous op's P are consumed
            build_p<K>(a, Pl, ex, 2, t, ord);
            for (int c = 0; c < C; ++c) {
                double va[K], vb[K], x[K], y[K], sa, sb, cml;
                node_vec<K>(a, op.a, c, tile, l, site_c, va, sa);
                node_vec<K>(a, op.b, c, tile, l, site_c, vb, sb);
                matvec_l<K>(Pl + (size_t)c * K * K, va, x);
                matvec_l<K>(Pl + (size_t)(C + c) * K * K, vb, y);
#pragma unroll
                for (int i = 0; i < K; ++i) x[i] = x[i] * y[i];
                rescale<K>(x, sa, sb, cml);
                const size_t row = (size_t)c * a.n_tiles + tile;
                store_site<K>(a.clv + (size_t)op.par_slot * a.slot_stride + row * K * kLanes, l,
                              x);
                a.scale[(size_t)op.par_slot * a.sstride + row * kLanes + l] = cml;
                // the slot's scalers may now be non-zero (k_prune skip-zero protocol)
                if (l == 0) a.sflag[(size_t)op.par_slot * nwt + tile * C + c] = 1u;
            }
            // the next op may read this parent: every lane reads only its own site, so no
            // cross-lane hazard exists; the stores are ordered before the next op's loads
            __threadfence_block();
        }
        return;
    } else {
        const EdgeOp op = a.op[0];
        const double t[4] = {0.0, op.t_b, op.t_b, op.t_b};
        const int ord[4] = {0, 0, 1, 2};
        build_p<K>(a, Pl, ex, nm, t, ord);
        const bool valid = site < a.S;
        double v0 = 0.0, v1 = 0.0, v2 = 0.0;
        // EDGE_DERIV: online mixture over categories, L = sum_c w_c e^{l_c - m}
        double mx = -INFINITY, L = 0.0, N1 = 0.0, N2 = 0.0;
        for (int c = 0; c < C; ++c) {
            double va[K], vb[K], x[K], y[K], sa, sb;
            node_vec<K>(a, op.a, c, tile, l, site_c, va, sa);
            node_vec<K>(a, op.b, c, tile, l, site_c, vb, sb);
            matvec_l<K>(Pl + (size_t)c * K * K, va, x);
            matvec_l<K>(Pl + (size_t)(C + c) * K * K, vb, y);
            if constexpr (MODE == EDGE_LNL) {
                double out[K], cml;
#pragma unroll
                for (int i = 0; i < K; ++i) out[i] = x[i] * y[i];
                rescale<K>(out, sa, sb, cml);
                const size_t row = (size_t)c * a.n_tiles + tile;
                store_site<K>(a.root_clv + row * K * kLanes, l, out);
                a.root_scale[row * kLanes + l] = cml;
                if (l == 0) a.sflag[(size_t)a.n_store * nwt + tile * C + c] = 1u;
                double f = 0.0;
#pragma unroll
                for (int i = 0; i < K; ++i) f = fma(out[i], a.pi[i], f);
                swl[c * kLanes + l] = ((f > 0.0) ? log(f) + cml : -INFINITY) + a.logw[c];
            } else {
                double yd[K], yd2[K];
                matvec_l<K>(Pl + (size_t)(2 * C + c) * K * K, vb, yd);
                matvec_l<K>(Pl + (size_t)(3 * C + c) * K * K, vb, yd2);
                double f = 0.0, f1 = 0.0, f2 = 0.0;
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const double px = a.pi[i] * x[i];
                    f = fma(px, y[i], f);
                    f1 = fma(px, yd[i], f1);
                    f2 = fma(px, yd2[i], f2);
                }
                if (f > 0.0) {
                    const double lc = log(f) + sa + sb + a.logw[c];
                    const double g1 = f1 / f, g2 = f2 / f;
                    if (lc > mx) {
                        const double sc = exp(mx - lc);  // 0 for the first category
                        L = L * sc + 1.0;
                        N1 = N1 * sc + g1;
                        N2 = N2 * sc + g2;
                        mx = lc;
                    } else {
                        const double e = exp(lc - mx);
                        L += e;
                        N1 += e * g1;
                        N2 += e * g2;
                    }
                }
            }
        }
        if constexpr (MODE == EDGE_LNL) {
            if (valid) {
                const double sl = lse64(swl + l, C);
                a.site_lnl[site] = sl;
                v0 = a.pattern_w[site] * sl;
            }
        } else if (valid) {
            const double w = a.pattern_w[site];
            if (L > 0.0) {
                const double d1 = N1 / L;
                v0 = w * (mx + log(L));
                v1 = w * d1;
                v2 = w * (N2 / L - d1 * d1);
            } else if (w != 0.0) {
                v0 = -INFINITY;  // every category has f = 0 (lnl_node's -inf)
            }
        }
        grid_reduce3(a, v0, v1, v2);
    }
}

// ---- stateless lnl_branch / lnl_branch_derivs (numba_likelihood_engine.py:49-79) ----
template <int M>
__global__ void __launch_bounds__(256)
    k_lnl_branch(int K, int64_t E, int n_p, const int32_t *__restrict__ pidx,
                 const double *__restrict__ probs, const double *__restrict__ pi,
                 const double *__restrict__ pa, const double *__restrict__ pb,
                 const double *__restrict__ sa, const double *__restrict__ sb,
                 double *__restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int p = pidx ? pidx[e] : (int)(e % n_p);
    const double *A = pa + e * K, *B = pb + e * K;
    double f[M];
    for (int m = 0; m < M; ++m) {
        // np.sum(np.dot(probs[m], partials_a) * partials_b * pi)
        const double *P = probs + ((size_t)p * M + m) * K * K;
        double acc = 0.0;
        for (int i = 0; i < K; ++i) {
            double x = 0.0;
            for (int j = 0; j < K; ++j) x = fma(P[i * K + j], A[j], x);
            acc += x * B[i] * pi[i];
        }
        f[m] = acc;
    }
    if constexpr (M == 1) {
        out[e] = log(f[0]) + sa[e] + sb[e];
    } else {
        out[3 * e] = log(f[0]) + sa[e] + sb[e];
        out[3 * e + 1] = f[1] / f[0];
        out[3 * e + 2] = ((f[2] * f[0]) - (f[1] * f[1])) / (f[0] * f[0]);
    }
}

template <int K>
int launch_edge_k(hipStream_t st, int mode, const EdgeArgs &a, size_t lds) {
    const dim3 grid((unsigned)a.n_tiles), block(kLanes);
    switch (mode) {
        case EDGE_UPDATE: hipLaunchKernelGGL((k_edge<K, EDGE_UPDATE>), grid, block, lds, st, a); break;
        case EDGE_LNL: hipLaunchKernelGGL((k_edge<K, EDGE_LNL>), grid, block, lds, st, a); break;
        case EDGE_DERIV: hipLaunchKernelGGL((k_edge<K, EDGE_DERIV>), grid, block, lds, st, a); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

}  // namespace

size_t edge_lds_bytes(int mode, int K, int C) {
    const size_t nm = edge_mats(mode);
    size_t d = nm * C * K * K + nm * C * K;
    if (mode == EDGE_LNL) d += (size_t)C * kLanes;
    return d * sizeof(double);
}

int launch_edge(hipStream_t st, int mode, const EdgeArgs &a) {
    const size_t lds = edge_lds_bytes(mode, a.K, a.C);
    if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
    switch (a.K) {
        case 2: return launch_edge_k<2>(st, mode, a, lds);
        case 4: return launch_edge_k<4>(st, mode, a, lds);
        case 20: return launch_edge_k<20>(st, mode, a, lds);
        default: return (int)hipErrorInvalidValue;
    }
}

int launch_lnl_branch(hipStream_t st, int K, int M, int64_t E, int n_p, const int32_t *pidx,
                      const double *probs, const double *pi, const double *pa,
                      const double *pb, const double *sa, const double *sb, double *out) {
    if (E == 0) return 0;
    const dim3 grid((unsigned)((E + 255) / 256)), block(256);
    if (M == 1)
        hipLaunchKernelGGL(k_lnl_branch<1>, grid, block, 0, st, K, E, n_p, pidx, probs, pi, pa,
                           pb, sa, sb, out);
    else if (M == 3)
        hipLaunchKernelGGL(k_lnl_branch<3>, grid, block, 0, st, K, E, n_p, pidx, probs, pi, pa,
                           pb, sa, sb, out);
    else
        return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
}

}  // namespace pu
