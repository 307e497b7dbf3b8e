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
// Mapping: a workgroup is one 64-site tile; wave w owns rate category w (categories are
// strided over at most 8 waves), a lane is a site, and every wave reads one contiguous
// category row of the tiled slot layout of pu_kernels.hip.  The categories of a site meet
// in LDS, where wave 0 mixes them.  The P matrices an edge needs are computed
// once per workgroup into LDS from the eigen-decomposition, with the arithmetic of
// k_pmatrix (so P(0) and P(t) are bit-identical to the traversal's), and read as LDS
// broadcasts.  The lnL / derivative sums are reduced in one launch: every workgroup writes
// its partial sums, and the last workgroup to finish (atomic ticket) adds them in a fixed
// order -- bitwise repeatable, no second launch, no spinning.
#include "pu_internal.h"
#include "pu_minimise.h"

#include <math.h>

#include <algorithm>

namespace pu {

namespace {

constexpr double kScaleThreshold = 0x1p-128;  // numba_likelihood_engine.py:7
constexpr int kLanes = 64;

typedef double dbl2 __attribute__((ext_vector_type(2)));

// ---- site vectors in the tiled slot layout (pu_kernels.hip k_untile / k_untile_aa) ----
template <int K>
__device__ __forceinline__ int tiled_index(int i, int l) {
    if constexpr (K == 20) {  // [wave 4][aa_row_off]: lane (g, s16) of wave w, rows g, g+4..
        const int w = l >> 4, s16 = l & 15;
        const int g = i < 16 ? (i & 3) : i - 16, r = i < 16 ? (i >> 2) : 4;
        return w * 5 * 64 + aa_row_off(r, g * 16 + s16);
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
        const size_t row = layout_row(K, a.C, a.tile_pitch, cat, tile);
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

// Waves per workgroup: one rate category per wave when C <= kMaxWaves (a wave's 64 sites of
// one category row are contiguous in the tiled layout), otherwise waves stride the categories.
constexpr int kMaxWaves = 8;
__host__ __device__ inline int edge_waves(int C) { return C < kMaxWaves ? C : kMaxWaves; }
__host__ __device__ inline int edge_mats(int mode) { return mode == EDGE_DERIV ? 4 : 2; }

// LDS of one workgroup (doubles): [evecs K*K][ivecs K*K][evals K][rates C][P matrices
// n_mat*C*K*K][exp workspace n_mat*C*K][per-(category, site) values: C*64*(1 | 4)][wave
// partial sums 3*kMaxWaves]
struct EdgeLds {
    size_t evecs, ivecs, evals, rates, P, ex, vals, red, total;
    __host__ __device__ EdgeLds(int mode, int K, int C) {
        const int nm = edge_mats(mode);
        evecs = 0;
        ivecs = evecs + (size_t)K * K;
        evals = ivecs + (size_t)K * K;
        rates = evals + K;
        P = (rates + C + 1) & ~size_t(1);  // 16-byte aligned matrices
        ex = P + (size_t)nm * C * K * K;
        vals = ex + (size_t)nm * C * K;
        red = vals + (mode == EDGE_UPDATE ? 0 : (size_t)C * 64 * (mode == EDGE_DERIV ? 4 : 1));
        total = red + 3 * kMaxWaves;
    }
};

// Workgroup barrier for LDS traffic only: waits for this wave's LDS operations, not for its
// in-flight global loads (__syncthreads would also wait for those, i.e. for the CLV
// prefetch issued before the P build)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// P matrices into LDS: n_mat matrices per category, matrix m of category c at
// P[(m * C + c) * K * K].  Matrix m uses length t[m] and derivative order ord[m]:
// evecs diag(x^ord e^{l t r}) ivecs with x = l r (k_pmatrix's arithmetic for ord 0).
template <int K>
__device__ void build_p(const EdgeArgs &a, double *lds, const EdgeLds &L, int n_mat,
                        const double (&t)[4], const int (&ord)[4], const double *host = nullptr) {
    const int C = a.C, nt = blockDim.x;
    if (host) {  // host-supplied matrices (non-reversible models), same [m][c][K][K] order
        double *P = lds + L.P;
        for (int idx = threadIdx.x; idx < n_mat * C * K * K; idx += nt) P[idx] = host[idx];
        lds_barrier();
        return;
    }
    const double *ev = lds + L.evecs, *iv = lds + L.ivecs, *el = lds + L.evals,
                 *rt = lds + L.rates;
    double *ex = lds + L.ex, *P = lds + L.P;
    for (int idx = threadIdx.x; idx < n_mat * C * K; idx += nt) {
        const int k = idx % K, mc = idx / K, c = mc % C, m = mc / C;
        const double r = rt[c];
        const double tt = t[m] * r;
        double e = exp(el[k] * tt);
        if (ord[m] > 0) {
            const double x = el[k] * r;
            e = ord[m] == 1 ? x * e : (x * x) * e;
        }
        ex[idx] = e;
    }
    lds_barrier();
    for (int idx = threadIdx.x; idx < n_mat * C * K * K; idx += nt) {
        const int ij = idx % (K * K), mc = idx / (K * K);
        const int i = ij / K, j = ij - i * K;
        const double *e = ex + mc * K;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) acc = fma(ev[i * K + k] * e[k], iv[k * K + j], acc);
        P[idx] = acc;
    }
    lds_barrier();
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Sum the per-workgroup partials: the last workgroup to arrive adds all of them in a fixed
// order (partial i by thread i % blockDim, then a fixed wave / workgroup tree), so the
// result does not depend on which workgroup finished last.  Called by every thread;
// v0..v2 are the workgroup's sums (valid in thread 0).
__device__ void grid_reduce3(const EdgeArgs &a, double *red, double v0, double v1,
                             double v2) {
    __shared__ unsigned int ticket;
    if (threadIdx.x == 0) {
        double *p = a.block_part + 3 * (size_t)blockIdx.x;
        p[0] = v0;
        p[1] = v1;
        p[2] = v2;
        __threadfence();  // release (agent scope): the partials are visible device-wide
        ticket = atomicAdd(a.counter, 1u);
    }
    __syncthreads();
    if (ticket != gridDim.x - 1) return;
    __threadfence();  // acquire (agent scope): no stale partials in this CU's caches
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
        const double *p = a.block_part + 3 * (size_t)b;
        s0 += p[0];
        s1 += p[1];
        s2 += p[2];
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[3 * w] = s0;
        red[3 * w + 1] = s1;
        red[3 * w + 2] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double r0 = 0.0, r1 = 0.0, r2 = 0.0;
        for (int k = 0; k < nw; ++k) {
            r0 += red[3 * k];
            r1 += red[3 * k + 1];
            r2 += red[3 * k + 2];
        }
        a.result[0] = r0;
        a.result[1] = r1;
        a.result[2] = r2;
        *a.counter = 0u;  // ready for the next launch on this stream
    }
}

// One workgroup = one 64-site tile; wave w handles categories w, w + nw, ...  (one each
// when C <= kMaxWaves).  EDGE_LNL / EDGE_DERIV leave per-(category, site) values in LDS and
// wave 0 combines the categories of its 64 sites.
template <int K, int MODE>
__global__ void __launch_bounds__(64 * kMaxWaves) k_edge(EdgeArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int C = a.C;
    const EdgeLds L(MODE, K, C);
    const int tile = blockIdx.x, l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
    const int64_t site = (int64_t)tile * kLanes + l;
    const int64_t site_c = site < a.S ? site : a.S - 1;
    const int nwt = a.n_tiles * C;
    double *Pl = lds + L.P, *vals = lds + L.vals;

    // the model, staged once for the P builds.  DNA edge evaluations request it through the
    // scalar unit after the wave's first CLV loads (below), so the LDS barrier before the
    // P build waits for it (lgkmcnt) and not for those loads (vmcnt); the other cases stage it
    // first with coalesced vector loads
    constexpr bool late_model = K <= 4 && MODE != EDGE_UPDATE;
    auto stage_model_scalar = [&]() {
        if (w == 0) {  // wave-uniform indices: scalar loads, lane 0 writes
#pragma unroll
            for (int i = 0; i < K * K; ++i) {
                const double e = a.evecs[i], v = a.ivecs[i];
                if (l == 0) {
                    lds[L.evecs + i] = e;
                    lds[L.ivecs + i] = v;
                }
            }
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const double e = a.evals[i];
                if (l == 0) lds[L.evals + i] = e;
            }
            for (int i = 0; i < C; ++i) {
                const double r = a.rates[i];
                if (l == 0) lds[L.rates + i] = r;
            }
        }
    };
    // matrices in the launch (EdgeArgs::hp, K <= 4): EDGE_DERIV P(0), P(t), dP, d2P; EDGE_UPDATE
    // P(t_a), P(t_b) of each of at most two ops -- read through the scalar unit
    const bool inline_p = K <= 4 && a.inline_p && MODE != EDGE_LNL;
    if (!late_model && !inline_p) {
        for (int i = threadIdx.x; i < K * K; i += blockDim.x) {
            lds[L.evecs + i] = a.evecs[i];
            lds[L.ivecs + i] = a.ivecs[i];
        }
        for (int i = threadIdx.x; i < K; i += blockDim.x) lds[L.evals + i] = a.evals[i];
        for (int i = threadIdx.x; i < C; i += blockDim.x) lds[L.rates + i] = a.rates[i];
        __syncthreads();  // (nothing is in flight yet)
    }

    if constexpr (MODE == EDGE_UPDATE) {
        for (int o = 0; o < a.n_ops; ++o) {
            const EdgeOp op = a.op[o];
            const double t[4] = {op.t_a, op.t_b, 0.0, 0.0};
            const int ord[4] = {0, 0, 0, 0};
            if (!inline_p) {
                if (o > 0) __syncthreads();  // the previous op's P are consumed
                build_p<K>(a, lds, L, 2, t, ord,
                           a.pmats ? a.pmats + (size_t)o * 2 * C * K * K : nullptr);
            }
            for (int c = w; c < C; c += nw) {
                double va[K], vb[K], x[K], y[K], sa, sb, cml;
                node_vec<K>(a, op.a, c, tile, l, site_c, va, sa);
                node_vec<K>(a, op.b, c, tile, l, site_c, vb, sb);
                if (inline_p) {
                    const double *hp = a.hp + (size_t)o * 2 * C * K * K;
                    matvec_l<K>(hp + (size_t)c * K * K, va, x);
                    matvec_l<K>(hp + (size_t)(C + c) * K * K, vb, y);
                } else {
                    matvec_l<K>(Pl + (size_t)c * K * K, va, x);
                    matvec_l<K>(Pl + (size_t)(C + c) * K * K, vb, y);
                }
#pragma unroll
                for (int i = 0; i < K; ++i) x[i] = x[i] * y[i];
                rescale<K>(x, sa, sb, cml);
                const size_t row = layout_row(K, C, a.tile_pitch, c, tile);
                store_site<K>(a.clv + (size_t)op.par_slot * a.slot_stride + row * K * kLanes, l,
                              x);
                a.scale[(size_t)op.par_slot * a.sstride + row * kLanes + l] = cml;
                // the slot's scalers may now be non-zero (k_prune skip-zero protocol)
                if (l == 0) a.sflag[(size_t)op.par_slot * nwt + tile * C + c] = 1u;
            }
            // a later op of this launch reads this parent at the same (site, category),
            // i.e. in the same lane of the same wave: program order covers it
        }
        return;
    } else {
        const EdgeOp op = a.op[0];
        const double t[4] = {0.0, op.t_b, op.t_b, op.t_b};
        const int ord[4] = {0, 0, 1, 2};
        // the wave's first category is loaded before the P build, so the HBM latency
        // overlaps it
        double va[K], vb[K], sa = 0.0, sb = 0.0;
        if (w < C) {
            node_vec<K>(a, op.a, w, tile, l, site_c, va, sa);
            node_vec<K>(a, op.b, w, tile, l, site_c, vb, sb);
        }
        // EDGE_DERIV with K <= 4, C <= 4: the host put P(0), P(t), dP/dt, d2P/dt2 in the
        // kernel arguments: no model staging, no P build
        if (!inline_p) {
            if constexpr (late_model) {
                if (!a.pmats) {
                    stage_model_scalar();
                    lds_barrier();
                }
            }
            build_p<K>(a, lds, L, edge_mats(MODE), t, ord, a.pmats);
        }
        for (int c = w; c < C; c += nw) {
            if (c != w) {
                node_vec<K>(a, op.a, c, tile, l, site_c, va, sa);
                node_vec<K>(a, op.b, c, tile, l, site_c, vb, sb);
            }
            if constexpr (MODE == EDGE_LNL) {
                double x[K], y[K], out[K], cml;
                matvec_l<K>(Pl + (size_t)c * K * K, va, x);
                matvec_l<K>(Pl + (size_t)(C + c) * K * K, vb, y);
#pragma unroll
                for (int i = 0; i < K; ++i) out[i] = x[i] * y[i];
                rescale<K>(out, sa, sb, cml);
                const size_t row = layout_row(K, C, a.tile_pitch, c, tile);
                store_site<K>(a.root_clv + row * K * kLanes, l, out);
                a.root_scale[row * kLanes + l] = cml;
                if (l == 0) a.sflag[(size_t)a.n_store * nwt + tile * C + c] = 1u;
                double f = 0.0;
#pragma unroll
                for (int i = 0; i < K; ++i) f = fma(out[i], a.pi[i], f);
                vals[c * kLanes + l] = ((f > 0.0) ? log(f) + cml : -INFINITY) + a.logw[c];
            } else {
                // row by row: only the two child vectors stay in registers (K = 20 would
                // otherwise spill six K-vectors)
                double f = 0.0, f1 = 0.0, f2 = 0.0;
                auto mix = [&](const double *Pm) {
                    const double *P0 = Pm + (size_t)c * K * K, *P1 = Pm + (size_t)(C + c) * K * K,
                                 *P2 = Pm + (size_t)(2 * C + c) * K * K,
                                 *P3 = Pm + (size_t)(3 * C + c) * K * K;
                    constexpr int kRowUnroll = K > 4 ? 1 : K;  // K = 20: P reads stay in LDS
#pragma unroll kRowUnroll
                    for (int i = 0; i < K; ++i) {
                        double xi = 0.0, yi = 0.0, di = 0.0, ei = 0.0;
#pragma unroll
                        for (int j = 0; j < K; ++j) {
                            xi = fma(P0[i * K + j], va[j], xi);
                            yi = fma(P1[i * K + j], vb[j], yi);
                            di = fma(P2[i * K + j], vb[j], di);
                            ei = fma(P3[i * K + j], vb[j], ei);
                        }
                        const double px = a.pi[i] * xi;
                        f = fma(px, yi, f);
                        f1 = fma(px, di, f1);
                        f2 = fma(px, ei, f2);
                    }
                };
                if (inline_p)
                    mix(a.hp);
                else
                    mix(Pl);
                // linear domain: f, f', f'' and the category's log scaler; the site mixes
                // them with one log and two divisions (below) instead of C logs, 2C
                // divisions and C exponentials
                vals[c * kLanes + l] = f;
                vals[(C + c) * kLanes + l] = f1;
                vals[(2 * C + c) * kLanes + l] = f2;
                vals[(3 * C + c) * kLanes + l] = sa + sb;
            }
        }
        __syncthreads();
        double v0 = 0.0, v1 = 0.0, v2 = 0.0;
        if (w == 0 && site < a.S) {
            const double pw = a.pattern_w[site];
            if constexpr (MODE == EDGE_LNL) {
                const double sl = lse64(vals + l, C);
                a.site_lnl[site] = sl;
                v0 = pw * sl;
            } else {
                // per site: L = sum_c w_c f_c e^{s_c} = e^smax sum_c w_c f_c e^{s_c - smax}
                // (s_c = sa + sb, the category's log scaler: equal across categories unless a
                // child was rescaled, so the exponential is usually skipped), and
                // dlnL/dt = sum_c w_c f'_c e^{..} / sum_c w_c f_c e^{..}, likewise d2.
                // Only categories with f_c > 0 take part (lnl_node's -inf for the others,
                // numba_likelihood_engine.py:82-87): an all-zero CLV keeps an unrescaled
                // scaler, which must not set smax and underflow every other category's
                // weight (e.g. an invariant category under host matrices, P(0) = I)
                double smax = -INFINITY;
                for (int c = 0; c < C; ++c)
                    if (vals[c * kLanes + l] > 0.0)
                        smax = fmax(smax, vals[(3 * C + c) * kLanes + l]);
                double Ls = 0.0, N1 = 0.0, N2 = 0.0;
                for (int c = 0; c < C; ++c) {
                    if (!(vals[c * kLanes + l] > 0.0)) continue;
                    const double sc = vals[(3 * C + c) * kLanes + l];
                    const double we = a.weights[c] * (sc == smax ? 1.0 : exp(sc - smax));
                    Ls += we * vals[c * kLanes + l];
                    N1 += we * vals[(C + c) * kLanes + l];
                    N2 += we * vals[(2 * C + c) * kLanes + l];
                }
                if (Ls > 0.0) {
                    const double d1 = N1 / Ls;
                    v0 = pw * (smax + log(Ls));
                    v1 = pw * d1;
                    v2 = pw * (N2 / Ls - d1 * d1);
                } else if (pw != 0.0) {
                    v0 = -INFINITY;  // every category has f = 0 (lnl_node's -inf)
                }
            }
        }
        // workgroup sum = wave 0's sum (the other waves contribute 0)
        if (w == 0) {
            v0 = wave_sum(v0);
            v1 = wave_sum(v1);
            v2 = wave_sum(v2);
        }
        if (a.two_pass) {  // partials only; k_edge_sum adds them (second launch)
            if (threadIdx.x == 0) {
                double *p = a.block_part + 3 * (size_t)blockIdx.x;
                p[0] = v0;
                p[1] = v1;
                p[2] = v2;
            }
            return;
        }
        grid_reduce3(a, lds + L.red, v0, v1, v2);
    }
}

// second launch of the two-pass reduction: the same fixed order as grid_reduce3
__global__ void __launch_bounds__(256) k_edge_sum(const double *__restrict__ part, int n,
                                                  double *__restrict__ result, double seq) {
    __shared__ double red[3 * 4];
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int b = threadIdx.x; b < n; b += blockDim.x) {
        s0 += part[3 * b];
        s1 += part[3 * b + 1];
        s2 += part[3 * b + 2];
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[3 * w] = s0;
        red[3 * w + 1] = s1;
        red[3 * w + 2] = s2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double r0 = 0.0, r1 = 0.0, r2 = 0.0;
        for (int k = 0; k < 4; ++k) {
            r0 += red[3 * k];
            r1 += red[3 * k + 1];
            r2 += red[3 * k + 2];
        }
        result[0] = r0;
        result[1] = r1;
        result[2] = r2;
        if (seq != 0.0) {
            // the host polls result[3] (mapped memory) instead of synchronising the stream:
            // the sums reach host memory before the sequence number does
            __threadfence_system();
            __hip_atomic_store(result + 3, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
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

// Ascertainment-bias correction after a traversal or an edge evaluation (AscArgs).  Every
// workgroup recomputes the correction from the K dummy sites (K x C lnl_node values), then
// corrects its slice of the sitewise lnL; workgroup 0 corrects the total.
template <int K>
__global__ void __launch_bounds__(256) k_ascbias(AscArgs a) {
    __shared__ double sw[K * 64];
    __shared__ double corr;
    const int C = a.C;
    for (int e = threadIdx.x; e < K * C; e += blockDim.x) {
        const int k = e / C, c = e - k * C;  // [state][category], as swlnls[-N:]
        const int64_t site = a.first + k;
        const int tile = (int)(site / kLanes), l = (int)(site % kLanes);
        const size_t row = layout_row(K, C, a.tile_pitch, c, tile);
        double v[K];
        load_site<K>(a.root_clv + row * K * kLanes, l, v);
        double f = 0.0;
#pragma unroll
        for (int i = 0; i < K; ++i) f = fma(v[i], a.pi[i], f);
        sw[e] = (f > 0.0) ? log(f) + a.root_scale[row * kLanes + l] : -INFINITY;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double x;
        if (a.mode == 1) {  // logsumexp over all K x C values (scipy form)
            double amax = -INFINITY, m = 0.0, t = 0.0;
            for (int e = 0; e < K * C; ++e) amax = sw[e] > amax ? sw[e] : amax;
            const double shift = isfinite(amax) ? amax : 0.0;
            for (int e = 0; e < K * C; ++e) {
                if (sw[e] == amax)
                    m += 1.0;
                else
                    t += exp(sw[e] - shift);
            }
            if (t != 0.0) t /= m;
            x = log1p(t) + log(m) + amax;
        } else {  // sum over states of the weighted site likelihoods
            double mx = -INFINITY, t = 0.0;
            for (int k = 0; k < K; ++k) mx = fmax(mx, a.site_lnl[a.first + k]);
            for (int k = 0; k < K; ++k) t += exp(a.site_lnl[a.first + k] - mx);
            x = mx + log(t);
        }
        corr = log(1.0 - exp(x));  // tree_model.py:213
    }
    __syncthreads();
    const double cr = corr;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < a.first;
         s += (int64_t)gridDim.x * blockDim.x)
        a.site_lnl[s] -= cr;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *a.lnl -= cr * a.sum_w;
        *a.corr = cr;
    }
}

// ---- device-side Newton on one edge (NewtonArgs, pu_internal.h; r06) ----
// pu_edge.cpp's newton() -- the same steps, safeguards and stopping rule -- in one persistent
// launch.  An evaluation needs, per (site, category), f = sum_i pi_i (P(0) a)_i (P(t) b)_i and
// its two t-derivatives.  With P(t) = V diag(e^{l r t}) V^-1 (the eigen form k_pmatrix and
// build_p use) that is f = sum_k c_k e^{l_k r t}, f' = sum_k c_k (l_k r) e^{..}, f'' = sum_k
// c_k (l_k r)^2 e^{..}, c_k = [V^T (pi o P(0) a)]_k [V^-1 b]_k: K coefficients per (site,
// category), computed once per launch and held in registers, so an evaluation reads no CLV
// and builds no matrix (the eigen-space "sum table" of branch-length optimisers).  Rounding
// differs from k_edge's direct products by ~1e-16 relative per site (tests: 1e-12 on lnL and
// derivatives, the same optimum to 1e-9).  A wave owns `tpw` whole tiles, all categories;
// the categories of a site are mixed in registers exactly as k_edge does.
constexpr double kNewtonMinLen = 1e-8, kNewtonMaxLen = 100.0;  // pu_edge.cpp kMinLen / kMaxLen
constexpr int kNewtonMaxC = 4;   // categories held per lane
constexpr int kNewtonTpw = 2;    // tiles per wave held in registers at most (template TPW)
constexpr int kNewtonWaves = 4;  // 256-thread workgroups

__device__ __forceinline__ void st_agent(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A 64-lane sum on the DPP crossbar (k_edge_newton's evaluation sums): quad swaps, half-row and
// row mirrors, then the row broadcasts 15 / 31 -- six dependent steps of two v_mov_dpp and one add
// (wave_sum's __shfl_xor steps are ds_bpermute round trips through the LDS unit: 1.8 us for the
// three sums of an evaluation, r06 stamps).  The total lands in lane 63 and is read from there.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_take(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWS, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_total(double v) {
    v += dpp_take<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
    v += dpp_take<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
    v += dpp_take<0x141, 0xf>(v);  // row_half_mirror
    v += dpp_take<0x140, 0xf>(v);  // row_mirror: every lane of a row holds the row's sum
    v += dpp_take<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
    v += dpp_take<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3: lane 63 holds the total
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// TPW tiles per wave: 1 at up to 3 workgroups per CU (<= 168 VGPRs, no spills), 2 at 2
template <int K, int TPW>
__global__ void __launch_bounds__(64 * kNewtonWaves, TPW == 1 ? 3 : 2)
    k_edge_newton(EdgeArgs a, NewtonArgs n) {
    __shared__ double model[2 * K * K + K + kNewtonMaxC + K];  // evecs, ivecs, evals, rates, pi
    __shared__ double p0[kNewtonMaxC * K * K];                 // P(0) per category
    __shared__ double egq[3 * kNewtonMaxC * K];                // e, (l r) e, (l r)^2 e
    __shared__ double vsum[3 * 256];                           // the combiner's slot sums
    __shared__ double wred[3 * kNewtonWaves];                  // the waves' sums
    __shared__ double sh_next[2];
    __shared__ double sh_nt[7];  // the combiner's newton() state: t, lnL, d1, d2, next t, iterations, halvings
    __shared__ MinState sh_ms;   // ... or brent's / dbrent's (NewtonArgs::mode)
    __shared__ double sh_mpar[4];  // their lo, t0, hi, tol
    __shared__ double sh_ss[TPW * kNewtonMaxC * 256];         // log scalers per tile, category, lane
    __shared__ double sh_we[TPW * kNewtonMaxC * 256];         // w_c e^{s_c - smax} per tile, category, lane
    __shared__ double sh_smx[TPW * 256], sh_pw[TPW * 256];     // max scaler, pattern weight per site
    const int C = a.C;
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double *ev = model, *iv = model + K * K, *el = model + 2 * K * K, *rt = el + K, *pi = rt + kNewtonMaxC;
    for (int i = threadIdx.x; i < K * K; i += blockDim.x) {
        ev[i] = a.evecs[i];
        iv[i] = a.ivecs[i];
    }
    for (int i = threadIdx.x; i < K; i += blockDim.x) {
        el[i] = a.evals[i];
        pi[i] = a.pi[i];
    }
    for (int i = threadIdx.x; i < C; i += blockDim.x) rt[i] = a.rates[i];
    if (threadIdx.x == 0) {
        sh_mpar[0] = n.lo;
        sh_mpar[1] = n.t0;
        sh_mpar[2] = n.hi;
        sh_mpar[3] = n.tol;
    }
    __syncthreads();
    // P(0) per category with build_p's arithmetic (e = exp(l * (0 * r)))
    for (int idx = threadIdx.x; idx < C * K * K; idx += blockDim.x) {
        const int ij = idx % (K * K), c = idx / (K * K), i = ij / K, j = ij - i * K;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) acc = fma(ev[i * K + k] * exp(el[k] * (0.0 * rt[c])), iv[k * K + j], acc);
        p0[idx] = acc;
    }
    __syncthreads();
    // this wave's tiles: c_k and the log scaler per category, in registers for the launch
    // per site, also (in LDS) the pattern weight and k_edge's category weights w_c e^{s_c - smax}
    // for the case every f_c > 0 (always, short of underflow), so an evaluation reads no global
    // memory and takes no exp; the log scalers are kept for the other case
    const EdgeOp op = a.op[0];
    double cf[TPW][kNewtonMaxC][K];
    const int tile_w = (blockIdx.x * kNewtonWaves + w) * n.tpw;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
        const int tile = tile_w + j;
        double ss[kNewtonMaxC];
#pragma unroll
        for (int c = 0; c < kNewtonMaxC; ++c) {
            ss[c] = 0.0;
#pragma unroll
            for (int k = 0; k < K; ++k) cf[j][c][k] = 0.0;
            if (j < n.tpw && tile < a.n_tiles && c < C) {
                const int64_t site = (int64_t)tile * kLanes + l;
                const int64_t site_c = site < a.S ? site : a.S - 1;
                double va[K], vb[K], sa, sb, xa[K];
                node_vec<K>(a, op.a, c, tile, l, site_c, va, sa);
                node_vec<K>(a, op.b, c, tile, l, site_c, vb, sb);
                matvec_l<K>(p0 + c * K * K, va, xa);  // k_edge's x = P(0) a
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    double A = 0.0, B = 0.0;
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        A = fma(pi[i] * xa[i], ev[i * K + k], A);
                        B = fma(iv[k * K + i], vb[i], B);
                    }
                    cf[j][c][k] = A * B;
                }
                ss[c] = sa + sb;
            }
            sh_ss[(j * kNewtonMaxC + c) * 256 + threadIdx.x] = ss[c];
        }
        double m = -INFINITY;
#pragma unroll
        for (int c = 0; c < kNewtonMaxC; ++c)
            if (c < C) m = fmax(m, ss[c]);
        sh_smx[j * 256 + threadIdx.x] = m;
#pragma unroll
        for (int c = 0; c < kNewtonMaxC; ++c)
            sh_we[(j * kNewtonMaxC + c) * 256 + threadIdx.x] =
                c < C ? a.weights[c] * (ss[c] == m ? 1.0 : exp(ss[c] - m)) : 0.0;
        const int64_t site = (int64_t)tile * kLanes + l;
        sh_pw[j * 256 + threadIdx.x] = j < n.tpw && tile < a.n_tiles && site < a.S ? a.pattern_w[site] : 0.0;
    }
    double x = n.t0;
    auto stamp = [&](unsigned e, int k) {  // debug stamps (PU_NT_TIMING)
        if (n.timing && (int)e < n.n_timing) n.timing[8 * e + k] = __builtin_amdgcn_s_memrealtime();
    };
    for (unsigned evn = 0;; ++evn) {
        if (blockIdx.x == 0 && threadIdx.x == 0) stamp(evn, 0);
        // e^{l r t} and its two t-derivative factors per (category, state), build_p's forms
        if (threadIdx.x < C * K) {
            const int c = threadIdx.x / K, k = threadIdx.x - c * K;
            const double r = rt[c];
            const double e = exp(el[k] * (x * r));
            const double xx = el[k] * r;
            egq[threadIdx.x] = e;
            egq[C * K + threadIdx.x] = xx * e;
            egq[2 * C * K + threadIdx.x] = (xx * xx) * e;
        }
        __syncthreads();
        if (blockIdx.x == 0 && threadIdx.x == 0) stamp(evn, 5);
        double wsum[3] = {0.0, 0.0, 0.0};  // this wave's tiles, in order
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
            const int tile = tile_w + j;
            if (j >= n.tpw || tile >= a.n_tiles) break;  // wave-uniform
            const int64_t site = (int64_t)tile * kLanes + l;
            double f[kNewtonMaxC], f1[kNewtonMaxC], f2[kNewtonMaxC];
#pragma unroll
            for (int c = 0; c < kNewtonMaxC; ++c) {
                f[c] = f1[c] = f2[c] = 0.0;
                if (c < C) {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        f[c] = fma(cf[j][c][k], egq[c * K + k], f[c]);
                        f1[c] = fma(cf[j][c][k], egq[C * K + c * K + k], f1[c]);
                        f2[c] = fma(cf[j][c][k], egq[2 * C * K + c * K + k], f2[c]);
                    }
                }
            }
            double v0 = 0.0, v1 = 0.0, v2 = 0.0;
            if (site < a.S) {  // k_edge's per-site category mix
                const double pw = sh_pw[j * 256 + threadIdx.x];
                bool allpos = true;
#pragma unroll
                for (int c = 0; c < kNewtonMaxC; ++c)
                    if (c < C) allpos &= f[c] > 0.0;
                double smax = sh_smx[j * 256 + threadIdx.x], Ls = 0.0, N1 = 0.0, N2 = 0.0;
                if (allpos) {  // the precomputed weights: k_edge's expression, the same values
                    const double *wej = sh_we + j * kNewtonMaxC * 256 + threadIdx.x;
#pragma unroll
                    for (int c = 0; c < kNewtonMaxC; ++c) {
                        if (c >= C) continue;
                        const double we = wej[c * 256];
                        Ls += we * f[c];
                        N1 += we * f1[c];
                        N2 += we * f2[c];
                    }
                } else {
                    const double *ssj = sh_ss + j * kNewtonMaxC * 256 + threadIdx.x;
                    smax = -INFINITY;
                    for (int c = 0; c < C; ++c)
                        if (f[c] > 0.0) smax = fmax(smax, ssj[c * 256]);
                    for (int c = 0; c < C; ++c) {
                        if (!(f[c] > 0.0)) continue;
                        const double sc = ssj[c * 256];
                        const double we = a.weights[c] * (sc == smax ? 1.0 : exp(sc - smax));
                        Ls += we * f[c];
                        N1 += we * f1[c];
                        N2 += we * f2[c];
                    }
                }
                if (Ls > 0.0) {
                    const double d1 = N1 / Ls;
                    v0 = pw * (smax + log(Ls));
                    v1 = pw * d1;
                    v2 = pw * (N2 / Ls - d1 * d1);
                } else if (pw != 0.0) {
                    v0 = -INFINITY;
                }
            }
            wsum[0] += wave_total(v0);
            wsum[1] += wave_total(v1);
            wsum[2] += wave_total(v2);
        }
        // the workgroup's sums, waves in order, into its 64-byte slot: six 8-byte words, each a
        // 32-bit half of a sum beside the evaluation's 32-bit generation, stored by six lanes.
        // An aligned 8-byte store is single-copy atomic, so a reader that sees the generation in
        // all six words holds the six halves of this evaluation -- no drain between data and
        // flag, no second read (the flag-in-word protocol of low-latency collectives)
        const unsigned ge = n.base + evn + 1;  // this evaluation's generation (< 2^31)
        if (blockIdx.x == 0 && threadIdx.x == 0) stamp(evn, 6);
        if (l == 0) {
            wred[3 * w] = wsum[0];
            wred[3 * w + 1] = wsum[1];
            wred[3 * w + 2] = wsum[2];
        }
        __syncthreads();
        if (blockIdx.x == 0 && threadIdx.x == 0) stamp(evn, 7);
        if (w == 0) {
            // every lane adds the waves' sums in the same order; lanes 0-5 store
            double s[3] = {0.0, 0.0, 0.0};
            for (int k = 0; k < kNewtonWaves; ++k) {
                s[0] += wred[3 * k];
                s[1] += wred[3 * k + 1];
                s[2] += wred[3 * k + 2];
            }
            if (l < 6) {
                const double v = l < 2 ? s[0] : (l < 4 ? s[1] : s[2]);
                const uint64_t bits = (uint64_t)__double_as_longlong(v);
                const uint64_t half = (l & 1) ? bits >> 32 : bits & 0xffffffffull;
                __hip_atomic_store(n.slots + 8 * (size_t)blockIdx.x + l, ((uint64_t)ge << 32) | half,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (blockIdx.x == 0 && l == 0) stamp(evn, 1);
        }
        if (blockIdx.x == 0) {
            // the combiner: thread v waits for slots v, v + 256, ... (six loads in flight per
            // poll), adds them in that fixed order, then four 64-wide xor trees
            double s0 = 0.0, s1 = 0.0, s2 = 0.0;
            bool ok = true;
            for (int b = threadIdx.x; b < (int)gridDim.x && ok; b += blockDim.x) {
                const uint64_t *sl = n.slots + 8 * (size_t)b;
                uint64_t q[6];
                for (unsigned spins = 0;;) {
                    bool all = true;
#pragma unroll
                    for (int i = 0; i < 6; ++i) {
                        q[i] = __hip_atomic_load(sl + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        all &= (unsigned)(q[i] >> 32) == ge;
                    }
                    if (all) break;
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins == n.spins) {
                        ok = false;
                        break;
                    }
                }
                if (ok) {
                    auto join = [](uint64_t lo, uint64_t hi) {
                        return __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
                    };
                    s0 += join(q[0], q[1]);
                    s1 += join(q[2], q[3]);
                    s2 += join(q[4], q[5]);
                }
            }
            vsum[threadIdx.x] = s0;
            vsum[256 + threadIdx.x] = s1;
            vsum[512 + threadIdx.x] = s2;
            const bool abort = __syncthreads_or(!ok);
            if (threadIdx.x == 0) stamp(evn, 2);
            if (w == 0) {
                // four strided entries per lane, then one DPP sum each
                const double r0 = wave_total(((vsum[l] + vsum[64 + l]) + vsum[128 + l]) + vsum[192 + l]);
                const double r1 = wave_total(((vsum[256 + l] + vsum[320 + l]) + vsum[384 + l]) + vsum[448 + l]);
                const double r2 = wave_total(((vsum[512 + l] + vsum[576 + l]) + vsum[640 + l]) + vsum[704 + l]);
                // newton()'s loop, one evaluation at a time; every lane of the wave holds the same
                // sums (read from lane 63) and so the same state
                // the state lives in LDS between evaluations (registers across the loop spill)
                double nt_t = sh_nt[0], nt_l = sh_nt[1], nt_d1 = sh_nt[2], nt_d2 = sh_nt[3];
                double nt_tn = sh_nt[4];
                int nt_it = (int)sh_nt[5], nt_h = (int)sh_nt[6];
                bool done = abort, plan = false;
                if (n.mode != PU_MIN_NEWTON) {
                    // brent / dbrent (pu_minimise.h, src/optimisation.pyx) on f = -lnL and
                    // f' = -dlnL/dt: one lane steps the state machine, whose state stays in LDS
                    double nx = 0.0;
                    int dn = 0;
                    if (l == 0 && !abort) {
                        if (evn == 0)  // (the bracket from LDS: kernel arguments held across
                                       // the loop for this one use spilled registers)
                            min_start(sh_ms, n.mode, sh_mpar[0], sh_mpar[1], sh_mpar[2], sh_mpar[3]);
                        nx = min_step(sh_ms, -r0, -r1);
                        dn = sh_ms.done;
                    }
                    nt_tn = __shfl(nx, 0);
                    done = abort || __shfl(dn, 0) != 0;
                } else if (abort) {
                } else if (evn == 0) {
                    nt_t = nt_tn = x;
                    nt_l = r0;
                    nt_d1 = r1;
                    nt_d2 = r2;
                    nt_it = nt_h = 0;
                    plan = true;
                } else if (r0 >= nt_l - 1e-13 * fabs(nt_l)) {  // accepted
                    const double dt = fabs(nt_tn - nt_t);
                    nt_t = nt_tn;
                    nt_l = r0;
                    nt_d1 = r1;
                    nt_d2 = r2;
                    ++nt_it;
                    if (dt <= n.tol * (1.0 + nt_t))
                        done = true;
                    else
                        plan = true;
                } else if (++nt_h >= 30) {
                    done = true;  // no ascent along this direction
                } else {
                    nt_tn = 0.5 * (nt_t + nt_tn);
                }
                if (plan) {
                    if (nt_it >= n.max_iter || !isfinite(nt_l)) {
                        done = true;
                    } else {
                        const double step = nt_d2 < 0.0 ? -nt_d1 / nt_d2
                                                         : (nt_d1 > 0.0 ? nt_t + 0.1 : -0.5 * nt_t);
                        nt_tn = fmin(fmax(nt_t + step, kNewtonMinLen), kNewtonMaxLen);
                        nt_h = 0;
                        if (nt_tn == nt_t) done = true;
                    }
                }
                if (done && l == 0) {  // the host's result, in mapped memory, then its sequence number
                    if (n.mode != PU_MIN_NEWTON) {  // out = (x, f(x), iterations); lnL = -f
                        n.res[0] = sh_ms.res_x;
                        n.res[1] = -sh_ms.res_f;
                        n.res[2] = -sh_ms.dx;
                        n.res[3] = 0.0;
                        n.res[4] = (double)sh_ms.res_it;
                    } else {
                        n.res[0] = nt_t;
                        n.res[1] = nt_l;
                        n.res[2] = nt_d1;
                        n.res[3] = nt_d2;
                        n.res[4] = (double)nt_it;
                    }
                    n.res[5] = (double)(evn + 1);
                    n.res[6] = abort ? 1.0 : 0.0;
                    __threadfence_system();
                    __hip_atomic_store(n.res + 7, n.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                // 8 publication lines of 64 bytes, one per group of pollers: the next length's two
                // halves, each beside flag = 2 generation + done (all ones: abort); lanes 0-15
                if (l < 16) {
                    const uint64_t bits = (uint64_t)__double_as_longlong(nt_tn);
                    const uint64_t half = (l & 1) ? bits >> 32 : bits & 0xffffffffull;
                    const unsigned flag = abort ? 0xffffffffu : 2u * ge + (done ? 1u : 0u);
                    int off = 8 * (l >> 1) + (l & 1);
                    asm volatile("" : "+v"(off));  // formed here: a hoisted 64-bit address spilled
                    __hip_atomic_store(n.pub + off, ((uint64_t)flag << 32) | half,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (l == 0) {
                    stamp(evn, 3);
                    sh_nt[0] = nt_t;
                    sh_nt[1] = nt_l;
                    sh_nt[2] = nt_d1;
                    sh_nt[3] = nt_d2;
                    sh_nt[4] = nt_tn;
                    sh_nt[5] = nt_it;
                    sh_nt[6] = nt_h;
                    sh_next[0] = nt_tn;
                    sh_next[1] = done ? 1.0 : 0.0;
                }
            }
            __syncthreads();
        } else {
            if (threadIdx.x == 0) {
                // ONE lane polls its group's line: both words, until both carry this generation
                const uint64_t *pb = n.pub + 8 * (blockIdx.x & 7);
                uint64_t q0, q1;
                unsigned f0, f1;
                unsigned spins = 0;
                bool fail = false;
                for (;;) {
                    q0 = __hip_atomic_load(pb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    q1 = __hip_atomic_load(pb + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    f0 = (unsigned)(q0 >> 32);
                    f1 = (unsigned)(q1 >> 32);
                    if (f0 == 0xffffffffu || f1 == 0xffffffffu) {
                        fail = true;
                        break;
                    }
                    if (f0 == f1 && (f0 >> 1) == ge) break;
                    __builtin_amdgcn_s_sleep(2);
                    if (++spins == n.spins) {  // the combiner never came: report (not the seq), stop
                        __hip_atomic_store(n.res + 6, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        fail = true;
                        break;
                    }
                }
                if (fail) {
                    sh_next[1] = 2.0;
                } else {
                    sh_next[0] = __longlong_as_double((long long)((q1 << 32) | (q0 & 0xffffffffull)));
                    sh_next[1] = (f0 & 1u) ? 1.0 : 0.0;
                    if (blockIdx.x == 1) stamp(evn, 4);
                }
            }
            __syncthreads();
        }
        if (sh_next[1] != 0.0) return;
        x = sh_next[0];
        __syncthreads();  // sh_next and egq are rewritten by the next evaluation
    }
}

template <int K>
int launch_edge_k(hipStream_t st, int mode, const EdgeArgs &a, size_t lds,
                  hipEvent_t after_edge) {
    const dim3 grid((unsigned)a.n_tiles), block(64 * edge_waves(a.C));
    switch (mode) {
        case EDGE_UPDATE: hipLaunchKernelGGL((k_edge<K, EDGE_UPDATE>), grid, block, lds, st, a); break;
        case EDGE_LNL: hipLaunchKernelGGL((k_edge<K, EDGE_LNL>), grid, block, lds, st, a); break;
        case EDGE_DERIV: hipLaunchKernelGGL((k_edge<K, EDGE_DERIV>), grid, block, lds, st, a); break;
        default: return (int)hipErrorInvalidValue;
    }
    if (after_edge) (void)hipEventRecord(after_edge, st);
    if (mode != EDGE_UPDATE && a.two_pass == 1)  // 2: the host adds the partials
        hipLaunchKernelGGL(k_edge_sum, dim3(1), dim3(256), 0, st, a.block_part, a.n_tiles,
                           a.result, a.seq);
    return (int)hipGetLastError();
}

}  // namespace

size_t edge_lds_bytes(int mode, int K, int C) { return EdgeLds(mode, K, C).total * sizeof(double); }

int launch_edge(hipStream_t st, int mode, const EdgeArgs &a, hipEvent_t after_edge) {
    const size_t lds = edge_lds_bytes(mode, a.K, a.C);
    if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
    switch (a.K) {
        case 2: return launch_edge_k<2>(st, mode, a, lds, after_edge);
        case 4: return launch_edge_k<4>(st, mode, a, lds, after_edge);
        case 20: return launch_edge_k<20>(st, mode, a, lds, after_edge);
        default: return (int)hipErrorInvalidValue;
    }
}

template <int TPW>
int newton_per_cu_t(int K) {
    int nb = 0;
    hipError_t e = K == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_edge_newton<2, TPW>, 64 * kNewtonWaves, 0)
                          : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_edge_newton<4, TPW>, 64 * kNewtonWaves, 0);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return nb;
}

int edge_newton_per_cu(int K, int C, int tpw) {
    if (C < 1 || C > kNewtonMaxC || (K != 2 && K != 4)) return 0;
    return tpw == 1 ? newton_per_cu_t<1>(K) : tpw == 2 ? newton_per_cu_t<2>(K) : 0;
}

int edge_newton_tiles_per_wg(int tpw) { return kNewtonWaves * tpw; }
int edge_newton_max_tpw() { return kNewtonTpw; }
size_t edge_newton_sync_words(int grid) { return 8 * (size_t)grid + 64; }

int launch_edge_newton(hipStream_t st, const EdgeArgs &a, const NewtonArgs &n, int grid) {
    if (a.C < 1 || a.C > kNewtonMaxC || n.tpw < 1 || n.tpw > kNewtonTpw ||
        (int64_t)grid * kNewtonWaves * n.tpw < a.n_tiles || (a.K != 2 && a.K != 4))
        return (int)hipErrorInvalidValue;
    EdgeArgs ac = a;
    NewtonArgs nc = n;
    void *args[] = {&ac, &nc};
    const dim3 g((unsigned)grid), b(64 * kNewtonWaves);
    const void *f = a.K == 2 ? (n.tpw == 1 ? (const void *)k_edge_newton<2, 1> : (const void *)k_edge_newton<2, 2>)
                             : (n.tpw == 1 ? (const void *)k_edge_newton<4, 1> : (const void *)k_edge_newton<4, 2>);
    if (n.plain) return (int)hipLaunchKernel(f, g, b, args, 0, st);
    return (int)hipLaunchCooperativeKernel(f, g, b, args, 0, st);
}

int launch_ascbias(hipStream_t st, const AscArgs &a) {
    if (a.C > 64) return (int)hipErrorInvalidValue;
    int64_t nb = (a.first + 255) / 256;
    const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(nb, 1024))), block(256);
    switch (a.K) {
        case 2: hipLaunchKernelGGL(k_ascbias<2>, grid, block, 0, st, a); break;
        case 4: hipLaunchKernelGGL(k_ascbias<4>, grid, block, 0, st, a); break;
        case 20: hipLaunchKernelGGL(k_ascbias<20>, grid, block, 0, st, a); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
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
