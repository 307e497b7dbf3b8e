// pu_kernels.hip -- CDNA4 (gfx950) kernels of the Felsenstein pruning engine.
//
// Reference behaviour (paths relative to the reference repository root):
//   clv          phylo_utils/likelihood/numba_likelihood_engine.py:14-46
//   lnl_node     numba_likelihood_engine.py:82-87
//   Model.p      phylo_utils/substitution_models/abstract.py:49-59, 99-105
//   traversal    phylo_utils/tree_model.py:160-217 (compute_partials, root combine,
//                lnl_node, logsumexp over categories, pattern-weighted sum)
//
// Design (DESIGN.md "Kernels"): every site pattern is independent through the
// whole post-order, so ONE launch walks the entire schedule: a workgroup owns
// 256/C site patterns x C categories (one (site, category) K-vector per lane,
// [site][category][state] layout => each wave reads/writes contiguous 64*8K
// bytes), the P matrices of a chunk of ops are staged once per workgroup in
// LDS, and a parent CLV that its consumer will read soon is kept in registers
// (host planner, pu_capi.cpp) so it is written to HBM once and never re-read.
#include "pu_internal.h"

#include <math.h>

namespace pu {

namespace {

constexpr double kScaleThreshold = 0x1p-128;  // numba_likelihood_engine.py:7
constexpr int kBlock = 256;

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <int K>
__device__ __forceinline__ void load_vec(const double *__restrict__ p, double (&v)[K]) {
    if constexpr (K % 2 == 0) {
        const dbl2 *q = reinterpret_cast<const dbl2 *>(p);
#pragma unroll
        for (int i = 0; i < K / 2; ++i) {
            const dbl2 t = q[i];
            v[2 * i] = t.x;
            v[2 * i + 1] = t.y;
        }
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) v[i] = p[i];
    }
}

template <int K>
__device__ __forceinline__ void store_vec(double *__restrict__ p, const double (&v)[K],
                                          bool streaming) {
    if constexpr (K % 2 == 0) {
        dbl2 *q = reinterpret_cast<dbl2 *>(p);
        if (streaming) {
#pragma unroll
            for (int i = 0; i < K / 2; ++i) {
                dbl2 t = {v[2 * i], v[2 * i + 1]};
                __builtin_nontemporal_store(t, q + i);
            }
        } else {
#pragma unroll
            for (int i = 0; i < K / 2; ++i) {
                dbl2 t = {v[2 * i], v[2 * i + 1]};
                q[i] = t;
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) p[i] = v[i];
    }
}

// P row i of a [K][K] matrix held in LDS (16-byte aligned rows when K is even).
template <int K>
__device__ __forceinline__ double matvec_row(const double *__restrict__ prow,
                                             const double (&a)[K]) {
    double x = 0.0;
    if constexpr (K % 2 == 0) {
        const dbl2 *q = reinterpret_cast<const dbl2 *>(prow);
#pragma unroll
        for (int j = 0; j < K / 2; ++j) {
            const dbl2 t = q[j];
            x = fma(t.x, a[2 * j], x);
            x = fma(t.y, a[2 * j + 1], x);
        }
    } else {
#pragma unroll
        for (int j = 0; j < K; ++j) x = fma(prow[j], a[j], x);
    }
    return x;
}

// One (site, category) update, numba_likelihood_engine.py:36-44.
template <int K>
__device__ __forceinline__ void clv_update(const double *__restrict__ p1,
                                           const double *__restrict__ p2,
                                           const double (&a)[K], const double (&b)[K],
                                           double sa, double sb, double (&out)[K],
                                           double &cml) {
#pragma unroll
    for (int i = 0; i < K; ++i)
        out[i] = matvec_row<K>(p1 + i * K, a) * matvec_row<K>(p2 + i * K, b);
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

// rescale rule of numba_likelihood_engine.py:37-44 on a finished product vector
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

// scipy 1.15 logsumexp over a short vector (tree_model.py:216).
__device__ __forceinline__ double lse_short(const double *a, int n) {
    double amax = -INFINITY;
    for (int c = 0; c < n; ++c) amax = (a[c] > amax) ? a[c] : amax;
    double m = 0.0, s = 0.0;
    const double shift = isfinite(amax) ? amax : 0.0;
    for (int c = 0; c < n; ++c) {
        if (a[c] == amax)
            m += 1.0;
        else
            s += exp(a[c] - shift);
    }
    if (s != 0.0) s /= m;
    return log1p(s) + log(m) + amax;
}

__device__ __forceinline__ double block_sum_256(double v, double *red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    return t;
}

// ---------------------------------------------------------------- P matrices / side LUTs
// For every side (one branch of one op) and category: P = (evecs * exp(evals * (t * r))) .
// ivecs (abstract.py:99-105, 49-59), written to the API buffer, and the side block the
// traversal stages: P itself, or -- for a coded tip child -- LUT[code][i] = sum_j P_ij
// table[code][j], the child's entire contribution, so the traversal does no arithmetic
// (and no table look-up) for tips.  The LUT row is the same fma chain the traversal would
// run, so results are unchanged bit for bit.
template <int K>
__global__ void __launch_bounds__(kBlock) k_pmatrix(PmatArgs a) {
    const int sd = blockIdx.x, c = blockIdx.y;
    __shared__ double ex[K];
    __shared__ double Pl[K * K];
    const double t = a.brlens[sd] * a.rates[c];
    if ((int)threadIdx.x < K) ex[threadIdx.x] = exp(a.evals[threadIdx.x] * t);
    __syncthreads();
    double *out = a.P + ((size_t)sd * a.C + c) * K * K;
    for (int idx = threadIdx.x; idx < K * K; idx += blockDim.x) {
        const int i = idx / K, j = idx - i * K;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) acc = fma(a.evecs[i * K + k] * ex[k], a.ivecs[k * K + j], acc);
        out[idx] = acc;
        Pl[idx] = acc;
    }
    __syncthreads();
    const int r = a.side_rows[sd];  // K: P side; -n_codes: tip LUT side
    const bool lut = r < 0;
    const int rows = lut ? -r : K;
    double *blk = a.side + a.side_off[sd] + (size_t)c * side_block(rows, K);
    if (!lut) {
        for (int idx = threadIdx.x; idx < K * K; idx += blockDim.x) blk[idx] = Pl[idx];
    } else {
        for (int idx = threadIdx.x; idx < rows * K; idx += blockDim.x) {
            const int code = idx / K, i = idx - code * K;
            const double *tv = a.code_table + (size_t)code * K;
            double x = 0.0;
#pragma unroll
            for (int j = 0; j < K; ++j) x = fma(Pl[i * K + j], tv[j], x);
            blk[idx] = x;
        }
    }
}

// ---------------------------------------------------------------- whole traversal
__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

// LDS carve-up of one traversal workgroup (every offset 16-byte aligned):
//   [descriptors][side arena][tip codes][scaler flags][CLV stash]
struct TravLds {
    size_t a_off, c_off, f_off, st_off, total;
    __host__ __device__ TravLds(int K, int C, int max_ops, int max_side, bool coded, int variant,
                                int L) {
        const int spb = kBlock / C;
        a_off = align16((size_t)max_ops * sizeof(OpDesc));
        size_t a_bytes = (size_t)max_side * sizeof(double);
        const size_t red = (kBlock + kBlock / 64) * sizeof(double);  // epilogue reuse
        if (a_bytes < red) a_bytes = red;
        c_off = a_off + align16(a_bytes);
        f_off = c_off + (coded ? align16((size_t)max_ops * 2 * spb) : 0);
        st_off = f_off + ((variant & TV_SKIP_ZERO_SCALE) ? align16((size_t)max_ops * 4) : 0);
        total = st_off + (size_t)L * (K + 1) * kBlock * sizeof(double);
    }
};

// x_i = sum_j P_ij v_j for one (side, category) block held in LDS
template <int K>
__device__ __forceinline__ void side_matvec(const double *__restrict__ P, const double (&v)[K],
                                            double (&x)[K]) {
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = matvec_row<K>(P + i * K, v);
}

// One child's contribution x (= P v, or the tip LUT row) and scaler for a (site, category)
// lane.  SRC_MEM (an HBM read-back) is compiled only into the general kernel: a
// vector-memory load in the op loop makes the compiler wait on vmcnt, which on CDNA also
// waits for every in-flight store.
template <int K, int R, int L, bool CODED, bool NOMEM>
__device__ __forceinline__ void child_contrib(int code, uint8_t tip_code, const double *blk,
                                              const TraverseArgs &a, int64_t site, int64_t e,
                                              int64_t SC, int tid, const double *stash,
                                              const double (&rv)[R][K], const double (&rs)[R],
                                              double (&x)[K], double &s) {
    const int kind = src_kind(code), idx = src_index(code);
    double v[K];
    if (CODED && kind == SRC_TIP) {
        const double *row = blk + (int)tip_code * K;  // LUT row: the whole contribution
        if constexpr (K % 2 == 0) {
            const dbl2 *q = reinterpret_cast<const dbl2 *>(row);
#pragma unroll
            for (int i = 0; i < K / 2; ++i) {
                const dbl2 t = q[i];
                x[2 * i] = t.x;
                x[2 * i + 1] = t.y;
            }
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) x[i] = row[i];
        }
        s = 0.0;
        return;
    }
    if (kind == SRC_REG) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (r == idx) {
#pragma unroll
                for (int i = 0; i < K; ++i) v[i] = rv[r][i];
                s = rs[r];
            }
    } else if (L > 0 && kind == SRC_LDS) {
        const double *p = stash + (size_t)idx * (K + 1) * kBlock + tid;
#pragma unroll
        for (int i = 0; i < K; ++i) v[i] = p[i * kBlock];
        s = p[K * kBlock];
    } else if (!CODED && kind == SRC_TIP) {
        load_vec<K>(a.tips + ((size_t)idx * a.S + site) * K, v);
        s = 0.0;
    } else if constexpr (!NOMEM) {
        load_vec<K>(a.clv + ((size_t)idx * SC + e) * K, v);
        s = a.scale[(size_t)idx * SC + e];
    }
    side_matvec<K>(blk, v, x);
}

template <int K, int R, int L, bool CODED, int V>
__global__ void __launch_bounds__(kBlock) k_traverse(TraverseArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    constexpr int RR = R > 0 ? R : 1;
    constexpr bool all_nt = (V & TV_STORE_NT) != 0;
    constexpr bool skip_zero = (V & TV_SKIP_ZERO_SCALE) != 0;
    constexpr bool nomem = (V & TV_NOMEM) != 0 && CODED;
    const int C = a.C;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int spb = kBlock / C;
    const int ls = tid / C;
    const int cat = tid - ls * C;
    const int64_t SC = a.S * C;
    const int64_t nwt = (int64_t)a.n_tiles * 4;  // wave tiles per flag row
    const int tile = blockIdx.x;
    const int64_t site0 = (int64_t)tile * spb;
    const bool active = (ls < spb) && (site0 + ls < a.S);
    // idle lanes of a partial tile compute on a valid site and store nothing
    const int64_t site = active ? site0 + ls : site0;
    const int64_t e = site * C + cat;
    const int64_t wtile = (int64_t)tile * 4 + wave;
    const int blk_tip = side_block(a.n_codes, K);  // category stride of a tip LUT side
    const int blk_p = side_block(K, K);            // ... of a P side

    const TravLds LY(K, C, a.max_chunk_ops, a.max_chunk_side, CODED, V, L);
    OpDesc *dlds = reinterpret_cast<OpDesc *>(lds_raw);
    double *arena = reinterpret_cast<double *>(lds_raw + LY.a_off);
    uint8_t *clds = lds_raw + LY.c_off;
    uint8_t *flds = lds_raw + LY.f_off;
    double *stash = reinterpret_cast<double *>(lds_raw + LY.st_off);

    double rv[RR][K];
    double rs[RR];
#pragma unroll
    for (int r = 0; r < RR; ++r) {
        rs[r] = 0.0;
#pragma unroll
        for (int i = 0; i < K; ++i) rv[r][i] = 0.0;
    }
    double sw = -INFINITY;

    for (int ch = 0; ch < a.n_chunks; ++ch) {
        const int o0 = a.chunk_op[ch];
        const int nch = a.chunk_op[ch + 1] - o0;
        const int g0 = a.chunk_side[ch];
        const int ng = a.chunk_side[ch + 1] - g0;
        __syncthreads();
        // stage the chunk: descriptors, side matrices, this tile's tip codes and scaler
        // flags -- every global load of the chunk is issued here, so the op loop below runs
        // on LDS and registers only
        for (int i = tid; i < nch; i += kBlock) dlds[i] = a.ops[o0 + i];
        {
            const dbl2 *src = reinterpret_cast<const dbl2 *>(a.side + g0);
            dbl2 *dst2 = reinterpret_cast<dbl2 *>(arena);
            for (int i = tid; i < ng / 2; i += kBlock) dst2[i] = src[i];
        }
        if constexpr (CODED) {
            const int per_op = 2 * spb;
            for (int idx = tid; idx < nch * per_op; idx += kBlock) {
                const int oi = idx / per_op;
                const int r = idx - oi * per_op;
                const int side = r >= spb;
                const int l = r - side * spb;
                const OpDesc d = a.ops[o0 + oi];
                const int code = side ? d.src_b : d.src_a;
                uint8_t v = 0;
                if (src_kind(code) == SRC_TIP && site0 + l < a.S)
                    v = a.codes[(size_t)src_index(code) * a.code_stride + site0 + l];
                clds[idx] = v;
            }
        }
        if constexpr (skip_zero) {
            for (int idx = tid; idx < nch * 4; idx += kBlock) {
                const int oi = idx >> 2, w = idx & 3;
                const int o = o0 + oi;
                const int slot = o < a.n_ops ? a.ops[o].par_slot : -2;  // -2: root row
                uint8_t f = 1;
                if (slot != -1) {
                    const int row = slot >= 0 ? slot : a.n_ops_store_rows;
                    f = a.sflag[(size_t)row * nwt + (int64_t)tile * 4 + w];
                }
                flds[idx] = f;
            }
        }
        __syncthreads();
        // software pipeline: the next op's descriptor and tip codes are read while the
        // current op computes
        OpDesc dn = dlds[0];
        uint8_t ca_n = 0, cb_n = 0;
        if constexpr (CODED) {
            ca_n = clds[ls];
            cb_n = clds[spb + ls];
        }
        for (int oi = 0; oi < nch; ++oi) {
            const int o = o0 + oi;
            const OpDesc d = dn;
            const uint8_t ca = ca_n, cb = cb_n;
            if (oi + 1 < nch) {
                dn = dlds[oi + 1];
                if constexpr (CODED) {
                    ca_n = clds[(2 * oi + 2) * spb + ls];
                    cb_n = clds[(2 * oi + 3) * spb + ls];
                }
            }
            const int code_a = __builtin_amdgcn_readfirstlane(d.src_a);
            const int code_b = __builtin_amdgcn_readfirstlane(d.src_b);
            const int par = __builtin_amdgcn_readfirstlane(d.par_slot);
            const int dst = __builtin_amdgcn_readfirstlane(d.dst);
            const int loff_a = __builtin_amdgcn_readfirstlane(d.loff_a);
            const int loff_b = __builtin_amdgcn_readfirstlane(d.loff_b);
            const bool tip_a = CODED && src_kind(code_a) == SRC_TIP;
            const bool tip_b = CODED && src_kind(code_b) == SRC_TIP;
            const double *blk_a = arena + loff_a + cat * (tip_a ? blk_tip : blk_p);
            const double *blk_b = arena + loff_b + cat * (tip_b ? blk_tip : blk_p);
            double x[K], y[K], sa = 0.0, sb = 0.0, out[K], cml;
            child_contrib<K, RR, L, CODED, nomem>(code_a, ca, blk_a, a, site, e, SC, tid, stash,
                                                 rv, rs, x, sa);
            child_contrib<K, RR, L, CODED, nomem>(code_b, cb, blk_b, a, site, e, SC, tid, stash,
                                                 rv, rs, y, sb);
#pragma unroll
            for (int i = 0; i < K; ++i) out[i] = x[i] * y[i];
            rescale<K>(out, sa, sb, cml);
            const bool is_root = o == a.n_ops;
            double *dst_clv = is_root ? a.root_clv
                                      : (par >= 0 ? a.clv + (size_t)par * SC * K : nullptr);
            double *dst_scale = is_root ? a.root_scale
                                        : (par >= 0 ? a.scale + (size_t)par * SC : nullptr);
            if (dst_clv) {
                // a CLV that stays on chip for its consumer is never re-read here: stream it
                const bool nt = all_nt || dst >= 0 || is_root;
                if (active) store_vec<K>(dst_clv + e * K, out, nt);
                // scalers: an all-zero wave tile whose memory is already zero is skipped
                bool write_scale = true;
                if constexpr (skip_zero) {
                    const bool nz = __any(active && cml != 0.0);
                    const bool dirty = flds[oi * 4 + wave] != 0;
                    write_scale = nz || dirty;
                    if (nz != dirty && lane == 0) {
                        const int row = is_root ? a.n_ops_store_rows : par;
                        a.sflag[(size_t)row * nwt + wtile] = nz ? 1 : 0;
                    }
                }
                if (write_scale && active) {
                    if (nt)
                        __builtin_nontemporal_store(cml, dst_scale + e);
                    else
                        dst_scale[e] = cml;
                }
            }
            if (!is_root) {
                if (dst >= 0) {
                    const int dk = src_kind(dst), di = src_index(dst);
                    if (L > 0 && dk == SRC_LDS) {
                        double *p = stash + (size_t)di * (K + 1) * kBlock + tid;
#pragma unroll
                        for (int i = 0; i < K; ++i) p[i * kBlock] = out[i];
                        p[K * kBlock] = cml;
                    } else if constexpr (R > 0) {
#pragma unroll
                        for (int r = 0; r < R; ++r)
                            if (r == di) {
#pragma unroll
                                for (int i = 0; i < K; ++i) rv[r][i] = out[i];
                                rs[r] = cml;
                            }
                    }
                }
            } else {
                // root combine stored above (tree_model.py:196-197); lnl_node (numba :82-87)
                double f = 0.0;
#pragma unroll
                for (int i = 0; i < K; ++i) f = fma(out[i], a.pi[i], f);
                sw = ((f > 0.0) ? log(f) + cml : -INFINITY) + a.logw[cat];
            }
        }
    }

    // per-pattern logsumexp over categories, pattern-weighted block sum
    __syncthreads();
    arena[tid] = sw;
    __syncthreads();
    double contrib = 0.0;
    if (active && cat == 0) {
        const double l = lse_short(arena + tid, C);
        a.site_lnl[site] = l;
        contrib = a.pattern_w[site] * l;
    }
    const double t = block_sum_256(contrib, arena + kBlock);
    if (tid == 0) a.block_sum[tile] = t;
}

// deterministic fixed-order sum of per-block partials
__global__ void __launch_bounds__(kBlock)
    k_reduce(const double *__restrict__ in, int n, double *__restrict__ out) {
    __shared__ double red[kBlock / 64];
    double v = 0.0;
    for (int i = threadIdx.x; i < n; i += kBlock) v += in[i];
    const double t = block_sum_256(v, red);
    if (threadIdx.x == 0) *out = t;
}

// ---------------------------------------------------------------- stateless seam
template <int K>
__global__ void __launch_bounds__(kBlock)
    k_clv(int C, int64_t S, const double *__restrict__ p1, const double *__restrict__ p2,
          const double *__restrict__ clv1, const double *__restrict__ clv2,
          const double *__restrict__ sa, const double *__restrict__ sb,
          double *__restrict__ cml, double *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    constexpr int KP = p_stride(K);
    for (int idx = threadIdx.x; idx < 2 * C * K * K; idx += kBlock) {
        const int m = idx / (K * K);
        const double v = (m < C) ? p1[idx] : p2[idx - C * K * K];
        lds[m * KP + (idx - m * K * K)] = v;
    }
    __syncthreads();
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= S * C) return;
    const int cat = (int)(e % C);
    double va[K], vb[K], o[K], c;
    load_vec<K>(clv1 + e * K, va);
    load_vec<K>(clv2 + e * K, vb);
    clv_update<K>(lds + cat * KP, lds + (C + cat) * KP, va, vb, sa[e], sb[e], o, c);
    store_vec<K>(out + e * K, o, false);
    cml[e] = c;
}

// runtime-K fallback for the stateless seam (any alphabet, K <= 64)
__global__ void __launch_bounds__(kBlock)
    k_clv_any(int K, int C, int64_t S, const double *__restrict__ p1,
              const double *__restrict__ p2, const double *__restrict__ clv1,
              const double *__restrict__ clv2, const double *__restrict__ sa,
              const double *__restrict__ sb, double *__restrict__ cml,
              double *__restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= S * C) return;
    const int cat = (int)(e % C);
    const double *P1 = p1 + (size_t)cat * K * K, *P2 = p2 + (size_t)cat * K * K;
    const double *A = clv1 + e * K, *B = clv2 + e * K;
    double *O = out + e * K;
    double m = 0.0;
    for (int i = 0; i < K; ++i) {
        double x = 0.0, y = 0.0;
        for (int j = 0; j < K; ++j) {
            x = fma(P1[i * K + j], A[j], x);
            y = fma(P2[i * K + j], B[j], y);
        }
        const double v = x * y;
        O[i] = v;
        m = (i == 0 || v > m || v != v) ? v : m;
    }
    const double base = sa[e] + sb[e];
    if (m < kScaleThreshold && m > 0.0) {
        cml[e] = base + log(m);
        for (int i = 0; i < K; ++i) O[i] = O[i] / m;
    } else {
        cml[e] = base;
    }
}

__global__ void __launch_bounds__(kBlock)
    k_lnl_node(int K, int C, int64_t S, const double *__restrict__ pi,
               const double *__restrict__ partials, const double *__restrict__ scale,
               double *__restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= S * C) return;
    const double *v = partials + e * K;
    double f = 0.0;
    for (int i = 0; i < K; ++i) f = fma(v[i], pi[i], f);
    out[e] = (f > 0.0) ? log(f) + scale[e] : -INFINITY;
}

// TreeModel.partials[tip] view: the tip vector copied into every category
// (tree_model.py:142-148), for pu_get_partials on a leaf node.
__global__ void __launch_bounds__(kBlock)
    k_expand_tip(int K, int C, int64_t S, int64_t cstride, int coded, int tip,
                 const double *__restrict__ tips, const uint8_t *__restrict__ codes,
                 const double *__restrict__ table, double *__restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= S * C) return;
    const int64_t s = e / C;
    const double *src = coded ? table + (size_t)codes[(size_t)tip * cstride + s] * K
                              : tips + ((size_t)tip * S + s) * K;
    for (int i = 0; i < K; ++i) out[e * K + i] = src[i];
}

template <int K, int R, int L, bool CODED>
int launch_traverse_k(hipStream_t st, const TraverseArgs &a, int grid) {
    const size_t lds =
        TravLds(K, a.C, a.max_chunk_ops, a.max_chunk_side, CODED, a.variant, L).total;
    switch (a.variant) {
        case 0: hipLaunchKernelGGL((k_traverse<K, R, L, CODED, 0>), dim3(grid), dim3(kBlock), lds, st, a); break;
        case TV_SKIP_ZERO_SCALE: hipLaunchKernelGGL((k_traverse<K, R, L, CODED, TV_SKIP_ZERO_SCALE>), dim3(grid), dim3(kBlock), lds, st, a); break;
        case TV_NOMEM: hipLaunchKernelGGL((k_traverse<K, R, L, CODED, TV_NOMEM>), dim3(grid), dim3(kBlock), lds, st, a); break;
        case TV_NOMEM | TV_SKIP_ZERO_SCALE: hipLaunchKernelGGL((k_traverse<K, R, L, CODED, TV_NOMEM | TV_SKIP_ZERO_SCALE>), dim3(grid), dim3(kBlock), lds, st, a); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

}  // namespace

// On-chip CLV slots per (site, category) lane: R in registers, L in the LDS stash.
// (K, R, L) combinations built (the planner falls back to HBM read-back beyond them).
#define PU_SLOT_CONFIGS(X)                                                   \
    X(2, 4, 0) X(2, 4, 2) X(2, 8, 0)                                         \
    X(4, 0, 0) X(4, 2, 0) X(4, 4, 0) X(4, 2, 2) X(4, 2, 4) X(4, 0, 4) X(4, 1, 3) \
    X(20, 0, 0) X(20, 1, 0) X(20, 2, 0)

void traverse_default_slots(int K, int *R, int *L) {
    switch (K) {
        case 2: *R = 4; *L = 2; return;
        case 4: *R = 2; *L = 2; return;
        case 20: *R = 1; *L = 0; return;
        default: *R = 0; *L = 0;
    }
}

bool traverse_supported(int K) { return K == 2 || K == 4 || K == 20; }

bool traverse_slots_supported(int K, int R, int L) {
#define PU_X(KK, RR, LL) if (K == KK && R == RR && L == LL) return true;
    PU_SLOT_CONFIGS(PU_X)
#undef PU_X
    return false;
}

size_t traverse_stash_bytes(int K, int L) { return (size_t)L * (K + 1) * kBlock * sizeof(double); }

int traverse_sites_per_block(int C) { return kBlock / C; }

size_t traverse_lds_bytes(int K, int C, int max_chunk_ops, int max_chunk_side, bool coded,
                          int variant, int L) {
    return TravLds(K, C, max_chunk_ops, max_chunk_side, coded, variant, L).total;
}

int launch_traverse(hipStream_t st, int K, int R, int L, bool coded, const TraverseArgs &a,
                    int grid) {
#define PU_X(KK, RR, LL)                                                            \
    if (K == KK && R == RR && L == LL)                                              \
        return coded ? launch_traverse_k<KK, RR, LL, true>(st, a, grid)           \
                     : launch_traverse_k<KK, RR, LL, false>(st, a, grid);
    PU_SLOT_CONFIGS(PU_X)
#undef PU_X
    return (int)hipErrorInvalidValue;
}

int launch_pmatrix(hipStream_t st, const PmatArgs &a) {
    const dim3 grid(a.n_sides, a.C);
    switch (a.K) {
        case 2: hipLaunchKernelGGL(k_pmatrix<2>, grid, dim3(kBlock), 0, st, a); break;
        case 4: hipLaunchKernelGGL(k_pmatrix<4>, grid, dim3(kBlock), 0, st, a); break;
        case 20: hipLaunchKernelGGL(k_pmatrix<20>, grid, dim3(kBlock), 0, st, a); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

int launch_reduce(hipStream_t st, const double *block_sum, int n, double *out) {
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kBlock), 0, st, block_sum, n, out);
    return (int)hipGetLastError();
}

int launch_clv(hipStream_t st, int K, int C, int64_t S, const double *p1, const double *p2,
               const double *clv1, const double *clv2, const double *sa, const double *sb,
               double *cml, double *out) {
    const int64_t n = S * C;
    if (n == 0) return 0;
    const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
    const size_t lds = (size_t)2 * C * p_stride(K) * sizeof(double);
    if (lds > 64 * 1024) K = -K;  // many categories: runtime-K kernel, P read from L2
    switch (K) {
        case 2: hipLaunchKernelGGL(k_clv<2>, grid, dim3(kBlock), lds, st, C, S, p1, p2, clv1, clv2, sa, sb, cml, out); break;
        case 4: hipLaunchKernelGGL(k_clv<4>, grid, dim3(kBlock), lds, st, C, S, p1, p2, clv1, clv2, sa, sb, cml, out); break;
        case 20: hipLaunchKernelGGL(k_clv<20>, grid, dim3(kBlock), lds, st, C, S, p1, p2, clv1, clv2, sa, sb, cml, out); break;
        default: hipLaunchKernelGGL(k_clv_any, grid, dim3(kBlock), 0, st, K < 0 ? -K : K, C, S, p1, p2, clv1, clv2, sa, sb, cml, out);
    }
    return (int)hipGetLastError();
}

int launch_lnl_node(hipStream_t st, int K, int C, int64_t S, const double *pi,
                    const double *partials, const double *scale, double *out) {
    const int64_t n = S * C;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_lnl_node, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       st, K, C, S, pi, partials, scale, out);
    return (int)hipGetLastError();
}

int launch_expand_tip(hipStream_t st, int K, int C, int64_t S, int64_t cstride, bool coded,
                      int tip, const double *tips, const uint8_t *codes,
                      const double *code_table, double *out) {
    const int64_t n = S * C;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_expand_tip, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       st, K, C, S, cstride, coded ? 1 : 0, tip, tips, codes, code_table, out);
    return (int)hipGetLastError();
}

}  // namespace pu
