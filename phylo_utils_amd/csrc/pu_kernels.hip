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

// scipy 1.15 logsumexp over a short strided vector (tree_model.py:216)
__device__ __forceinline__ double lse_strided(const double *a, int n, int64_t stride) {
    double amax = -INFINITY;
    for (int c = 0; c < n; ++c) amax = (a[c * stride] > amax) ? a[c * stride] : amax;
    double m = 0.0, s = 0.0;
    const double shift = isfinite(amax) ? amax : 0.0;
    for (int c = 0; c < n; ++c) {
        const double x = a[c * stride];
        if (x == amax)
            m += 1.0;
        else
            s += exp(x - shift);
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

// ---------------------------------------------------------------- P matrices
// P = (evecs * exp(evals * (t * r))) . ivecs for every side (one branch of one op) and
// category (abstract.py:99-105, 49-59).
template <int K>
__global__ void __launch_bounds__(kBlock) k_pmatrix(PmatArgs a) {
    const int sd = blockIdx.x, c = blockIdx.y;
    __shared__ double ex[K];
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
    }
}

// ---------------------------------------------------------------- whole traversal
// Read-only, wave-uniform data (descriptors, P, pi, log weights) is read through the
// constant address space: the loads become s_load into SGPRs, and every P entry enters
// the matrix-vector product as the SGPR operand of a v_fma_f64 -- no LDS traffic and no
// per-lane address arithmetic for P.
template <class T>
using cptr = const __attribute__((address_space(4))) T *;
template <class T>
__device__ __forceinline__ cptr<T> as_const(const T *p) {
    return (cptr<T>)(uintptr_t)p;
}

__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15) & ~size_t(15); }
constexpr int kWaves = kBlock / 64;

// tiles whose waves share a workgroup (wave tile wt = 4 * block + wave = tile * C + cat)
__host__ __device__ inline int block_tiles(int C) {
    return kWaves % C == 0 ? kWaves / C : (kWaves + C - 1) / C + 1;
}

// LDS of one traversal workgroup (4 waves; every offset 16-byte aligned):
//   [code table][tip codes: the workgroup's tiles x one chunk's uses x 64][CLV stash:
//   n_lds slots x (K + 1) x 256 lanes]; after the op loop the lnl exchange of the epilogue
//   reuses the codes / stash bytes.  Smaller is better: the LDS of a workgroup decides how
//   many workgroups share a CU.
struct TravLds {
    size_t codes_off, stash_off, lnl_off, total;
    __host__ __device__ TravLds(int K, int n_codes, int max_uses, bool coded, int n_lds, int C) {
        codes_off = coded ? align16((size_t)n_codes * K * sizeof(double)) : 0;
        stash_off =
            codes_off + (coded ? align16((size_t)block_tiles(C) * max_uses * kTile) : 0);
        lnl_off = codes_off;
        const size_t end = stash_off + (size_t)n_lds * (K + 1) * kBlock * sizeof(double);
        const size_t lnl_end = lnl_off + (kBlock + kWaves) * sizeof(double);
        total = end > lnl_end ? end : lnl_end;
    }
};

// x = P v for one (side, category): P in SGPRs, v and x in VGPRs (same fma chain as the
// stateless k_clv, so results agree bit for bit)
template <int K>
__device__ __forceinline__ void matvec_s(cptr<double> P, const double (&v)[K], double (&x)[K]) {
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) acc = fma(P[i * K + j], v[j], acc);
        x[i] = acc;
    }
}

// element (slot row, category, tile) of the tiled CLV / scaler arrays
__device__ __forceinline__ size_t tile_row(int row, int C, int cat, int n_tiles, int tile) {
    return ((size_t)row * C + cat) * n_tiles + tile;
}

template <int K>
__device__ __forceinline__ void load_tiled(const double *base, int lane, double (&v)[K]) {
    const dbl2 *q = reinterpret_cast<const dbl2 *>(base) + lane;
#pragma unroll
    for (int i = 0; i < K / 2; ++i) {
        const dbl2 t = q[i * kTile];
        v[2 * i] = t.x;
        v[2 * i + 1] = t.y;
    }
}

template <int K>
__device__ __forceinline__ void store_tiled(double *base, int lane, const double (&v)[K],
                                            bool nt) {
    dbl2 *q = reinterpret_cast<dbl2 *>(base) + lane;
#pragma unroll
    for (int i = 0; i < K / 2; ++i) {
        const dbl2 t = {v[2 * i], v[2 * i + 1]};
        if (nt)
            __builtin_nontemporal_store(t, q + i * kTile);
        else
            q[i * kTile] = t;
    }
}

// One child's vector from the code table (coded tips) or the dense tip array.
template <int K, bool CODED>
__device__ __forceinline__ void tip_vec(const TraverseArgs &a, const double *table,
                                        const uint8_t *ucode, int tip, int64_t site_c,
                                        double (&v)[K]) {
    if constexpr (CODED) {
        const dbl2 *row = reinterpret_cast<const dbl2 *>(table + (int)*ucode * K);
#pragma unroll
        for (int i = 0; i < K / 2; ++i) {
            const dbl2 t = row[i];
            v[2 * i] = t.x;
            v[2 * i + 1] = t.y;
        }
    } else {
        load_vec<K>(a.tips + ((size_t)tip * a.S + site_c) * K, v);
    }
}

// CLV (K doubles + scaler) of one lane in an LDS stash slot: [slot][K + 1][4 waves][64]
template <int K>
__device__ __forceinline__ void stash_get(const double *p, double (&v)[K], double &s) {
#pragma unroll
    for (int i = 0; i < K; ++i) v[i] = p[i * kBlock];
    s = p[K * kBlock];
}

template <int K>
__device__ __forceinline__ void stash_put(double *p, const double (&v)[K], double s) {
#pragma unroll
    for (int i = 0; i < K; ++i) p[i * kBlock] = v[i];
    p[K * kBlock] = s;
}

// The two children of op t as x = P_a v_a, y = P_b v_b with their scalers.
template <int K, bool CODED, bool GENERIC>
__device__ __forceinline__ void op_children(const TraverseArgs &a, int pat, int ia, int ib,
                                            cptr<double> Pa, cptr<double> Pb,
                                            const double (&cur)[K], double cur_s,
                                            const double *table, const uint8_t *ca,
                                            const uint8_t *cb, const double *stash_l,
                                            const double *clv_w, const double *scale_w,
                                            size_t slot_stride, size_t sstride, int lane,
                                            int64_t site_c, double (&x)[K], double (&y)[K],
                                            double &sa, double &sb) {
    double v[K];
    // child a
    if (pat == PAT_LC) {
        stash_get<K>(stash_l + (size_t)ia * (K + 1) * kBlock, v, sa);
        matvec_s<K>(Pa, v, x);
    } else if (pat == PAT_CT) {
        matvec_s<K>(Pa, cur, x);
        sa = cur_s;
    } else if (pat == PAT_TT) {
        tip_vec<K, CODED>(a, table, ca, ia, site_c, v);
        matvec_s<K>(Pa, v, x);
        sa = 0.0;
    } else if constexpr (GENERIC) {  // PAT_MC, PAT_MT, PAT_MM: read back from HBM
        load_tiled<K>(clv_w + (size_t)ia * slot_stride, lane, v);
        sa = scale_w[(size_t)ia * sstride + lane];
        matvec_s<K>(Pa, v, x);
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = 0.0;  // unreachable: the host picked the variant
        sa = 0.0;
    }
    // child b
    if (pat == PAT_LC || (GENERIC && pat == PAT_MC)) {
        matvec_s<K>(Pb, cur, y);
        sb = cur_s;
    } else if (GENERIC && pat == PAT_MM) {
        load_tiled<K>(clv_w + (size_t)ib * slot_stride, lane, v);
        sb = scale_w[(size_t)ib * sstride + lane];
        matvec_s<K>(Pb, v, y);
    } else {
        tip_vec<K, CODED>(a, table, cb, ib, site_c, v);
        matvec_s<K>(Pb, v, y);
        sb = 0.0;
    }
}

// Whole traversal in one launch.  Wave w of block b owns category `cat` of the 64-site
// tile `tile` (wave tile wt = 4b + w = tile * C + cat); each lane is one site.
//
// The host evaluates the tree in DFS post-order, so the parent an op produces is usually
// the very next op's second child: it stays in the "current" registers.  A parent that
// waits for a later consumer is kept in one of L LDS stash slots (host-chosen, Belady), so
// the op loop issues no vector-memory loads: a load's wait would also wait for every
// in-flight store (vmcnt counts both, and for mixed loads and stores the compiler can only
// wait for zero).  Only a waiting parent that does not fit the stash is read back from
// HBM (PAT_MC).  Descriptors and P matrices arrive in SGPRs through scalar loads; P enters
// every v_fma_f64 as its SGPR operand.  Tip codes of a 64-op chunk are staged in LDS once
// per workgroup (the C category-waves of a tile share them); the code table is in LDS.
// W > 0: ask the compiler for W resident waves per SIMD (it then trims SGPRs -- with 106
// SGPRs only 6 waves fit, see scripts/occupancy_probe.hip -- at the cost of a few spills
// to VGPR lanes)
template <int K, bool CODED, int V, int W>
__global__ void __launch_bounds__(kBlock, W) k_prune(TraverseArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    constexpr bool skip_zero = (V & TV_SKIP_ZERO_SCALE) != 0;
    constexpr bool generic = (V & TV_GENERIC) != 0;  // HBM read-backs (PAT_M*) compiled in
    const int C = a.C;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wt = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + wave);
    const int tile = wt / C;
    const int cat = wt - tile * C;
    const int n_tiles = a.n_tiles;
    const int tile0 = (blockIdx.x * kWaves) / C;       // first tile of this workgroup
    const int n_wtiles = block_tiles(C);              // tiles a workgroup can touch
    const bool live = tile < n_tiles;
    const int64_t site = (int64_t)tile * kTile + lane;  // < n_tiles * 64 (padded arrays)
    const int64_t site_c = site < a.S ? site : a.S - 1;
    const int nwt = n_tiles * C;

    const TravLds LY(K, a.n_codes, a.max_chunk_uses, CODED, a.n_lds, C);
    double *table = reinterpret_cast<double *>(lds_raw);
    uint8_t *bcodes = lds_raw + LY.codes_off;  // [tile - tile0][chunk use][64]
    const uint8_t *wcodes = bcodes + (size_t)(tile - tile0) * a.max_chunk_uses * kTile;
    double *stash_l = reinterpret_cast<double *>(lds_raw + LY.stash_off) + threadIdx.x;
    double *lnl_x = reinterpret_cast<double *>(lds_raw + LY.lnl_off);

    if constexpr (CODED)
        for (int i = threadIdx.x; i < a.n_codes * K; i += kBlock) table[i] = a.table[i];

    const cptr<int> ops = as_const(reinterpret_cast<const int *>(a.ops));
    const size_t pside = (size_t)C * K * K;  // doubles per side (all categories)
    const cptr<double> Pw = as_const(a.P) + (size_t)cat * K * K;
    const size_t slot_stride = (size_t)C * n_tiles * K * kTile;  // doubles per CLV slot
    const size_t sstride = (size_t)C * n_tiles * kTile;          // doubles per scaler slot
    const size_t row0 = (size_t)cat * n_tiles + tile;
    double *clv_w = a.clv + row0 * K * kTile;
    double *scale_w = a.scale + row0 * kTile;

    double cur[K], cur_s = 0.0;  // the previous op's parent
#pragma unroll
    for (int i = 0; i < K; ++i) cur[i] = 0.0;
    double sw = -INFINITY;

    int u = 0, u_base = 0, o0 = 0;  // tip uses so far; first use / op of the chunk
    uint64_t dirty_mask = ~0ull;
    for (int ch = 0; ch < a.n_chunks; ++ch) {
        o0 = as_const(a.chunk_op0)[ch];
        const int o1 = as_const(a.chunk_op0)[ch + 1];  // the last chunk holds the root
        __syncthreads();  // previous chunk's codes are consumed (first chunk: table staged)
        if constexpr (CODED) {
            // the workgroup's tiles' codes of every tip use in the chunk, 4 bytes per load
            const int u0 = as_const(a.chunk_tip0)[ch], nu = as_const(a.chunk_tip0)[ch + 1] - u0;
            uint32_t *w32 = reinterpret_cast<uint32_t *>(bcodes);
            const int per_tile = nu * (kTile / 4);
            for (int k = threadIdx.x; k < n_wtiles * per_tile; k += kBlock) {
                const int tt = k / per_tile, r = k - tt * per_tile;
                const int uu = r >> 4, q = r & 15;
                const int tl = min(tile0 + tt, n_tiles - 1);
                const int tip = a.tip_seq[u0 + uu];
                w32[(size_t)tt * a.max_chunk_uses * (kTile / 4) + r] =
                    *reinterpret_cast<const uint32_t *>(a.codes + (size_t)tip * a.code_stride +
                                                        (size_t)tl * kTile + 4 * q);
            }
            u = u_base = u0;
        }
        if constexpr (skip_zero) {
            uint32_t f = 1;
            const int o = o0 + lane;
            if (live && o < o1) {
                const int slot = o < a.n_ops ? a.ops[o].par_slot : a.n_store;
                if (slot >= 0) f = a.sflag[(size_t)(slot & ~kReadBack) * nwt + wt];
            }
            dirty_mask = __ballot(f != 0);
        }
        __syncthreads();
        if (!live) continue;

        const int oe = min(o1, a.n_ops);
        for (int t = o0; t < oe; ++t) {
            const int par = ops[8 * t], pat = ops[8 * t + 1], ia = ops[8 * t + 2],
                      ib = ops[8 * t + 3], dst = ops[8 * t + 4];
            // (store_mode bit 4: timing experiment -- every op reads side 0's P)
            const cptr<double> Pa = Pw + (size_t)((a.store_mode & 16) ? 0 : 2 * t) * pside;
            const cptr<double> Pb = Pa + pside;
            const uint8_t *ca = wcodes + (u - u_base) * kTile + lane;
            const uint8_t *cb = ca + (pat == PAT_TT ? kTile : 0);
            u += pat == PAT_TT ? 2 : ((pat == PAT_CT || pat == PAT_MT) ? 1 : 0);
            double x[K], y[K], sa, sb;
            op_children<K, CODED, generic>(a, pat, ia, ib, Pa, Pb, cur, cur_s, table, ca, cb,
                                           stash_l, clv_w, scale_w, slot_stride, sstride,
                                           lane, site_c, x, y, sa, sb);
#pragma unroll
            for (int i = 0; i < K; ++i) cur[i] = x[i] * y[i];
            rescale<K>(cur, sa, sb, cur_s);
            if (dst >= 0) stash_put<K>(stash_l + (size_t)dst * (K + 1) * kBlock, cur, cur_s);
            if (par >= 0) {
                const int slot = par & ~kReadBack;
                // a CLV that is not read back in this run is streamed past the caches
                const int sm = a.store_mode & 3;
                const bool nt = sm == 0 ? (par & kReadBack) == 0 : sm == 2;
                store_tiled<K>(clv_w + (size_t)slot * slot_stride, lane, cur, nt);
                double *dscale = scale_w + (size_t)slot * sstride;
                bool write_scale = true;
                if constexpr (skip_zero) {
                    // an all-zero scaler wave tile whose memory is already zero is skipped
                    const bool nz = __any(cur_s != 0.0);
                    const bool dirty = (dirty_mask >> (t - o0)) & 1;
                    write_scale = nz || dirty;
                    if (nz != dirty && lane == 0) a.sflag[(size_t)slot * nwt + wt] = nz;
                }
                if (write_scale) {
                    if (nt)
                        __builtin_nontemporal_store(cur_s, dscale + lane);
                    else
                        dscale[lane] = cur_s;
                }
            }
        }
    }
    if (live) {
        // root combine (tree_model.py:189-197): the last descriptor, in the last chunk
        const int t = a.n_ops;
        const int pat = ops[8 * t + 1], ia = ops[8 * t + 2], ib = ops[8 * t + 3];
        const cptr<double> Pa = Pw + (size_t)(2 * t) * pside;
        const cptr<double> Pb = Pa + pside;
        const uint8_t *ca = wcodes + (u - u_base) * kTile + lane;
        const uint8_t *cb = ca + (pat == PAT_TT ? kTile : 0);
        double x[K], y[K], sa, sb;
        op_children<K, CODED, generic>(a, pat, ia, ib, Pa, Pb, cur, cur_s, table, ca, cb,
                                       stash_l, clv_w, scale_w, slot_stride, sstride, lane,
                                       site_c, x, y, sa, sb);
        double out[K], cml;
#pragma unroll
        for (int i = 0; i < K; ++i) out[i] = x[i] * y[i];
        rescale<K>(out, sa, sb, cml);
        store_tiled<K>(a.root_clv + row0 * K * kTile, lane, out, true);
        bool write_scale = true;
        if constexpr (skip_zero) {
            const bool nz = __any(cml != 0.0);
            const bool dirty = (dirty_mask >> (t - o0)) & 1;
            write_scale = nz || dirty;
            if (nz != dirty && lane == 0) a.sflag[(size_t)a.n_store * nwt + wt] = nz;
        }
        if (write_scale) __builtin_nontemporal_store(cml, a.root_scale + row0 * kTile + lane);
        // lnl_node (numba_likelihood_engine.py:82-87) plus the category's log weight
        const cptr<double> pi = as_const(a.pi);
        double f = 0.0;
#pragma unroll
        for (int i = 0; i < K; ++i) f = fma(out[i], pi[i], f);
        sw = ((f > 0.0) ? log(f) + cml : -INFINITY) + as_const(a.logw)[cat];
    }

    if (a.cat_lnl) {  // 4 % C != 0: a tile's categories span workgroups (k_site_lse)
        if (live) a.cat_lnl[(size_t)cat * n_tiles * kTile + site] = sw;
        return;
    }
    // per-pattern logsumexp over categories (tree_model.py:216), pattern-weighted block sum;
    // the C waves of a tile are in this workgroup (lnl_x aliases the codes and the stash)
    __syncthreads();
    lnl_x[threadIdx.x] = sw;
    __syncthreads();
    double contrib = 0.0;
    if (live && cat == 0 && site < a.S) {
        const double l = lse_strided(lnl_x + wave * 64 + lane, C, 64);
        a.site_lnl[site] = l;
        contrib = a.pattern_w[site] * l;
    }
    const double t = block_sum_256(contrib, lnl_x + kBlock);
    if (threadIdx.x == 0) a.block_sum[blockIdx.x] = t;
}

// ---------------------------------------------------------------- protein traversal
// K = 20 has too little parallelism for one (site, category) per lane (cfg3: 10k sites x 4
// categories = 625 waves for 1024 SIMDs) and 800 dependent fp64 FMAs per lane and op.
// k_prune_rows splits the rows of every update across the waves of a workgroup: a
// workgroup owns one category of one 64-site tile, wave w computes parent rows
// [RW*w, RW*w + RW) with its P rows in SGPRs (wave-uniform, as in k_prune), and the full
// child vectors every wave needs are exchanged through LDS ("current" parent, stash slots).
// The rescale maximum over all K rows is combined across waves in LDS.  Two barriers per op.
// Same descriptors, planner and tiled HBM layout as k_prune (wave w stores state pairs
// [RW*w/2, RW*w/2 + RW/2)); categories are combined by k_site_lse.
template <int K, int RW>
struct RowsLds {
    // [code table][tip codes: uses x 64][current: (K+1) x 64][stash: L x (K+1) x 64][max: W x 64]
    size_t codes_off, cur_off, stash_off, red_off, total;
    __host__ __device__ RowsLds(int n_codes, int max_uses, bool coded, int n_lds) {
        codes_off = coded ? align16((size_t)n_codes * K * sizeof(double)) : 0;
        cur_off = codes_off + (coded ? align16((size_t)max_uses * kTile) : 0);
        stash_off = cur_off + (size_t)(K + 1) * kTile * sizeof(double);
        red_off = stash_off + (size_t)n_lds * (K + 1) * kTile * sizeof(double);
        total = red_off + (size_t)(K / RW) * kTile * sizeof(double) + 16;
    }
};

// a full child CLV of this lane from an LDS buffer laid out [K/2][64][2] + scaler [64]
template <int K>
__device__ __forceinline__ void lds_vec(const double *buf, int lane, double (&v)[K],
                                        double &s) {
    const dbl2 *q = reinterpret_cast<const dbl2 *>(buf) + lane;
#pragma unroll
    for (int i = 0; i < K / 2; ++i) {
        const dbl2 t = q[i * kTile];
        v[2 * i] = t.x;
        v[2 * i + 1] = t.y;
    }
    s = buf[K * kTile + lane];
}

// rows [r0, r0 + RW) of a parent into an LDS buffer (the scaler by wave 0)
template <int K, int RW>
__device__ __forceinline__ void lds_put_rows(double *buf, int lane, int r0,
                                             const double (&o)[RW], double s, bool put_s) {
    dbl2 *q = reinterpret_cast<dbl2 *>(buf) + lane;
#pragma unroll
    for (int h = 0; h < RW / 2; ++h) q[(r0 / 2 + h) * kTile] = dbl2{o[2 * h], o[2 * h + 1]};
    if (put_s) buf[K * kTile + lane] = s;
}

// x[r] = sum_j P[r0 + r][j] v[j] for this wave's rows; P rows in SGPRs
template <int K, int RW>
__device__ __forceinline__ void matvec_rows(cptr<double> P, const double (&v)[K],
                                            double (&x)[RW]) {
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) acc = fma(P[r * K + j], v[j], acc);
        x[r] = acc;
    }
}

template <int K, bool CODED, bool GENERIC>
__device__ __forceinline__ void rows_child(const TraverseArgs &a, int kind, int idx,
                                           const double *table, const uint8_t *ucode,
                                           const double *cur_l, const double *stash_l,
                                           const double *clv_w, const double *scale_w,
                                           size_t slot_stride, size_t sstride, int lane,
                                           int64_t site_c, double (&v)[K], double &s) {
    if (kind == 0) {  // the current parent
        lds_vec<K>(cur_l, lane, v, s);
    } else if (kind == 1) {  // a tip
        tip_vec<K, CODED>(a, table, ucode, idx, site_c, v);
        s = 0.0;
    } else if (kind == 2) {  // an LDS stash slot
        lds_vec<K>(stash_l + (size_t)idx * (K + 1) * kTile, lane, v, s);
    } else if constexpr (GENERIC) {  // read back from HBM
        load_tiled<K>(clv_w + (size_t)idx * slot_stride, lane, v);
        s = scale_w[(size_t)idx * sstride + lane];
    }
}

template <int K, int RW, bool CODED, int V>
__global__ void __launch_bounds__(64 * (K / RW)) k_prune_rows(TraverseArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    constexpr int W = K / RW;
    constexpr bool skip_zero = (V & TV_SKIP_ZERO_SCALE) != 0;
    constexpr bool generic = (V & TV_GENERIC) != 0;
    const int C = a.C;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r0 = w * RW;
    const int wt = blockIdx.x;  // = tile * C + cat
    const int tile = wt / C;
    const int cat = wt - tile * C;
    const int n_tiles = a.n_tiles;
    const int64_t site = (int64_t)tile * kTile + lane;
    const int64_t site_c = site < a.S ? site : a.S - 1;
    const int nwt = n_tiles * C;

    const RowsLds<K, RW> LY(a.n_codes, a.max_chunk_uses, CODED, a.n_lds);
    double *table = reinterpret_cast<double *>(lds_raw);
    uint8_t *codes_l = lds_raw + LY.codes_off;
    double *cur_l = reinterpret_cast<double *>(lds_raw + LY.cur_off);
    double *stash_l = reinterpret_cast<double *>(lds_raw + LY.stash_off);
    double *red = reinterpret_cast<double *>(lds_raw + LY.red_off);

    if constexpr (CODED)
        for (int i = threadIdx.x; i < a.n_codes * K; i += 64 * W) table[i] = a.table[i];

    const cptr<int> ops = as_const(reinterpret_cast<const int *>(a.ops));
    const size_t pside = (size_t)C * K * K;
    const cptr<double> Pw = as_const(a.P) + (size_t)cat * K * K + (size_t)r0 * K;
    const size_t slot_stride = (size_t)C * n_tiles * K * kTile;
    const size_t sstride = (size_t)C * n_tiles * kTile;
    const size_t row0 = (size_t)cat * n_tiles + tile;
    double *clv_w = a.clv + row0 * K * kTile;
    double *scale_w = a.scale + row0 * kTile;

    int u = 0, u_base = 0, o0 = 0;
    uint64_t dirty_mask = ~0ull;
    double out[RW], cml = 0.0;
    for (int ch = 0; ch < a.n_chunks; ++ch) {
        o0 = as_const(a.chunk_op0)[ch];
        const int o1 = as_const(a.chunk_op0)[ch + 1];
        __syncthreads();
        if constexpr (CODED) {
            const int u0 = as_const(a.chunk_tip0)[ch], nu = as_const(a.chunk_tip0)[ch + 1] - u0;
            uint32_t *w32 = reinterpret_cast<uint32_t *>(codes_l);
            for (int k = threadIdx.x; k < nu * (kTile / 4); k += 64 * W) {
                const int uu = k >> 4, q = k & 15;
                const int tip = a.tip_seq[u0 + uu];
                w32[k] = *reinterpret_cast<const uint32_t *>(
                    a.codes + (size_t)tip * a.code_stride + (size_t)tile * kTile + 4 * q);
            }
            u = u_base = u0;
        }
        if constexpr (skip_zero) {
            uint32_t f = 1;
            const int o = o0 + lane;
            if (w == 0 && o < o1) {
                const int slot = o < a.n_ops ? a.ops[o].par_slot : a.n_store;
                if (slot >= 0) f = a.sflag[(size_t)(slot & ~kReadBack) * nwt + wt];
            }
            dirty_mask = __ballot(f != 0);
        }
        __syncthreads();
        for (int t = o0; t < o1; ++t) {
            const bool is_root = t == a.n_ops;
            const int par = ops[8 * t], pat = ops[8 * t + 1], ia = ops[8 * t + 2],
                      ib = ops[8 * t + 3], dst = ops[8 * t + 4];
            const cptr<double> Pa = Pw + (size_t)((a.store_mode & 16) ? 0 : 2 * t) * pside;
            const cptr<double> Pb = Pa + pside;
            const uint8_t *ca = codes_l + (u - u_base) * kTile + lane;
            const uint8_t *cb = ca + (pat == PAT_TT ? kTile : 0);
            u += pat == PAT_TT ? 2 : ((pat == PAT_CT || pat == PAT_MT) ? 1 : 0);
            // child kinds: 0 current, 1 tip, 2 stash, 3 HBM
            const int ka = pat == PAT_LC ? 2 : pat == PAT_CT ? 0 : pat == PAT_TT ? 1 : 3;
            const int kb = (pat == PAT_LC || pat == PAT_MC) ? 0 : pat == PAT_MM ? 3 : 1;
            double v[K], x[RW], y[RW], sa, sb;
            rows_child<K, CODED, generic>(a, ka, ia, table, ca, cur_l, stash_l, clv_w, scale_w,
                                          slot_stride, sstride, lane, site_c, v, sa);
            matvec_rows<K, RW>(Pa, v, x);
            // side b's P rows are loaded only after side a's product: both sides' rows would
            // not fit the SGPRs, and the compiler, left alone, hoists all the scalar loads and
            // spills them to VGPR lanes
            uintptr_t pb_addr = (uintptr_t)Pb;
            asm volatile("" : "+s"(pb_addr) : "v"(x[RW - 1]));
            const cptr<double> Pb2 = (cptr<double>)pb_addr;
            rows_child<K, CODED, generic>(a, kb, ib, table, cb, cur_l, stash_l, clv_w, scale_w,
                                          slot_stride, sstride, lane, site_c, v, sb);
            matvec_rows<K, RW>(Pb2, v, y);
            double m = 0.0;
#pragma unroll
            for (int r = 0; r < RW; ++r) {
                out[r] = x[r] * y[r];
                m = (r == 0 || out[r] > m || out[r] != out[r]) ? out[r] : m;
            }
            // np.max over all K rows (NaN propagates): combine the waves' maxima in row order
            red[w * kTile + lane] = m;
            __syncthreads();  // (A) every wave has read this op's inputs and posted its max
            m = red[lane];
#pragma unroll
            for (int q = 1; q < W; ++q) {
                const double o = red[q * kTile + lane];
                m = (o > m || o != o) ? o : m;
            }
            const double base = sa + sb;
            if (m < kScaleThreshold && m > 0.0) {
                cml = base + log(m);
#pragma unroll
                for (int r = 0; r < RW; ++r) out[r] = out[r] / m;
            } else {
                cml = base;
            }
            if (!is_root) {
                lds_put_rows<K, RW>(cur_l, lane, r0, out, cml, w == 0);
                if (dst >= 0)
                    lds_put_rows<K, RW>(stash_l + (size_t)dst * (K + 1) * kTile, lane, r0, out,
                                        cml, w == 0);
            }
            if (par >= 0 || is_root) {
                const int slot = is_root ? 0 : (par & ~kReadBack);
                const bool nt = is_root || (par & kReadBack) == 0;
                double *dclv = (is_root ? a.root_clv + row0 * K * kTile
                                        : clv_w + (size_t)slot * slot_stride) +
                               (size_t)(r0 / 2) * 2 * kTile;
                dbl2 *q = reinterpret_cast<dbl2 *>(dclv) + lane;
#pragma unroll
                for (int h = 0; h < RW / 2; ++h) {
                    const dbl2 tv = {out[2 * h], out[2 * h + 1]};
                    if (nt)
                        __builtin_nontemporal_store(tv, q + h * kTile);
                    else
                        q[h * kTile] = tv;
                }
                if (w == 0) {
                    double *dscale = is_root ? a.root_scale + row0 * kTile
                                             : scale_w + (size_t)slot * sstride;
                    bool write_scale = true;
                    if constexpr (skip_zero) {
                        const bool nz = __any(cml != 0.0);
                        const bool dirty = (dirty_mask >> (t - o0)) & 1;
                        write_scale = nz || dirty;
                        const int frow = is_root ? a.n_store : slot;
                        if (nz != dirty && lane == 0) a.sflag[(size_t)frow * nwt + wt] = nz;
                    }
                    if (write_scale) {
                        if (nt)
                            __builtin_nontemporal_store(cml, dscale + lane);
                        else
                            dscale[lane] = cml;
                    }
                }
            }
            __syncthreads();  // (B) the new current parent is complete
        }
    }
    // lnl_node (numba_likelihood_engine.py:82-87): sum over all K rows, wave by wave in row
    // order, then the category's log weight; k_site_lse combines the categories
    const cptr<double> pi = as_const(a.pi) + r0;
    double f = 0.0;
#pragma unroll
    for (int r = 0; r < RW; ++r) f = fma(out[r], pi[r], f);
    red[w * kTile + lane] = f;
    __syncthreads();
    if (w == 0 && tile < n_tiles) {
        double ft = 0.0;
        for (int q = 0; q < W; ++q) ft += red[q * kTile + lane];
        const double sw = ((ft > 0.0) ? log(ft) + cml : -INFINITY) + as_const(a.logw)[cat];
        a.cat_lnl[(size_t)cat * n_tiles * kTile + site] = sw;
    }
}

// categories of a site combined when they are not all in one traversal workgroup
__global__ void __launch_bounds__(kBlock)
    k_site_lse(int C, int64_t S, int64_t S_pad, const double *__restrict__ cat_lnl,
               const double *__restrict__ pattern_w, double *__restrict__ site_lnl,
               double *__restrict__ block_sum) {
    __shared__ double red[kWaves];
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double contrib = 0.0;
    if (s < S) {
        const double l = lse_strided(cat_lnl + s, C, S_pad);
        site_lnl[s] = l;
        contrib = pattern_w[s] * l;
    }
    const double t = block_sum_256(contrib, red);
    if (threadIdx.x == 0) block_sum[blockIdx.x] = t;
}

// tiled [C][n_tiles][K/2][64][2] CLV (+ [C][n_tiles][64] scaler) -> [S][C][K] (+ [S][C])
__global__ void __launch_bounds__(kBlock)
    k_untile(int K, int C, int64_t S, const double *__restrict__ clv,
             const double *__restrict__ scale, double *__restrict__ out,
             double *__restrict__ out_scale) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // (site, cat)
    if (e >= S * C) return;
    const int64_t s = e / C;
    const int c = (int)(e - s * C);
    const int64_t n_tiles = tile_count(S);
    const size_t row = (size_t)c * n_tiles + s / kTile;
    const int l = (int)(s % kTile);
    const double *src = clv + row * K * kTile;
    for (int i = 0; i < K; ++i) out[e * K + i] = src[(i / 2) * 2 * kTile + 2 * l + (i & 1)];
    if (out_scale) out_scale[e] = scale[row * kTile + l];
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


template <int K, bool CODED, int W>
int launch_prune_w(hipStream_t st, int variant, const TraverseArgs &a, int grid, size_t lds) {
    switch (variant) {
        case 0: hipLaunchKernelGGL((k_prune<K, CODED, 0, W>), dim3(grid), dim3(kBlock), lds, st, a); break;
        case TV_SKIP_ZERO_SCALE: hipLaunchKernelGGL((k_prune<K, CODED, TV_SKIP_ZERO_SCALE, W>), dim3(grid), dim3(kBlock), lds, st, a); break;
        case TV_GENERIC: hipLaunchKernelGGL((k_prune<K, CODED, TV_GENERIC, W>), dim3(grid), dim3(kBlock), lds, st, a); break;
        case TV_GENERIC | TV_SKIP_ZERO_SCALE: hipLaunchKernelGGL((k_prune<K, CODED, TV_GENERIC | TV_SKIP_ZERO_SCALE, W>), dim3(grid), dim3(kBlock), lds, st, a); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

template <int K, int RW, bool CODED>
int launch_rows_k(hipStream_t st, int variant, const TraverseArgs &a) {
    const size_t lds = RowsLds<K, RW>(a.n_codes, a.max_chunk_uses, CODED, a.n_lds).total;
    const dim3 grid((unsigned)(a.n_tiles * a.C)), block(64 * (K / RW));
    switch (variant) {
        case 0: hipLaunchKernelGGL((k_prune_rows<K, RW, CODED, 0>), grid, block, lds, st, a); break;
        case TV_SKIP_ZERO_SCALE: hipLaunchKernelGGL((k_prune_rows<K, RW, CODED, TV_SKIP_ZERO_SCALE>), grid, block, lds, st, a); break;
        case TV_GENERIC: hipLaunchKernelGGL((k_prune_rows<K, RW, CODED, TV_GENERIC>), grid, block, lds, st, a); break;
        case TV_GENERIC | TV_SKIP_ZERO_SCALE: hipLaunchKernelGGL((k_prune_rows<K, RW, CODED, TV_GENERIC | TV_SKIP_ZERO_SCALE>), grid, block, lds, st, a); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

template <int K, bool CODED>
int launch_prune_k(hipStream_t st, int variant, const TraverseArgs &a, int grid) {
    const size_t lds =
        TravLds(K, a.n_codes, a.max_chunk_uses, CODED, a.n_lds, a.C).total + a.lds_pad;
    switch (a.waves) {
        case 7: return launch_prune_w<K, CODED, 7>(st, variant, a, grid, lds);
        case 8: return launch_prune_w<K, CODED, 8>(st, variant, a, grid, lds);
        default: return launch_prune_w<K, CODED, 1>(st, variant, a, grid, lds);
    }
}

}  // namespace

bool traverse_supported(int K) { return K == 2 || K == 4 || K == 20; }

size_t traverse_lds_bytes(int K, int C, int n_codes, int max_chunk_uses, bool coded, int n_lds) {
    if (K == 20) return RowsLds<20, 2>(n_codes, max_chunk_uses, coded, n_lds).total;
    return TravLds(K, n_codes, max_chunk_uses, coded, n_lds, C).total;
}

int launch_traverse(hipStream_t st, int K, bool coded, int variant, const TraverseArgs &a,
                    int grid) {
    int rc;
    switch (K) {
        case 2: rc = coded ? launch_prune_k<2, true>(st, variant, a, grid) : launch_prune_k<2, false>(st, variant, a, grid); break;
        case 4: rc = coded ? launch_prune_k<4, true>(st, variant, a, grid) : launch_prune_k<4, false>(st, variant, a, grid); break;
        case 20: rc = coded ? launch_rows_k<20, 2, true>(st, variant, a) : launch_rows_k<20, 2, false>(st, variant, a); break;
        default: return (int)hipErrorInvalidValue;
    }
    if (rc || !a.cat_lnl) return rc;
    const int64_t nb = (a.S + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_site_lse, dim3((unsigned)nb), dim3(kBlock), 0, st, a.C, a.S,
                       (int64_t)a.n_tiles * kTile, a.cat_lnl, a.pattern_w, a.site_lnl,
                       a.block_sum);
    return (int)hipGetLastError();
}

bool traverse_per_category(int K, int C) { return K == 20 || 4 % C != 0; }

int traverse_block_sums(int K, int C, int64_t S) {
    return !traverse_per_category(K, C) ? (int)((tile_count(S) * C + kWaves - 1) / kWaves)
                                        : (int)((S + kBlock - 1) / kBlock);
}

int launch_untile(hipStream_t st, int K, int C, int64_t S, const double *clv,
                  const double *scale, double *out, double *out_scale) {
    const int64_t n = S * C;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_untile, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       st, K, C, S, clv, scale, out, out_scale);
    return (int)hipGetLastError();
}

int launch_pmatrix(hipStream_t st, const PmatArgs &a) {
    const dim3 grid(a.n_sides, a.C);
    switch (a.K) {
        case 2: hipLaunchKernelGGL(k_pmatrix<2>, grid, dim3(64), 0, st, a); break;
        case 4: hipLaunchKernelGGL(k_pmatrix<4>, grid, dim3(64), 0, st, a); break;
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
