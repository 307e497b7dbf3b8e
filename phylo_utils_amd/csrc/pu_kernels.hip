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

// The in-launch hand-offs (k_prune / k_prune_mfma chain roots to the top task, the protein
// per-tile category combine) publish with NO release: every byte is stored write-through
// (`sc1`), every storing wave waits `s_waitcnt vmcnt(0)`, a workgroup barrier, then ONE relaxed
// agent-scope add; only the last arriver acquires (agent fence = `buffer_inv sc1`) before its
// loads.  Under the HIP/C++ model that is a race; it is correct on gfx950 because an sc1 store
// has left the CU's write path for the coherent level once vmcnt(0) retires it
// (MI355X_MICROARCH.md, "Valid forms": producer sc1 stores + drained vmcnt + counter after every
// wave's wait, consumer one acquire).  A release in its place costs an L2 write-back per XCD
// (measured 0.91 vs 0.33 ms on cfg3).  Any other target must not build these kernels.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "pu_kernels.hip: the chain / category hand-offs rely on gfx950 sc1 store semantics"
#endif

#include <type_traits>

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

// rescale rule of numba_likelihood_engine.py:37-44 on a finished product vector.
// FMAX (lnL-only traversals): v_max_f64, which skips NaN where np.max propagates it.  The
// lnL cannot differ: a NaN entry makes every entry of every ancestor NaN, so the site's
// root sum f is NaN and its lnL -inf whatever the scalers; nothing else is returned.
// (r06: the protein kernel's wave-uniform "every entry below the threshold" pre-test, which
// skips this max, made the DNA traversal slower -- cfg2 0.1204-0.1236 vs 0.1110-0.1158 ms, cfg5
// unchanged, same box, alternating; profiles/r06_dna_ballot_ab.txt -- so K <= 4 keeps the
// direct form.)
template <int K, bool FMAX = false>
__device__ __forceinline__ void rescale(double (&out)[K], double sa, double sb, double &cml) {
    double m = out[0];  // np.max: NaN propagates
#pragma unroll
    for (int i = 1; i < K; ++i)
        m = FMAX ? __builtin_fmax(m, out[i]) : ((out[i] > m || out[i] != out[i]) ? out[i] : m);
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
// ---------------------------------------------------------------- P matrices
// P = (evecs * exp(evals * (t * r))) . ivecs for every side (one branch of one op) and
// category (abstract.py:99-105, 49-59): P[i][j] = sum_k fma(evecs[i][k] * exp(evals[k] t r),
// ivecs[k][j]) in k order -- the form every P builder here (and pu_edge's) shares bitwise.
//
// K = 2, 4: one lane per P row over the flattened [side][category][i] rows.  A lane takes the
// K exponentials of its (side, category), its row's K entries, and -- with tip products
// (TV_PTIP) -- row i of every code's product PT[side][cat][code][i] from the entries it holds.
// No LDS and no barrier, so every global load of a lane (branch length, rate, eigen-system)
// is in flight at once: one memory round trip per launch.  (r06: the r01-r05 form took one
// lane per P entry and per PT entry, each with its own K exponentials and its own P row: 32
// exponentials per needed one with cfg5's 4 codes, 21.8 us of k_pmatrix_lane_trees per
// 125-tree launch; now 4.)  The arithmetic of each entry is unchanged, bit for bit.
template <int K>
__host__ __device__ inline int pmatrix_rows(int n_sides, int C) { return n_sides * C * K; }
template <int K, class AR>
__device__ __forceinline__ void pmatrix_lane(const AR &a, const int e) {
    if (e >= pmatrix_rows<K>(a.n_sides, a.C)) return;
    const int m = e / K, i = e - m * K;
    const int sd = m / a.C, c = m - sd * a.C;
    const double t = a.brlens[sd] * a.rates[c];
    // the eigen-system and the code table are wave-uniform: scalar loads, which a store does
    // not hold up (vector loads after the P stores waited for them, 10 us per batch launch)
    const cptr<double> ev = as_const(a.evals), U = as_const(a.evecs), V = as_const(a.ivecs);
    double p[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k)
            acc = fma(U[i * K + k] * exp(ev[k] * t), V[k * K + j], acc);
        p[j] = acc;
    }
    double *P = a.P + (size_t)e * K;
#pragma unroll
    for (int j = 0; j < K; ++j) P[j] = p[j];
    if (!a.PT) return;
    const int nc = a.n_codes;
    const cptr<double> tab = as_const(a.table);
    double *PT = a.PT + (size_t)m * nc * K + i;
    for (int code = 0; code < nc; ++code) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) acc = fma(p[j], tab[code * K + j], acc);
        PT[code * K] = acc;
    }
}
template <int K>
__global__ void __launch_bounds__(64) k_pmatrix_lane(PmatArgs a) {
    pmatrix_lane<K>(a, (int)(blockIdx.x * 64 + threadIdx.x));
}

// ---------------------------------------------------------------- whole traversal
// one whole OpDesc (32 bytes) per scalar load
typedef int int8v __attribute__((ext_vector_type(8)));

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
template <int K, class PM>
__device__ __forceinline__ void matvec_s(const PM &P, const double (&v)[K], double (&x)[K]) {
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) acc = fma(P[i * K + j], v[j], acc);
        x[i] = acc;
    }
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

// Cache policy of the streamed (write-once) CLV stores: 1 nt, 2 sc1 (written through the
// L2), 3 sc1 nt.  DNA (k_prune) takes sc1 nt: same box, alternating, cfg2 kernel 0.137-0.141
// -> 0.121-0.125 ms, cfg4 3.63 -> 3.35-3.40 ms (nt: the r01-r03 form; sc1 alone: no gain).
// Protein (k_prune_mfma) keeps nt: sc1 nt measured equal on cfg3, sc1 alone 20 % slower.
#ifndef PU_DNA_POL
#define PU_DNA_POL 3
#endif
#ifndef PU_AA_POL
#define PU_AA_POL 1
#endif
// the scaler stores of a streamed CLV (PU_DNA_SPOL, default: the CLV stores' policy)
#ifndef PU_DNA_SPOL
#define PU_DNA_SPOL PU_DNA_POL
#endif
__device__ __forceinline__ void store_scale_nt(double *p, double v) {
    if constexpr (PU_DNA_SPOL == 2)
        asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (PU_DNA_SPOL == 3)
        asm volatile("global_store_dwordx2 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    else
        __builtin_nontemporal_store(v, p);
}
template <int K>
__device__ __forceinline__ void store_tiled(double *base, int lane, const double (&v)[K],
                                            bool nt) {
    dbl2 *q = reinterpret_cast<dbl2 *>(base) + lane;
#pragma unroll
    for (int i = 0; i < K / 2; ++i) {
        const dbl2 t = {v[2 * i], v[2 * i + 1]};
        if (nt) {
            if constexpr (PU_DNA_POL == 2)
                asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(q + i * kTile), "v"(t)
                             : "memory");
            else if constexpr (PU_DNA_POL == 3)
                asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(q + i * kTile),
                             "v"(t)
                             : "memory");
            else
                __builtin_nontemporal_store(t, q + i * kTile);
        } else {
            q[i * kTile] = t;
        }
    }
}

// A chain root of a split plan: written through (sc1 stores, MI355X_MICROARCH.md) for the
// workgroup that runs the top task
template <int K>
__device__ __forceinline__ void store_tiled_wt(double *base, int lane, const double (&v)[K]) {
    dbl2 *q = reinterpret_cast<dbl2 *>(base) + lane;
#pragma unroll
    for (int i = 0; i < K / 2; ++i) {
        double *d = reinterpret_cast<double *>(q + i * kTile);
        __hip_atomic_store(d, v[2 * i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d + 1, v[2 * i + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// One child's vector from the code table (coded tips) or the dense tip array.
template <int K, bool CODED, class TA>
__device__ __forceinline__ void tip_vec(const TA &a, const double *table,
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
// PTIP: a coded tip child's product is one row of PT (k_pmatrix_lane), loaded from global
// memory (an lnL-only traversal has almost no stores for the load's wait to drain)
template <int K>
__device__ __forceinline__ void pt_row(const double *pt, const uint8_t *ucode, double (&x)[K]) {
    const dbl2 *row = reinterpret_cast<const dbl2 *>(pt + (int)*ucode * K);
#pragma unroll
    for (int i = 0; i < K / 2; ++i) {
        const dbl2 t = row[i];
        x[2 * i] = t.x;
        x[2 * i + 1] = t.y;
    }
}

// RS register stash slots follow the n_lds LDS slots (slot index n_lds + r, KEEP plans of the
// default build: keep_occupancy).  Two named register sets chosen by a wave-uniform branch:
// nothing is indexed or address-taken, so the slots stay in VGPRs.  (r04 kept them in an array
// reached through a pointer and a lambda: the compiler placed it in scratch memory, 88 bytes per
// lane of private segment; tests/test_kernel_isa.py now requires none.)
template <int K, int RS>
struct RegStash {
    double v0[K], v1[K], s0 = 0.0, s1 = 0.0;
    __device__ __forceinline__ RegStash() {
#pragma unroll
        for (int i = 0; i < K; ++i) v0[i] = v1[i] = 0.0;
    }
    __device__ __forceinline__ void get(int r, double (&v)[K], double &s) const {
        const bool one = RS > 1 && r > 0;
        // the selects act on register values: an empty asm keeps the compiler from turning
        // `one ? s1 : s0` into a load through a selected address, which pins the stash in
        // memory (it did for the scalers, and a select against an LDS stash slot then became
        // a flat load)
        double a0[K], a1[K], t0 = s0, t1 = s1;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            a0[i] = v0[i];
            a1[i] = v1[i];
            asm volatile("" : "+v"(a0[i]), "+v"(a1[i]));
        }
        asm volatile("" : "+v"(t0), "+v"(t1));
#pragma unroll
        for (int i = 0; i < K; ++i) v[i] = one ? a1[i] : a0[i];
        s = one ? t1 : t0;
    }
    __device__ __forceinline__ void put(int r, const double (&v)[K], double s) {
        if (RS > 1 && r > 0) {
#pragma unroll
            for (int i = 0; i < K; ++i) v1[i] = v[i];
            s1 = s;
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i) v0[i] = v[i];
            s0 = s;
        }
    }
};

// a tip child's product: a row of PT (PTIP) or P * its code-table row / dense tip vector
template <int K, bool CODED, bool PTIP, class PM, class TA>
__device__ __forceinline__ void tip_child(const TA &a, const double *table, const PM &P,
                                          const double *pt, const uint8_t *c, int tip,
                                          int64_t site_c, double (&o)[K]) {
    if constexpr (PTIP) {
        pt_row<K>(pt, c, o);
    } else {
        double v[K];
        tip_vec<K, CODED>(a, table, c, tip, site_c, v);
        matvec_s<K>(P, v, o);
    }
}

template <int K, bool CODED, bool GENERIC, bool PTIP = false, class PA = cptr<double>,
          int RS = 0, class TA = TraverseArgs>
__device__ __forceinline__ void op_children(const TA &a, int pat, int ia, int ib,
                                            const PA &Pa, cptr<double> Pb,
                                            const double (&cur)[K], double cur_s,
                                            const double *table, const uint8_t *ca,
                                            const uint8_t *cb, const double *stash_l,
                                            const double *clv_w, const double *scale_w,
                                            uint32_t srows, int lane,
                                            int64_t site_c, double (&x)[K], double (&y)[K],
                                            double &sa, double &sb, const double *pta,
                                            const double *ptb, const RegStash<K, RS> &rst) {
    double v[K];
    // One wave-uniform case per child pair: each case is straight-line code, so the dispatch
    // costs a compare chain instead of a web of flag tests per child (r04, fewer SALU)
    switch (pat) {
        case PAT_CT:
            matvec_s<K>(Pa, cur, x);
            sa = cur_s;
            tip_child<K, CODED, PTIP>(a, table, Pb, ptb, cb, ib, site_c, y);
            sb = 0.0;
            break;
        case PAT_LC:
            if (RS > 0 && ia >= a.n_lds)
                rst.get(ia - a.n_lds, v, sa);
            else
                stash_get<K>(stash_l + (size_t)ia * (K + 1) * kBlock, v, sa);
            matvec_s<K>(Pa, v, x);
            matvec_s<K>(Pb, cur, y);
            sb = cur_s;
            break;
        case PAT_TT:
            tip_child<K, CODED, PTIP>(a, table, Pa, pta, ca, ia, site_c, x);
            tip_child<K, CODED, PTIP>(a, table, Pb, ptb, cb, ib, site_c, y);
            sa = sb = 0.0;
            break;
        default:
            if constexpr (GENERIC) {  // PAT_MC, PAT_MT, PAT_MM: child a read back from HBM
                // slot offsets as 32-bit row counts (srows 64-site rows per scaler slot) and a
                // shift: fewer SGPRs than 64-bit multiplies by the slot strides
                const size_t oa = (size_t)((uint32_t)ia * srows) << 6;
                load_tiled<K>(clv_w + oa * K, lane, v);
                sa = scale_w[oa + lane];
                matvec_s<K>(Pa, v, x);
                if (pat == PAT_MC) {
                    matvec_s<K>(Pb, cur, y);
                    sb = cur_s;
                } else if (pat == PAT_MM) {
                    const size_t ob = (size_t)((uint32_t)ib * srows) << 6;
                    load_tiled<K>(clv_w + ob * K, lane, v);
                    sb = scale_w[ob + lane];
                    matvec_s<K>(Pb, v, y);
                } else {
                    tip_child<K, CODED, PTIP>(a, table, Pb, ptb, cb, ib, site_c, y);
                    sb = 0.0;
                }
            } else {
#pragma unroll
                for (int i = 0; i < K; ++i) x[i] = y[i] = 0.0;  // unreachable: host-picked variant
                sa = sb = 0.0;
            }
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
// SGPRs only 6 waves fit, see scripts/probes/occupancy_probe.hip -- at the cost of a few spills
// to VGPR lanes)
// The lnL sum without a k_reduce launch (TraverseArgs::red_slots, r06): the block sum t
// (valid in thread 0) goes out as two 8-byte words, a 32-bit half beside the launch's 32-bit
// generation each -- single-copy atomic, so a reader that sees the generation in both holds
// this launch's value, no drain and no ticket (1563 atomic adds on one counter cost more than
// the launch they saved: r03 / r04).  The grid's last workgroup, dispatched after
// every other one, waits for all red_n slots and adds them exactly as k_reduce does (thread i:
// slots i, i + 256, ..., then block_sum_256), so the lnL is k_reduce's, bit for bit.  Bounded
// waits: a slot that never arrives makes the lnL NaN.
template <int kPer, class TA>
__device__ __forceinline__ void fused_reduce(const TA &a, int bid, double t, double *red) {
    const double tt = __shfl(t, 0);
    const unsigned gen = a.red_gen;
    if (threadIdx.x < 2) {
        const uint64_t bits = (uint64_t)__double_as_longlong(tt);
        const uint64_t half = threadIdx.x ? bits >> 32 : bits & 0xffffffffull;
        __hip_atomic_store(a.red_slots + 2 * (size_t)bid + threadIdx.x,
                           ((uint64_t)gen << 32) | half, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if ((int)blockIdx.x != (int)gridDim.x - 1) return;
    double v = 0.0;
    bool ok = true;
    // Thread t adds slots t, t + 256, ... in that order, kPer of them requested together, then
    // only the missing ones again (by the time the last workgroup gets here nearly all have
    // arrived: one L2 round trip per kPer instead of per slot; cfg2: 1563 sums, 2 groups).
    // kPer 4: 8 would raise the traversal's VGPRs 65 -> 83 (7 -> 5 waves per SIMD); the
    // 7-wave and register-stash builds take 1 (no registers for the loads in flight).
    for (int base = threadIdx.x; base < a.red_n && ok; base += kPer * kBlock) {
        uint64_t lo[kPer], hi[kPer];
        unsigned pending = 0;
#pragma unroll
        for (int m = 0; m < kPer; ++m)
            if (base + m * kBlock < a.red_n) pending |= 1u << m;
        const unsigned all = pending;
        for (unsigned spins = 0;;) {
#pragma unroll
            for (int m = 0; m < kPer; ++m)
                if (pending >> m & 1) {
                    const size_t i = (size_t)base + m * kBlock;
                    lo[m] = __hip_atomic_load(a.red_slots + 2 * i, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
                    hi[m] = __hip_atomic_load(a.red_slots + 2 * i + 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
                }
#pragma unroll
            for (int m = 0; m < kPer; ++m)
                if ((pending >> m & 1) && (unsigned)(lo[m] >> 32) == gen &&
                    (unsigned)(hi[m] >> 32) == gen)
                    pending &= ~(1u << m);
            if (!pending) break;
            __builtin_amdgcn_s_sleep(1);
            if (++spins == (1u << 26)) {  // ≈ 1-2 s: only a lost workgroup ends here
                ok = false;
                break;
            }
        }
#pragma unroll
        for (int m = 0; m < kPer; ++m)
            if (all >> m & 1)
                v += __longlong_as_double((long long)((hi[m] << 32) | (lo[m] & 0xffffffffull)));
    }
    const double total = block_sum_256(ok ? v : __longlong_as_double(0x7ff8000000000000ll), red);
    if (threadIdx.x == 0) *a.red_out = total;
}

// TV_CHAIN (split plans, make_plan): block = task * blocks + bid; the workgroup runs its
// chain task, and the one that finishes the last chain of its tiles runs the top task, the
// root combine and the lnL (the hand-off as in k_prune_mfma: write-through chain roots, a
// relaxed ticket per workgroup tile set, one acquire).
// TA: TraverseArgs (a kernel argument) or its constant-address-space form (k_prune_trees)
template <int K, bool CODED, int V, int W, class TA>
__device__ __forceinline__ void prune_tree(const TA &a, const int bid0) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    constexpr bool skip_zero = (V & TV_SKIP_ZERO_SCALE) != 0;
    constexpr bool generic = (V & TV_GENERIC) != 0;  // HBM read-backs (PAT_M*) compiled in
    constexpr bool chain = (V & TV_CHAIN) != 0;
    constexpr bool ptip = CODED && (V & TV_PTIP) != 0;
    const int C = a.C;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int n_tiles = a.n_tiles;
    const int n_wtiles = block_tiles(C);  // tiles a workgroup can touch
    const int nwt = n_tiles * C;
#ifdef PU_WG_STAMPS  // diagnostic build: per-workgroup timeline (scripts/wg_timeline.py)
    const unsigned long long st_begin = __builtin_amdgcn_s_memrealtime();
    unsigned long long st_ops = 0, st_loop = 0;
#endif

    const TravLds LY(K, a.n_codes, a.max_chunk_uses, CODED, a.n_lds, C);
    double *table = reinterpret_cast<double *>(lds_raw);
    uint8_t *bcodes = lds_raw + LY.codes_off;  // [tile - tile0][chunk use][64]
    double *stash_l = reinterpret_cast<double *>(lds_raw + LY.stash_off) + threadIdx.x;
    double *lnl_x = reinterpret_cast<double *>(lds_raw + LY.lnl_off);

    if constexpr (CODED)
        for (int i = threadIdx.x; i < a.n_codes * K; i += kBlock) table[i] = a.table[i];

    const cptr<int> ops = as_const(reinterpret_cast<const int *>(a.ops));
    const size_t pside = (size_t)C * K * K;  // doubles per side (all categories)
    // TV_PTIP: this category's tip products, [side][cat][code][K]
    const size_t ptside = ptip ? (size_t)C * a.n_codes * K : 0, ptstep = 2 * ptside;
    const int pitch = a.tile_pitch;                            // tiles per layout row
    // 64-site rows per scaler slot (K per CLV slot); a slot index times it fits 32 bits
    const uint32_t srows = (uint32_t)(C * pitch);
    // TV_RSLOTS (KEEP plans of the default build at 4 workgroups per CU, VGPRs to spare): two
    // more waiting parents in registers (stash slots n_lds, n_lds + 1) -- fewer HBM read-backs
    // without LDS that would cost occupancy
    constexpr int RS = (V & TV_RSLOTS) ? 2 : 0;
    RegStash<K, RS> rst;

    int bid = bid0;
    int op_hi = a.n_ops, ch_lo = 0, ch_hi = a.n_chunks;
    if constexpr (chain) {
        const int nb = (a.n_tiles * C + kWaves - 1) / kWaves;
        const int task = bid / nb;
        bid -= task * nb;
        const cptr<int> tk = as_const(a.tasks) + 4 * task;
        op_hi = tk[1];
        ch_lo = tk[2];
        ch_hi = tk[3];
    }
    const int wt = __builtin_amdgcn_readfirstlane(bid * kWaves + wave);
    const int tile = wt / C;
    const int cat = wt - tile * C;
    const int tile0 = (bid * kWaves) / C;              // first tile of this workgroup
    const bool live = tile < n_tiles;
    const int64_t site = (int64_t)tile * kTile + lane;  // < n_tiles * 64 (padded arrays)
    const int64_t site_c = site < a.S ? site : a.S - 1;
    const uint8_t *wcodes = bcodes + (size_t)(tile - tile0) * a.max_chunk_uses * kTile;
    // The site's pattern weight, loaded and waited for before the first store (r05): loaded in
    // the epilogue, its wait (vmcnt counts loads and stores in issue order) held the workgroup
    // until every CLV store of its last ops had retired -- 4 us per workgroup at the end of
    // each dispatch round (scripts/wg_timeline.py)
    const double pw_site = (live && cat == 0 && site < a.S) ? a.pattern_w[site] : 0.0;
    asm volatile("" ::"v"(pw_site));
    const cptr<double> Pw = as_const(a.P) + (size_t)cat * K * K;
    const double *PTw = ptip ? a.PT + (size_t)cat * a.n_codes * K : nullptr;
    const size_t row0 = layout_row(K, C, pitch, cat, tile);
    double *clv_w = a.clv + row0 * K * kTile;
    double *scale_w = a.scale + row0 * kTile;

    double cur[K], cur_s = 0.0;  // the previous op's parent
#pragma unroll
    for (int i = 0; i < K; ++i) cur[i] = 0.0;
    double sw = -INFINITY;
    int o0 = 0;  // first op of the chunk
    uint64_t dirty_mask = ~0ull;
    // chunks [c0, c1) with ops below op_end; hand_off: the op whose parent (a chain root) is
    // written through (-1: none)
    auto run_chunks = [&](int c0, int c1, int op_end, int hand_off) __attribute__((always_inline)) {
    for (int ch = c0; ch < c1; ++ch) {
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
#ifdef PU_WG_STAMPS
        if (st_ops == 0) st_ops = __builtin_amdgcn_s_memrealtime();
#endif
        if (!live) continue;

        const int ob = o0;
        const int oe = min(o1, op_end);
        // descriptor and P pointers advance by a loop-invariant step (no per-op index
        // arithmetic on the scalar unit)
        const size_t pstep = 2 * pside;
        cptr<int> opp = ops + 8 * (size_t)ob;
        cptr<double> Pa = Pw + (size_t)ob * pstep;
        const double *pta = ptip ? PTw + (size_t)ob * ptstep : nullptr;
        for (int t = ob; t < oe; ++t, opp += 8, Pa += pstep, pta += ptip ? ptstep : 0) {
            const int par = opp[0], pat = opp[1], ia = opp[2], ib = opp[3], dst = opp[4];
            const cptr<double> Pb = Pa + pside;
            const uint8_t *ca = wcodes + opp[5] * kTile + lane;  // OpDesc::use0
            const uint8_t *cb = ca + (pat == PAT_TT ? kTile : 0);
            double x[K], y[K], sa, sb;
            op_children<K, CODED, generic, ptip, cptr<double>, RS>(
                a, pat, ia, ib, Pa, Pb, cur, cur_s, table, ca, cb, stash_l, clv_w, scale_w,
                srows, lane, site_c, x, y, sa, sb, pta,
                pta + (ptip ? ptside : 0), rst);
#pragma unroll
            for (int i = 0; i < K; ++i) cur[i] = x[i] * y[i];
            rescale<K, ptip>(cur, sa, sb, cur_s);
            if (dst >= 0) {
                if (RS > 0 && dst >= a.n_lds)
                    rst.put(dst - a.n_lds, cur, cur_s);
                else
                    stash_put<K>(stash_l + (size_t)dst * (K + 1) * kBlock, cur, cur_s);
            }
            if (par >= 0) {
                // the slot's byte offset from the descriptor (OpDesc::par_off); the scaler
                // slot is 1 / K of it
                const uint64_t off = *reinterpret_cast<cptr<uint64_t>>(opp + 6);
                double *dclv = reinterpret_cast<double *>(reinterpret_cast<char *>(clv_w) + off);
                double *dscale = reinterpret_cast<double *>(reinterpret_cast<char *>(scale_w) +
                                                            (off >> (K == 4 ? 2 : 1)));
                bool write_scale = true;
                if constexpr (skip_zero) {
                    // an all-zero scaler wave tile whose memory is already zero is skipped: one
                    // ballot and the chunk's dirty bit of this op (the mask shifts per op)
                    const uint64_t nzm = __ballot(cur_s != 0.0);
                    const uint64_t dbit = dirty_mask & 1;
                    write_scale = (nzm | dbit) != 0;
                    if (write_scale && (nzm != 0) != (dbit != 0) && lane == 0)
                        a.sflag[(size_t)(par & ~kReadBack) * nwt + wt] = nzm != 0;
                }
                // one wave-uniform branch per op picks the store form: a chain root written
                // through for the top task, a CLV read back in this run cached, every other
                // one streamed past the caches
                if (chain && t == hand_off) {
                    store_tiled_wt<K>(dclv, lane, cur);
                    if (write_scale)
                        __hip_atomic_store(dscale + lane, cur_s, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                } else if ((par & kReadBack) == 0) {
                    store_tiled<K>(dclv, lane, cur, true);
                    if (write_scale) store_scale_nt(dscale + lane, cur_s);
                } else {
                    store_tiled<K>(dclv, lane, cur, false);
                    if (write_scale) dscale[lane] = cur_s;
                }
            }
            if constexpr (skip_zero) dirty_mask >>= 1;
        }
    }
    };
    // one instance of the op loop for both phases (a second inlined copy cost SGPR spills)
    int c0 = ch_lo, c1 = ch_hi, op_end = op_hi, hand_off = chain ? op_hi - 1 : -1;
    for (int phase = 0;; ++phase) {
        run_chunks(c0, c1, op_end, hand_off);
        if (!chain || phase == 1) break;
        __shared__ int last_arrival;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            const int prev = __hip_atomic_fetch_add(a.ticket + bid, 1, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
            last_arrival = prev == a.n_tasks - 1;
            if (last_arrival) {
                __hip_atomic_store(a.ticket + bid, 0, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
        if (!last_arrival) return;
        c0 = as_const(a.tasks)[4 * a.n_tasks + 2];  // the top task
        c1 = a.n_chunks;
        op_end = a.n_ops;
        hand_off = -1;
    }
#ifdef PU_WG_STAMPS
    st_loop = __builtin_amdgcn_s_memrealtime();
#endif
    if (live) {
        // root combine (tree_model.py:189-197): the last descriptor, in the last chunk
        const int t = a.n_ops;
        const int pat = ops[8 * t + 1], ia = ops[8 * t + 2], ib = ops[8 * t + 3];
        const cptr<double> Pa = Pw + (size_t)(2 * t) * pside;
        const cptr<double> Pb = Pa + pside;
        const uint8_t *ca = wcodes + ops[8 * t + 5] * kTile + lane;  // OpDesc::use0
        const uint8_t *cb = ca + (pat == PAT_TT ? kTile : 0);
        double x[K], y[K], sa, sb;
        const double *pta = ptip ? PTw + (size_t)t * ptstep : nullptr;
        op_children<K, CODED, generic, ptip, cptr<double>, RS>(
            a, pat, ia, ib, Pa, Pb, cur, cur_s, table, ca, cb, stash_l, clv_w, scale_w,
            srows, lane, site_c, x, y, sa, sb, pta, pta + (ptip ? ptside : 0),
            rst);
        double out[K], cml;
#pragma unroll
        for (int i = 0; i < K; ++i) out[i] = x[i] * y[i];
        rescale<K, ptip>(out, sa, sb, cml);
        // root_clv null (pu_batch, r06): nothing reads the root partials of a batched lnL-only
        // tree, so they are not written (cfg5: 1.0 of 4.84 GB per 125-tree launch)
        if (a.root_clv) {
            store_tiled<K>(a.root_clv + row0 * K * kTile, lane, out, true);
            bool write_scale = true;
            if constexpr (skip_zero) {
                const bool nz = __any(cml != 0.0);
                const bool dirty = dirty_mask & 1;  // shifted once per op of the chunk
                write_scale = nz || dirty;
                if (nz != dirty && lane == 0) a.sflag[(size_t)a.n_store * nwt + wt] = nz;
            }
            if (write_scale) store_scale_nt(a.root_scale + row0 * kTile + lane, cml);
        }
        // lnl_node (numba_likelihood_engine.py:82-87) plus the category's log weight
        const cptr<double> pi = as_const(a.pi);
        double f = 0.0;
#pragma unroll
        for (int i = 0; i < K; ++i) f = fma(out[i], pi[i], f);
        sw = ((f > 0.0) ? log(f) + cml : -INFINITY) + as_const(a.logw)[cat];
    }

    if (a.cat_lnl) {  // 4 % C != 0: a tile's categories span workgroups (k_site_lse)
        if (live) a.cat_lnl[(size_t)cat * n_tiles * kTile + site] = sw;
    } else {
        // per-pattern logsumexp over categories (tree_model.py:216), pattern-weighted block
        // sum; the C waves of a tile are in this workgroup (lnl_x aliases codes and stash)
        __syncthreads();
        lnl_x[threadIdx.x] = sw;
        __syncthreads();
        double contrib = 0.0;
        if (live && cat == 0 && site < a.S) {
            const double l = lse_strided(lnl_x + wave * 64 + lane, C, 64);
            a.site_lnl[site] = l;
            contrib = pw_site * l;
        }
        const double t = block_sum_256(contrib, lnl_x + kBlock);
        // single-tree DNA launches only (K = 2 builds would take a stack frame; a batch sums
        // in k_reduce_trees)
        if constexpr (K == 4 && !chain && std::is_same<TA, TraverseArgs>::value) {
            if (a.red_slots) {
                fused_reduce<(W == 7 || (V & TV_RSLOTS)) ? 1 : 4>(a, bid, t, lnl_x + kBlock);
            } else if (threadIdx.x == 0) {
                a.block_sum[bid] = t;
            }
        } else {
            if (threadIdx.x == 0) a.block_sum[bid] = t;
        }
    }
#ifdef PU_WG_STAMPS
    if (threadIdx.x == 0 && a.timing) {  // vector stores of lane 0
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        unsigned long long *o = a.timing + 8 * (size_t)blockIdx.x;
        o[0] = st_begin;
        o[1] = st_ops;
        o[2] = st_loop;
        o[3] = __builtin_amdgcn_s_memrealtime();
        o[4] = hw;
        o[5] = xcc;
    }
#endif
}

template <int K, bool CODED, int V, int W>
__global__ void __launch_bounds__(kBlock, W) k_prune(TraverseArgs a) {
    prune_tree<K, CODED, V, W>(a, blockIdx.x);
}

// Several trees in one launch: tree t's workgroups are blocks
// [t * blocks, (t + 1) * blocks) of the grid, each a whole traversal of that tree's tile and
// category exactly as k_prune runs it (same arithmetic and order: every value, the block sums
// and so the lnL bitwise those of the tree's own launch).  The per-tree arguments are read
// through the constant address space (scalar loads, like a kernel argument).
template <int K, bool CODED, int V, int W>
__global__ void __launch_bounds__(kBlock, W)
    k_prune_trees(const TraverseArgs *__restrict__ trees, int blocks, int n_trees, int group) {
    // groups of `group` trees in turn; inside a group the trees' workgroups of one tile index
    // are adjacent (block = b * g + tree), so the dispatcher's round-robin over the 8 XCDs
    // keeps a tree on one XCD when g % 8 == 0 and each XCD's L2 holds g / 8 trees' P and tip
    // products; group 0: tree-major (block = tree * blocks + b)
    const int x = (int)blockIdx.x;
    int t, b;
    if (group > 0) {
        const int gi = x / (group * blocks), r = x - gi * group * blocks;
        const int g = min(group, n_trees - gi * group);  // (the last group may be smaller)
        t = gi * group + r % g;
        b = r / g;
    } else {
        t = x / blocks;
        b = x - t * blocks;
    }
    t = __builtin_amdgcn_readfirstlane(t);
    b = __builtin_amdgcn_readfirstlane(b);
    const auto &a = *as_const(trees + t);
    prune_tree<K, CODED, V, W>(a, b);
}

// ---------------------------------------------------------------- protein traversal (MFMA)
// K = 20 on the fp64 matrix cores.  One wave owns one rate category of 16 sites; the K-vector
// of a site is spread over the 4 lane groups g = lane >> 4: lane (g, s = lane & 15) holds
// rows g, g+4, g+8, g+12 and 16+g.  That is exactly where v_mfma_f64_16x16x4_f64 leaves its
// result (D: col = lane & 15, row = (lane >> 4) + 4 * reg -- cdna_hip_programming.md) and
// exactly the B operand the next op's k-steps need (B: k = lane >> 4, col = lane & 15), so a
// parent feeds its consumer with no lane movement.  x = P v is 5 k-steps of one 16x16x4 tile
// (rows 0..15) and one 4x4x4_4b product (rows 16..19, which land in the same lanes):
// 10 MFMAs per child, no padded rows (mfma_step).
//
// P enters as the A operands (10 doubles per lane and side, laid out by k_pa) and is
// prefetched one op ahead.  Those loads and the CLV stores are issued by inline asm with
// counted s_waitcnt vmcnt(N): vector-memory operations retire in issue order on gfx950
// (MI355X_MICROARCH.md), so waiting for a prefetch never waits for the stores issued after
// it -- the compiler, which only sees mixed loads and stores, would wait for zero.
typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kAaRows = 5;   // doubles per lane of a protein CLV
constexpr int kAaSites = 16; // sites per wave

// Vector-memory operations with a wave-uniform base in SGPRs, the lane's byte offset in one
// VGPR and an immediate offset (no 64-bit per-lane addresses held in registers)
// (the PU_CHECK build makes the base provably uniform: its checks hide that from the compiler)
template <typename T>
__device__ __forceinline__ T *uniform_ptr(T *p) {
#if defined(PU_CHECK) || defined(PU_TIMING_BUILD)
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (T *)(((uint64_t)hi << 32) | lo);
#else
    return p;
#endif
}
template <int OFF>
__device__ __forceinline__ void asm_ld4(dbl2 &v, uint32_t voff, const double *sbase) {
    sbase = uniform_ptr(sbase);
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3"
                 : "=v"(v)
                 : "v"(voff), "s"(sbase), "n"(OFF)
                 : "memory");
}
// store policy POL: 0 plain, 1 streamed (nt), 2 write-through (sc1: visible to another CU
// after this wave's vmcnt(0) wait without an agent release, MI355X_MICROARCH.md)
template <int OFF, int POL>
__device__ __forceinline__ void asm_st2(uint32_t voff, double *sbase, double v) {
    sbase = uniform_ptr(sbase);
    if constexpr (POL == 1)
        asm volatile("global_store_dwordx2 %0, %1, %2 offset:%3 nt" ::"v"(voff), "v"(v),
                     "s"(sbase), "n"(OFF)
                     : "memory");
    else if constexpr (POL == 3)
        asm volatile("global_store_dwordx2 %0, %1, %2 offset:%3 sc1 nt" ::"v"(voff), "v"(v),
                     "s"(sbase), "n"(OFF)
                     : "memory");
    else if constexpr (POL == 2)
        asm volatile("global_store_dwordx2 %0, %1, %2 offset:%3 sc1" ::"v"(voff), "v"(v),
                     "s"(sbase), "n"(OFF)
                     : "memory");
    else
        asm volatile("global_store_dwordx2 %0, %1, %2 offset:%3" ::"v"(voff), "v"(v),
                     "s"(sbase), "n"(OFF)
                     : "memory");
}

// A operands of one side (k-step q: {row block 0, row block 1}), prefetched one op ahead;
// voff = 16 lane, voff4 = voff + 4096 (past the 13-bit immediate)
__device__ __forceinline__ void pa_load(dbl2 (&r)[5], const double *base, uint32_t voff,
                                        uint32_t voff4) {
    asm_ld4<0>(r[0], voff, base);
    asm_ld4<1024>(r[1], voff, base);
    asm_ld4<2048>(r[2], voff, base);
    asm_ld4<3072>(r[3], voff, base);
    asm_ld4<0>(r[4], voff4, base);
}

// a 16-byte store of a lane (POL as asm_st2); the s_nop keeps the compiler's next instruction
// from overwriting the data registers before the store has read them
template <int OFF, int POL>
__device__ __forceinline__ void asm_st4(uint32_t voff, double *sbase, dbl2 v) {
    sbase = uniform_ptr(sbase);
    if constexpr (POL == 1)
        asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3 nt\n\ts_nop 1" ::"v"(voff),
                     "v"(v), "s"(sbase), "n"(OFF)
                     : "memory");
    else if constexpr (POL == 3)
        asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3 sc1 nt\n\ts_nop 1" ::"v"(voff),
                     "v"(v), "s"(sbase), "n"(OFF)
                     : "memory");
    else if constexpr (POL == 2)
        asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3 sc1\n\ts_nop 1" ::"v"(voff),
                     "v"(v), "s"(sbase), "n"(OFF)
                     : "memory");
    else
        asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3\n\ts_nop 1" ::"v"(voff), "v"(v),
                     "s"(sbase), "n"(OFF)
                     : "memory");
}

// the 5 rows of a lane (+ the site's scaler) to a tiled protein slot (aa_row_off): kAaStores
// stores on either path (streamed past the caches unless the slot is read back in this run)
constexpr int kAaStores = 4;
template <int POL>
__device__ __forceinline__ void aa_store6(double *clv_base, double *scale_base, uint32_t voff,
                                          uint32_t soff, const double (&o)[5], double cml) {
    asm_st4<0, POL>(2 * voff, clv_base, dbl2{o[0], o[1]});
    asm_st4<1024, POL>(2 * voff, clv_base, dbl2{o[2], o[3]});
    asm_st2<2048, POL>(voff, clv_base, o[4]);
    asm_st2<0, POL>(soff, scale_base, cml);  // 4 lanes per site, same value
}
__device__ __forceinline__ void aa_store(double *clv_base, double *scale_base, uint32_t voff,
                                         uint32_t soff, const double (&o)[5], double cml,
                                         bool nt) {
    if (nt)
        aa_store6<PU_AA_POL>(clv_base, scale_base, voff, soff, o, cml);
    else
        aa_store6<0>(clv_base, scale_base, voff, soff, o, cml);
}

// wait until at most N vector-memory operations are outstanding.  No operands (tied "+v"
// operands made the compiler copy the in-flight registers into fresh ones ahead of the
// wait); the scheduling barrier keeps every use of the P registers below it.
template <int N>
__device__ __forceinline__ void pa_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// NaN-propagating max (np.max) of this lane's value and the lane `lane ^ 16` (X = 16) or
// `lane ^ 32` (X = 32): v_permlane{16,32}_swap of a register with itself leaves the pair's
// two values in the two results, in lane-dependent order -- both lanes then hold the max
// of the same pair
template <int X>
__device__ __forceinline__ double pair_max(double m) {
    const uint32_t lo = __double2loint(m), hi = __double2hiint(m);
    auto l2 = X == 16 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false)
                      : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto h2 = X == 16 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false)
                      : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const double a = __hiloint2double(h2[0], l2[0]), b = __hiloint2double(h2[1], l2[1]);
    return (b > a || b != b) ? b : a;
}

// x = P v on the matrix cores: v is this lane's 5 rows of the child.  Rows 0..15 are one
// 16x16x4 tile per k-step (x0: row (lane >> 4) + 4 reg); rows 16..19 are a 4x4x4_4b product
// per k-step -- 4 blocks of 4 sites, A lane 16k + 4b + i = P[16 + i][4q + k], B lane
// 16k + 4b + j = v[4q + k] of site 4b + j (this lane's v[q]), D lane 16i + 4b + j = row
// 16 + i of site 4b + j, i.e. this lane's row 16 + (lane >> 4) (layout measured by
// scripts/probes/mfma_f64_probe.hip).  The 4x4x4_4b form runs at ~1.6x the FLOP rate of 16x16x4 on
// gfx950 and pads nothing, where a second 16-row tile would compute 12 zero rows.
//
// Both children's products are interleaved per k-step (4 independent accumulation chains in
// flight), and each A operand register is refilled with op t + 1's value as soon as its MFMA
// has issued: the prefetch then has a whole op to land.  na / nb: op t + 1's operands.
template <int Q, bool PREFETCH>
__device__ __forceinline__ void mfma_step(dbl2 (&PA)[5], dbl2 (&PB)[5], const double (&va)[5],
                                          const double (&vb)[5], d4 &x0, double &x4, d4 &y0,
                                          double &y4, const double *na, const double *nb,
                                          uint32_t poff, uint32_t poff4) {
    x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(PA[Q].x, va[Q], x0, 0, 0, 0);
    y0 = __builtin_amdgcn_mfma_f64_16x16x4f64(PB[Q].x, vb[Q], y0, 0, 0, 0);
    x4 = __builtin_amdgcn_mfma_f64_4x4x4f64(PA[Q].y, va[Q], x4, 0, 0, 0);
    y4 = __builtin_amdgcn_mfma_f64_4x4x4f64(PB[Q].y, vb[Q], y4, 0, 0, 0);
    // nothing crosses this point: an MFMA reading the old operand scheduled after the load
    // of the new one would keep both alive, and the register allocator would then copy the
    // loop-carried operand at the top of the next op -- before its wait.  (The empty asm
    // "uses" the 4x4x4 accumulators: the MFMA intrinsics are pure, and the optimizer would
    // otherwise sink that chain past the barriers to its single use after the last step.)
    asm volatile("" : "+v"(x4), "+v"(y4));
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!PREFETCH) {
    } else if constexpr (Q < 4) {
        asm_ld4<Q * 1024>(PA[Q], poff, na);
        asm_ld4<Q * 1024>(PB[Q], poff, nb);
    } else {
        asm_ld4<0>(PA[Q], poff4, na);
        asm_ld4<0>(PB[Q], poff4, nb);
    }
    __builtin_amdgcn_sched_barrier(0);
}

// LDS of one protein workgroup (4 waves x 16 sites of one 64-site tile, one category):
//   [code table][tip codes: uses x 64][stash: per wave L x 6 x 64][lnl exchange]
struct AaLds {
    size_t codes_off, stash_off, total;
    __host__ __device__ AaLds(int K, int n_codes, int max_uses, bool coded, int n_lds) {
        codes_off = coded ? align16((size_t)n_codes * K * sizeof(double)) : 0;
        stash_off = codes_off + (coded ? align16((size_t)max_uses * kTile) : 0);
        total = stash_off + (size_t)kWaves * n_lds * (kAaRows + 1) * 64 * sizeof(double);
    }
};

// The counted waits need only a LOWER bound on the vector-memory operations issued after
// the awaited loads (retirement is in order): more operations -- the compiler's own loads of
// HBM read-backs (PAT_M*, which it waits for itself), or stores the count did not assume --
// only make a wait more conservative.
// MODE 0: PU_LNL_ONLY: assumes no stores; a parent stored for an HBM read-back makes the
//         next op's waits also drain those stores
// MODE 1: KEEP: every op stores its parent, exactly 6 stores per op
// MODE 2: waits for zero everywhere (PU_FORCE_GENERIC: the check of the counted modes)
// PU_CHECK diagnostic build: [p, p + n) must lie in [base, base + size); a violation is
// reported (once per wave, lane 0) and the caller substitutes a safe address
__device__ __forceinline__ bool in_bounds(const void *p, size_t n, const void *base,
                                          size_t size, int site, int t) {
#ifdef PU_CHECK
    const char *q = (const char *)p, *b = (const char *)base;
    const bool ok = q >= b && q + n <= b + size;
    if (!ok && (threadIdx.x & 63) == 0)
        printf("[pu check] site %d op %d block %d wave %d: %p + %zu outside [%p, +%zu)\n", site,
               t, (int)blockIdx.x, (int)(threadIdx.x >> 6), p, n, base, size);
    return ok;
#else
    return true;
#endif
}

// the same for a wave-uniform address (the result stays provably uniform)
__device__ __forceinline__ bool in_bounds_u(const void *p, size_t n, const void *base,
                                            size_t size, int site, int t) {
    return __builtin_amdgcn_readfirstlane((int)in_bounds(p, n, base, size, site, t)) != 0;
}

// CHAIN: a chain task of a split plan (make_plan): its last op is peeled like the root
// combine (no prefetch) and stores its parent.  The workgroup that finishes the last chain of
// its (tile, category) -- a ticket per (tile, category) -- then runs the top task (the ops
// above the chains, reading the chain roots back from HBM) and the lnL, so one launch does the
// whole traversal and the top's reads overlap other workgroups' chains.
template <bool CODED, int MODE, bool CHAIN = false>
__global__ void __launch_bounds__(kBlock, 3) k_prune_mfma(TraverseArgs a) {
    constexpr int K = 20;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    const int C = a.C;
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, s16 = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int wt = blockIdx.x;  // = [task * n_tiles * C +] tile * C + cat
    int op_lo = 0, op_hi = a.n_ops, ch_lo = 0, ch_hi = a.n_chunks;
    if constexpr (CHAIN) {
        const int task = wt / (a.n_tiles * C);
        wt -= task * a.n_tiles * C;
        const cptr<int> tk = as_const(a.tasks) + 4 * task;
        op_lo = tk[0];
        op_hi = tk[1];
        ch_lo = tk[2];
        ch_hi = tk[3];
    }
    const int tile = wt / C;
    const int cat = wt - tile * C;
    const int n_tiles = a.n_tiles;
    const int lsite = w * kAaSites + s16;  // site within the 64-site tile
    const int64_t site = (int64_t)tile * kTile + lsite;
    const int64_t site_c = site < a.S ? site : a.S - 1;

    const AaLds LY(K, a.n_codes, a.max_chunk_uses, CODED, a.n_lds);
    double *table = reinterpret_cast<double *>(lds_raw);
    uint8_t *codes_l = lds_raw + LY.codes_off;
    double *stash = reinterpret_cast<double *>(lds_raw + LY.stash_off) +
                    (size_t)w * a.n_lds * (kAaRows + 1) * 64 + lane;

    if constexpr (CODED)
        for (int i = threadIdx.x; i < a.n_codes * K; i += kBlock) table[i] = a.table[i];

    const cptr<int> ops = as_const(reinterpret_cast<const int *>(a.ops));
    // A-operand P: [side][cat][5][64][2], 2 (n_ops + 1) sides
    const size_t pa_side = (size_t)C * 5 * 128;
    const double *pa_w = a.Pa + (size_t)cat * 5 * 128;
    // protein CLV layout: per (slot, cat, tile) [wave 4][aa_row_off: 2.5 KB]; scaler [64 sites]
    const int pitch = a.tile_pitch;  // tiles per layout row
    const size_t slot_stride = (size_t)C * pitch * K * kTile;
    const size_t sstride = (size_t)C * pitch * kTile;
    const size_t row0 = layout_row(K, C, pitch, cat, tile);
    double *clv_w = a.clv + row0 * K * kTile + (size_t)w * kAaRows * 64;  // wave-uniform
    double *scale_w = a.scale + row0 * kTile + w * kAaSites;
    const uint32_t voff = lane * 8, soff = s16 * 8;  // byte offsets of the lane
    const uint32_t poff = lane * 16, poff4 = poff + 4096;

    // (r06: the next op's tip codes read one op ahead -- one LDS round trip less per tip
    // child -- made cfg3 slower, 0.3055-0.3070 vs 0.2979-0.2988 ms same box;
    // profiles/r06_cfg3_code_ahead_ab.txt.  Not kept.)
    // row index of this lane's 5 values: g, g+4, g+8, g+12, 16+g
    auto tip_rows = [&](const uint8_t *ucode, int tip, double (&v)[kAaRows]) {
        if constexpr (CODED) {
            const double *row = table + (int)*ucode * K + g;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = row[4 * r];
            v[4] = row[16];
        } else {
            const double *row = a.tips + ((size_t)tip * a.S + site_c) * K + g;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = row[4 * r];
            v[4] = row[16];
        }
    };
    // HBM read-back (PAT_M*): the compiler's loads, completed here -- the empty asm uses
    // the values, so the compiler's wait for them stays on this (rare) path instead of
    // landing among the prefetches of the common path
    auto hbm_rows = [&](int slot, double (&v)[kAaRows], double &sc) {
        const double *p = clv_w + (size_t)slot * slot_stride;
#pragma unroll
        for (int r = 0; r < kAaRows; ++r) v[r] = p[aa_row_off(r, lane)];
        sc = scale_w[(size_t)slot * sstride + s16];
        asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(sc));
    };

    double cur[kAaRows], cur_s = 0.0;
#pragma unroll
    for (int r = 0; r < kAaRows; ++r) cur[r] = 0.0;

    // P of op t is loaded during op t - 1, each A register as soon as op t - 1's MFMA has
    // read it (mfma_step).  The operations younger than op t's loads are then exactly op
    // t - 1's NS stores, so the wait at the top of op t never drains stores.  Every op of the
    // loop issues the same loads and stores on every path, and the root combine (which
    // prefetches nothing) is peeled off the loop: no P register merges paths with different
    // counts, and none is in flight when the loop ends.  Before the first op, NS stores into
    // this wave's root slot stand in for "the previous op's stores" (the root's own stores,
    // issued later, overwrite them in order).
    constexpr int NS = MODE == 1 ? kAaStores : 0;
    constexpr int WAIT = MODE == 2 ? 0 : NS;  // op t's P: only op t - 1's stores are younger
    double *root_cw = a.root_clv + row0 * K * kTile + (size_t)w * kAaRows * 64;
    double *root_sw = a.root_scale + row0 * kTile + w * kAaSites;
    dbl2 PA[5], PB[5];
    pa_load(PA, pa_w + (size_t)(2 * op_lo) * pa_side, poff, poff4);
    pa_load(PB, pa_w + (size_t)(2 * op_lo + 1) * pa_side, poff, poff4);
    if constexpr (CHAIN && MODE == 1) {
        // into the chain root's own slot, which this wave rewrites last: the root slot is the
        // top task's, and a stand-in store left in another XCD's L2 could land after it
        const int rs = ops[8 * (op_hi - 1)] & ~kReadBack;
        aa_store(clv_w + (size_t)rs * slot_stride, scale_w + (size_t)rs * sstride, voff, soff,
                 cur, 0.0, true);
    } else if constexpr (MODE == 1) {
        aa_store(root_cw, root_sw, voff, soff, cur, 0.0, true);
    }

    cptr<int> opp = ops + 8 * (size_t)op_lo;                 // op t's descriptor
    const double *pa_t = pa_w + (size_t)(2 * op_lo) * pa_side;  // op t's A operands
    // one op (the root combine: ROOT, no prefetch, the root slot)
    // debug timing (PU_TIMING_BUILD + PU_TIMING=1): wave 0 of workgroup 0 sums s_memtime per
    // op phase
#ifdef PU_TIMING_BUILD
    const bool timed = a.timing != nullptr && blockIdx.x == 0 && w == 0;
#else
    constexpr bool timed = false;  // (build with -DPU_TIMING_BUILD and run with PU_TIMING=1)
#endif
    unsigned long long tsum[6] = {0, 0, 0, 0, 0, 0}, tprev = 0;
    auto tmark = [&](int ph) {
        if (timed) {
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            if (ph > 0) tsum[ph] += now - tprev;
            tprev = now;
        }
    };
    // The children of an op that do not depend on the previous op's parent: a waiting parent
    // in the LDS stash, tips (staged code -> code table), HBM read-backs.  They are loaded one
    // op ahead, while the previous op's MFMAs execute, so an op starts with its operands in
    // registers (PAT_CT's child a and PAT_LC / PAT_MC's child b are the previous op's
    // parent, `cur`).  A stash slot an op reads is never the one the previous op writes: both
    // values are live across that op, so the planner gave them different slots.

    // one op; ROOT: the root combine (no P prefetch, the root slot); LAST: a chain's last op
    // (no P prefetch, its own slot)
    auto op = [&](int t, auto root_tag, auto last_tag) {
        constexpr bool ROOT = decltype(root_tag)::value;
        constexpr bool LAST = decltype(last_tag)::value;
        constexpr bool PREFETCH = !ROOT && !LAST;
        tmark(0);
        // the descriptor and P pointers advance by a loop-invariant step (ops run in order
        // within a phase): no per-op index multiplies on the scalar unit.  The whole 32-byte
        // descriptor arrives in one scalar load (r04; three loads, each waited for, before).
        const int8v d = *reinterpret_cast<cptr<int8v>>(opp);
        const int par = d[0], pat = d[1], ia = d[2], ib = d[3], dst = d[4];
        // op t + 1 (not at the root)
        const double *pn = pa_t + 2 * pa_side;
#ifdef PU_CHECK
        if (PREFETCH && !in_bounds_u(pn, (pa_side + 5 * 128) * 8, a.Pa, a.pa_bytes, 1, t)) pn = a.Pa;
#endif
        double va[kAaRows], vb[kAaRows], sa, sb;
        {  // the children straight into the MFMA operands, one straight-line case per child
           // pair (r04: the if-chains compiled to a web of flag tests on the scalar unit)
            const uint8_t *ca = codes_l + d[5] * kTile + lsite;  // OpDesc::use0
            auto take_cur = [&](double (&v)[kAaRows], double &s) {
#pragma unroll
                for (int r = 0; r < kAaRows; ++r) v[r] = cur[r];
                s = cur_s;
            };
            switch (pat) {
                case PAT_CT:
                    take_cur(va, sa);
                    tip_rows(ca, ib, vb);
                    sb = 0.0;
                    break;
                case PAT_LC: {
                    const double *p = stash + (size_t)ia * (kAaRows + 1) * 64;
#pragma unroll
                    for (int r = 0; r < kAaRows; ++r) va[r] = p[r * 64];
                    sa = p[kAaRows * 64];
                    take_cur(vb, sb);
                    break;
                }
                case PAT_TT:
                    tip_rows(ca, ia, va);
                    tip_rows(ca + kTile, ib, vb);
                    sa = sb = 0.0;
                    break;
                case PAT_MC:  // read back from HBM
                    hbm_rows(ia, va, sa);
                    take_cur(vb, sb);
                    break;
                case PAT_MT:
                    hbm_rows(ia, va, sa);
                    tip_rows(ca, ib, vb);
                    sb = 0.0;
                    break;
                default:  // PAT_MM
                    hbm_rows(ia, va, sa);
                    hbm_rows(ib, vb, sb);
            }
        }
        if (timed) {
            asm volatile("" ::"v"(va[0]), "v"(va[4]), "v"(vb[0]), "v"(vb[4]), "v"(sa), "v"(sb));
            tmark(1);
        }
        pa_wait<WAIT>();
        tmark(2);
        d4 x0 = {0.0, 0.0, 0.0, 0.0}, y0 = {0.0, 0.0, 0.0, 0.0};
        double x4 = 0.0, y4 = 0.0;
        const double *nb = pn + pa_side;
        mfma_step<0, PREFETCH>(PA, PB, va, vb, x0, x4, y0, y4, pn, nb, poff, poff4);
        mfma_step<1, PREFETCH>(PA, PB, va, vb, x0, x4, y0, y4, pn, nb, poff, poff4);
        mfma_step<2, PREFETCH>(PA, PB, va, vb, x0, x4, y0, y4, pn, nb, poff, poff4);
        mfma_step<3, PREFETCH>(PA, PB, va, vb, x0, x4, y0, y4, pn, nb, poff, poff4);
        mfma_step<4, PREFETCH>(PA, PB, va, vb, x0, x4, y0, y4, pn, nb, poff, poff4);
        if (timed) {
            asm volatile("" ::"v"(x0), "v"(y0), "v"(x4), "v"(y4));
            tmark(3);
        }
        double o[kAaRows];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = x0[r] * y0[r];
        o[4] = x4 * y4;
        // rescale (numba_likelihood_engine.py:40-44): a site whose np.max over its 20 rows m
        // has 0 < m < threshold.  That needs every row below the threshold, so (r06) a
        // wave-uniform test first: the lanes whose 5 rows are all below it, ANDed over the 4
        // lanes of a site -- no such site in the wave (the common case) means nothing rescales
        // and the NaN-propagating max (a long dependent chain of compares and lane swaps) is
        // skipped.  Otherwise the exact per-site rule below, as before.  Same box, three
        // alternating rounds (profiles/r06_cfg3_ballot_ab.txt): cfg3 traversal 0.3015-0.3033
        // vs 0.3152-0.3165 ms, lnL bitwise equal; the next op's descriptor requested one op
        // ahead as well made no difference (0.3012-0.3025) and was not kept.
        bool below = true;
#pragma unroll
        for (int r = 0; r < kAaRows; ++r) below &= o[r] < kScaleThreshold;
        const uint64_t lb = __ballot(below);
        const double base = sa + sb;
        double cml = base;
        if ((lb & (lb >> 16) & (lb >> 32) & (lb >> 48) & 0xFFFFull) != 0) {
            // np.max over the site's 20 rows (NaN propagates): this lane's 5, then lane groups
            double m = o[0];
#pragma unroll
            for (int r = 1; r < kAaRows; ++r) m = (o[r] > m || o[r] != o[r]) ? o[r] : m;
            m = pair_max<32>(pair_max<16>(m));
            if (m < kScaleThreshold && m > 0.0) {
                cml = base + log(m);
#pragma unroll
                for (int r = 0; r < kAaRows; ++r) o[r] = o[r] / m;
            }
        }
        if (timed) {
            asm volatile("" ::"v"(cml), "v"(o[0]), "v"(o[4]));
            tmark(4);
        }
        if constexpr (!ROOT) {
            if (dst >= 0) {
                double *p = stash + (size_t)dst * (kAaRows + 1) * 64;
#pragma unroll
                for (int r = 0; r < kAaRows; ++r) p[r * 64] = o[r];
                p[kAaRows * 64] = cml;
            }
            // the slot from the descriptor's byte offset (OpDesc::par_off: for K = 20 the
            // scaler slot's, the CLV slot's is 20 times it -- two shifts and an add instead
            // of two 64-bit multiplies on the scalar unit)
            uint64_t soffb = (uint64_t)(uint32_t)d[6] | ((uint64_t)(uint32_t)d[7] << 32);
#ifdef PU_CHECK
            const int slot = par & ~kReadBack;
            if ((MODE == 1 || par >= 0) &&
                (!in_bounds_u(clv_w + (size_t)slot * slot_stride, (4 * 64 + 64) * 8, a.clv,
                              a.clv_bytes, 2, t) ||
                 !in_bounds_u(scale_w + (size_t)slot * sstride, 16 * 8, a.scale, a.scale_bytes,
                              3, t)))
                soffb = 0;
#endif
            double *pclv = reinterpret_cast<double *>(reinterpret_cast<char *>(clv_w) +
                                                      ((soffb << 4) + (soffb << 2)));
            double *pscl = reinterpret_cast<double *>(reinterpret_cast<char *>(scale_w) + soffb);
            if constexpr (MODE == 1) {
                // KEEP: streamed, also the few read-back slots (a branch between the two store
                // forms would give the wait count two paths); a chain's root (LAST, peeled) is
                // written through for the top task in another workgroup
                aa_store6<LAST ? 2 : PU_AA_POL>(pclv, pscl, voff, soff, o, cml);
            } else if (LAST) {  // lnL only: a chain's root, written through for the top task
                aa_store6<2>(pclv, pscl, voff, soff, o, cml);
            } else if (par >= 0) {
                aa_store(pclv, pscl, voff, soff, o, cml, (par & kReadBack) == 0);
            }
        } else {
            aa_store6<PU_AA_POL>(root_cw, root_sw, voff, soff, o, cml);
        }
#pragma unroll
        for (int r = 0; r < kAaRows; ++r) cur[r] = o[r];
        cur_s = cml;
        opp += 8;
        pa_t = pn;
        tmark(5);
    };

    // chunks [c0, c1) with their staged tip codes, ops up to (excluding) `last`: the peeled op
    auto run_chunks = [&](int c0, int c1, int last) {
        for (int ch = c0; ch < c1; ++ch) {
            const int o0 = as_const(a.chunk_op0)[ch];
            const int o1f = as_const(a.chunk_op0)[ch + 1];  // the last chunk holds the peeled op
            const int o1 = min(o1f, last);
            __syncthreads();
            if constexpr (CODED) {
                const int u0 = as_const(a.chunk_tip0)[ch],
                          nu = as_const(a.chunk_tip0)[ch + 1] - u0;
                uint32_t *w32 = reinterpret_cast<uint32_t *>(codes_l);
                for (int k = threadIdx.x; k < nu * (kTile / 4); k += kBlock) {
                    const int uu = k >> 4, q = k & 15;
                    const int tip = a.tip_seq[u0 + uu];
                    w32[k] = *reinterpret_cast<const uint32_t *>(
                        a.codes + (size_t)tip * a.code_stride + (size_t)tile * kTile + 4 * q);
                }
            }
            __syncthreads();
            for (int t = o0; t < o1; ++t) op(t, std::false_type{}, std::false_type{});
        }
    };
    if constexpr (CHAIN) {
        run_chunks(ch_lo, ch_hi, op_hi - 1);
        op(op_hi - 1, std::false_type{}, std::true_type{});  // in its chunk, still staged
        // Ticket of this (tile, category), the hand-off of MI355X_MICROARCH.md's valid forms:
        // the chain root was stored write-through (sc1) and every wave waits for its stores,
        // so no release fence; after a barrier one lane adds to the ticket (agent scope,
        // relaxed); the workgroup whose add returns n_tasks - 1 is last and acquires (one
        // lane: invalidate, wait) before a barrier, after which its waves load the chain roots.
        __shared__ int last_arrival;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            const int prev = __hip_atomic_fetch_add(a.ticket + wt, 1, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
            last_arrival = prev == a.n_tasks - 1;
            if (last_arrival) {
                __hip_atomic_store(a.ticket + wt, 0, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
        if (!last_arrival) return;
        // the top task, started like a whole traversal: its first P, then NS stores into the
        // root slot standing in for a previous op's (the root's own stores come later, in order)
        const cptr<int> tk = as_const(a.tasks) + 4 * a.n_tasks;
        const int top_lo = tk[0], top_ch = tk[2];
        opp = ops + 8 * (size_t)top_lo;
        pa_t = pa_w + (size_t)(2 * top_lo) * pa_side;
        pa_load(PA, pa_t, poff, poff4);
        pa_load(PB, pa_t + pa_side, poff, poff4);
        if constexpr (MODE == 1) aa_store(root_cw, root_sw, voff, soff, cur, 0.0, true);
        run_chunks(top_ch, a.n_chunks, a.n_ops);
    } else {
        run_chunks(ch_lo, ch_hi, a.n_ops);
    }
    op(a.n_ops, std::true_type{}, std::false_type{});  // in the last chunk, still staged
    if (timed && lane == 0)
        for (int i = 1; i < 6; ++i) atomicAdd(a.timing + i, tsum[i]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // lnl_node (numba_likelihood_engine.py:82-87) of the root combine, then the category's
    // log weight; k_site_lse combines the categories
    const cptr<double> pi = as_const(a.pi);
    double f = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) f = fma(cur[r], pi[g + 4 * r], f);
    f = fma(cur[4], pi[16 + g], f);
    f += __shfl_xor(f, 16);
    f += __shfl_xor(f, 32);
    const double sw = ((f > 0.0) ? log(f) + cur_s : -INFINITY) + as_const(a.logw)[cat];
    double *cl = a.cat_lnl + (size_t)cat * n_tiles * kTile + (size_t)tile * kTile + w * kAaSites;
    if (!a.lse_ticket) {  // k_site_lse combines the categories
        if (g == 0) cl[s16] = sw;
        return;
    }
    // The last of the tile's C workgroups combines its categories (the hand-off of the chain
    // tasks: values written through, every wave waits, one relaxed agent add, one acquire in
    // the last arriver), so no k_site_lse launch follows the traversal
    if (g == 0) asm_st2<0, 2>(soff, cl, sw);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int last_cat;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int prev = __hip_atomic_fetch_add(a.lse_ticket + tile, 1, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
        last_cat = prev == C - 1;
        if (last_cat) {
            __hip_atomic_store(a.lse_ticket + tile, 0, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!last_cat) return;
    // per-pattern logsumexp over categories (tree_model.py:216) as k_site_lse takes it, and
    // the tile's pattern-weighted sum (k_reduce adds the tiles in order)
    __shared__ double red[kWaves];
    double contrib = 0.0;
    const int64_t st = (int64_t)tile * kTile + threadIdx.x;
    if (threadIdx.x < kTile && st < a.S) {
        const double l = lse_strided(a.cat_lnl + st, C, (int64_t)n_tiles * kTile);
        a.site_lnl[st] = l;
        contrib = a.pattern_w[st] * l;
    }
    const double t = block_sum_256(contrib, red);
    if (!a.lnl_out) {  // k_reduce adds the tiles
        if (threadIdx.x == 0) a.block_sum[tile] = t;
        return;
    }
    // r04: and the last of the n_tiles tile sums adds them all, in k_reduce's order (bitwise
    // its result), so no k_reduce launch follows: the same hand-off one level up -- the tile
    // sum written through, a wait, one relaxed add to the grid ticket (lse_ticket[n_tiles]),
    // one acquire in the last arriver
    __shared__ int last_tile;
    if (threadIdx.x == 0) {
        __hip_atomic_store(a.block_sum + tile, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int *gt = a.lse_ticket + n_tiles;
        const int prev = __hip_atomic_fetch_add(gt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_tile = prev == n_tiles - 1;
        if (last_tile) {
            __hip_atomic_store(gt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!last_tile) return;
    double v = 0.0;  // k_reduce's loop and block sum
    for (int i = threadIdx.x; i < n_tiles; i += kBlock) v += a.block_sum[i];
    const double total = block_sum_256(v, red);
    if (threadIdx.x == 0) *a.lnl_out = total;
}

// P [side][cat][K][K] -> A operands [side][cat][5][64][2] of k_prune_mfma: per k-step q the
// 16x16x4 operand (rows 0..15) and the 4x4x4_4b operand (rows 16..19)
__global__ void __launch_bounds__(64) k_pa(int C, const double *__restrict__ P,
                                           double *__restrict__ Pa) {
    constexpr int K = 20;
    const int sd = blockIdx.x, c = blockIdx.y, l = threadIdx.x;
    const double *p = P + ((size_t)sd * C + c) * K * K;
    double *o = Pa + ((size_t)sd * C + c) * 5 * 128 + 2 * l;
    const int k = l >> 4;
    for (int q = 0; q < 5; ++q) {
        o[q * 128] = p[(l & 15) * K + 4 * q + k];            // 16x16x4: A[row][k]
        o[q * 128 + 1] = p[(16 + (l & 3)) * K + 4 * q + k];  // 4x4x4_4b: A_b[i][k]
    }
}

// K = 20 in one launch: k_prune_mfma's A operands (k_pa's layout), one workgroup per (side,
// category).  The eigen-system is staged in LDS with the exponentials (one global round trip),
// each entry is computed in the shared fma order above -- evecs[i][k] * ex[k] rounded once, then
// fma(., ivecs[k][j], acc) in k order, bitwise the P of every other builder -- into an LDS copy
// of P, from which the 640 A-operand doubles are written as one contiguous run.  The plain P is
// not written: the traversal reads only the A operands, and pu_get_pmatrices rebuilds P from
// them (r05: 8.8 -> 6.7-7.0 us back to back in scripts/probes/pmat_aa_probe.hip, where a grid
// of this shape with an empty body costs 2.8-3.4 us; one workgroup per side and four categories
// was slower, 11.2 us: too few workgroups to issue the stores)
__global__ void __launch_bounds__(kBlock) k_pmatrix_aa(PmatArgs a) {
    constexpr int K = 20, KK = K * K, NA = 5 * 128;
    static_assert(KK > kBlock && KK <= 2 * kBlock, "two eigen-system entries per thread");
    __shared__ double evx[KK], iv[KK], ex[K], pm[KK];
    const int sd = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
    const bool hi = tid + kBlock < KK;
    // every global read is issued before the first barrier (one round trip)
    const double e0 = a.evecs[tid], e1 = hi ? a.evecs[tid + kBlock] : 0.0;
    iv[tid] = a.ivecs[tid];
    if (hi) iv[tid + kBlock] = a.ivecs[tid + kBlock];
    if (tid < K) ex[tid] = exp(a.evals[tid] * (a.brlens[sd] * a.rates[c]));
    __syncthreads();
    evx[tid] = e0 * ex[tid % K];
    if (hi) evx[tid + kBlock] = e1 * ex[(tid + kBlock) % K];
    __syncthreads();
    // thread (row group r, column j): rows r and r + 12 share each ivecs[k][j] read
    if (tid < 12 * K) {
        const int r = tid / K, j = tid - r * K;
        const bool two = r + 12 < K;
        double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double b = iv[k * K + j];
            acc0 = fma(evx[r * K + k], b, acc0);
            if (two) acc1 = fma(evx[(r + 12) * K + k], b, acc1);
        }
        pm[r * K + j] = acc0;
        if (two) pm[(r + 12) * K + j] = acc1;
    }
    __syncthreads();
    // [k-step q][lane][2]: .x = P[lane & 15][4q + (lane >> 4)] (the 16x16x4 rows),
    // .y = P[16 + (lane & 3)][4q + (lane >> 4)] (the 4x4x4_4b rows)
    double *pa = a.Pa + ((size_t)sd * a.C + c) * NA;
    for (int o = tid; o < NA; o += kBlock) {
        const int q = o >> 7, lane = (o & 127) >> 1, h = o & 1;
        const int col = 4 * q + (lane >> 4), row = h ? 16 + (lane & 3) : (lane & 15);
        pa[o] = pm[row * K + col];
    }
}

// protein tiled CLV (+ scaler) -> [S][C][K] (+ [S][C])
__global__ void __launch_bounds__(kBlock)
    k_untile_aa(int C, int64_t S, int64_t pitch, const double *__restrict__ clv,
                const double *__restrict__ scale, double *__restrict__ out,
                double *__restrict__ out_scale) {
    constexpr int K = 20;
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // (site, cat)
    if (e >= S * C) return;
    const int64_t s = e / C;
    const int c = (int)(e - s * C);
    const size_t row = layout_row(K, C, pitch, c, s / kTile);
    const int ls = (int)(s % kTile), w = ls / kAaSites, s16 = ls % kAaSites;
    const double *src = clv + row * K * kTile + (size_t)w * kAaRows * 64;
    for (int i = 0; i < K; ++i) {
        const int g = i < 16 ? (i & 3) : i - 16, r = i < 16 ? (i >> 2) : 4;
        out[e * K + i] = src[aa_row_off(r, g * 16 + s16)];
    }
    if (out_scale) out_scale[e] = scale[row * kTile + ls];
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
    k_untile(int K, int C, int64_t S, int64_t pitch, const double *__restrict__ clv,
             const double *__restrict__ scale, double *__restrict__ out,
             double *__restrict__ out_scale) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // (site, cat)
    if (e >= S * C) return;
    const int64_t s = e / C;
    const int c = (int)(e - s * C);
    const size_t row = layout_row(K, C, pitch, c, s / kTile);
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

// ---------------------------------------------------------------- several trees per launch
// (r05, SURVEY 8(e) G2: pu_batch_enqueue).  Tree t's arguments are read through the constant
// address space; each tree's arithmetic is its own launch's.
template <int K>
__global__ void __launch_bounds__(kBlock) k_pmatrix_lane_trees(const PmatArgs *__restrict__ trees) {
    const auto &a = *as_const(trees + blockIdx.y);
    pmatrix_lane<K>(a, (int)(blockIdx.x * kBlock + threadIdx.x));
}

// k_reduce of tree blockIdx.x
__global__ void __launch_bounds__(kBlock) k_reduce_trees(const ReduceItem *__restrict__ items) {
    __shared__ double red[kBlock / 64];
    const auto &r = *as_const(items + blockIdx.x);
    const double *in = r.in;
    const int n = (int)r.n;
    double v = 0.0;
    for (int i = threadIdx.x; i < n; i += kBlock) v += in[i];
    const double t = block_sum_256(v, red);
    if (threadIdx.x == 0) *r.out = t;
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
    if (variant & TV_CHAIN) {
        if (!a.tasks || a.n_tasks < 2 || !a.ticket || !(variant & TV_GENERIC))
            return (int)hipErrorInvalidValue;
        const dim3 g((unsigned)(grid * a.n_tasks));
        if constexpr (CODED) {
            if (variant & TV_PTIP) {  // a split lnL-only plan with tip products
                if (!a.PT || (variant & TV_SKIP_ZERO_SCALE)) return (int)hipErrorInvalidValue;
                hipLaunchKernelGGL((k_prune<K, CODED, TV_GENERIC | TV_CHAIN | TV_PTIP, W>), g,
                                   dim3(kBlock), lds, st, a);
                return (int)hipGetLastError();
            }
        }
        if (variant & TV_PTIP) return (int)hipErrorInvalidValue;
        if (variant & TV_SKIP_ZERO_SCALE)
            hipLaunchKernelGGL((k_prune<K, CODED, TV_GENERIC | TV_SKIP_ZERO_SCALE | TV_CHAIN, W>),
                               g, dim3(kBlock), lds, st, a);
        else
            hipLaunchKernelGGL((k_prune<K, CODED, TV_GENERIC | TV_CHAIN, W>), g, dim3(kBlock),
                               lds, st, a);
        return (int)hipGetLastError();
    }
    if (variant & TV_PTIP) {  // lnL-only coded plans (no skip-zero scalers, no split)
        if constexpr (CODED) {
            if (!a.PT || (variant & (TV_SKIP_ZERO_SCALE | TV_CHAIN)))
                return (int)hipErrorInvalidValue;
            if (variant & TV_GENERIC)
                hipLaunchKernelGGL((k_prune<K, CODED, TV_PTIP | TV_GENERIC, W>), dim3(grid),
                                   dim3(kBlock), lds, st, a);
            else
                hipLaunchKernelGGL((k_prune<K, CODED, TV_PTIP, W>), dim3(grid), dim3(kBlock),
                                   lds, st, a);
            return (int)hipGetLastError();
        } else {
            return (int)hipErrorInvalidValue;
        }
    }
    if (variant & TV_RSLOTS) {  // KEEP occupancy plans of the default build only
        if constexpr (W == 1) {
            if (variant == (TV_SKIP_ZERO_SCALE | TV_RSLOTS))
                hipLaunchKernelGGL((k_prune<K, CODED, TV_SKIP_ZERO_SCALE | TV_RSLOTS, 1>), dim3(grid), dim3(kBlock), lds, st, a);
            else if (variant == (TV_GENERIC | TV_SKIP_ZERO_SCALE | TV_RSLOTS))
                hipLaunchKernelGGL((k_prune<K, CODED, TV_GENERIC | TV_SKIP_ZERO_SCALE | TV_RSLOTS, 1>), dim3(grid), dim3(kBlock), lds, st, a);
            else
                return (int)hipErrorInvalidValue;
            return (int)hipGetLastError();
        }
        return (int)hipErrorInvalidValue;
    }
    switch (variant) {
        case 0:
            // K = 2 coded tips without tip products (lnL-only host-matrix models, PU_NO_PTIP):
            // the general variant, same arithmetic (test_kernel_builds_and_plans_bitwise_equal);
            // the plain one compiled with a dead 64-byte stack object (a private segment with
            // no scratch access; test_kernel_isa.py allows none)
            if constexpr (K == 2 && CODED)
                hipLaunchKernelGGL((k_prune<K, CODED, TV_GENERIC, W>), dim3(grid), dim3(kBlock), lds, st, a);
            else
                hipLaunchKernelGGL((k_prune<K, CODED, 0, W>), dim3(grid), dim3(kBlock), lds, st, a);
            break;
        case TV_SKIP_ZERO_SCALE: hipLaunchKernelGGL((k_prune<K, CODED, TV_SKIP_ZERO_SCALE, W>), dim3(grid), dim3(kBlock), lds, st, a); break;
        case TV_GENERIC: hipLaunchKernelGGL((k_prune<K, CODED, TV_GENERIC, W>), dim3(grid), dim3(kBlock), lds, st, a); break;
        case TV_GENERIC | TV_SKIP_ZERO_SCALE: hipLaunchKernelGGL((k_prune<K, CODED, TV_GENERIC | TV_SKIP_ZERO_SCALE, W>), dim3(grid), dim3(kBlock), lds, st, a); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

template <bool CODED>
int launch_mfma(hipStream_t st, int variant, const TraverseArgs &a) {
    const size_t lds = AaLds(20, a.n_codes, a.max_chunk_uses, CODED, a.n_lds).total;
    const dim3 grid((unsigned)(a.n_tiles * a.C)), block(kBlock);
    if (a.tasks) {  // split plans: KEEP (counted waits) or lnL only
        if ((variant & TV_GENERIC) || a.n_tasks < 2 || !a.ticket) return (int)hipErrorInvalidValue;
        if (variant & TV_KEEP)
            hipLaunchKernelGGL((k_prune_mfma<CODED, 1, true>), dim3(grid.x * a.n_tasks), block,
                               lds, st, a);
        else
            hipLaunchKernelGGL((k_prune_mfma<CODED, 0, true>), dim3(grid.x * a.n_tasks), block,
                               lds, st, a);
    } else if (variant & TV_GENERIC)
        hipLaunchKernelGGL((k_prune_mfma<CODED, 2>), grid, block, lds, st, a);
    else if (variant & TV_KEEP)
        hipLaunchKernelGGL((k_prune_mfma<CODED, 1>), grid, block, lds, st, a);
    else
        hipLaunchKernelGGL((k_prune_mfma<CODED, 0>), grid, block, lds, st, a);
    return (int)hipGetLastError();
}

template <int K, bool CODED>
int launch_prune_k(hipStream_t st, int variant, const TraverseArgs &a, int grid) {
    const size_t lds =
        TravLds(K, a.n_codes, a.max_chunk_uses, CODED, a.n_lds, a.C).total + a.lds_pad;
    // The default build's 106 SGPRs allow 6 waves per SIMD.  The 7-wave build (SGPRs trimmed,
    // spilled to VGPR lanes) serves the two variants that run one dispatch round of 7
    // workgroups per CU: DNA KEEP occupancy plans whose grid needs 5-6 per CU (keep_per_cu)
    // and lnL-only tip-product plans (pick_waves).  r05: the other 7-wave variants and the
    // 8-wave builds spilled into scratch and are gone (test_kernel_isa.py allows no scratch)
    if (a.waves == 7) {
        if (variant == TV_SKIP_ZERO_SCALE) {
            hipLaunchKernelGGL((k_prune<K, CODED, TV_SKIP_ZERO_SCALE, 7>), dim3(grid),
                               dim3(kBlock), lds, st, a);
            return (int)hipGetLastError();
        }
        if constexpr (CODED) {
            if (variant == TV_PTIP && a.PT) {
                hipLaunchKernelGGL((k_prune<K, CODED, TV_PTIP, 7>), dim3(grid), dim3(kBlock),
                                   lds, st, a);
                return (int)hipGetLastError();
            }
        }
    }
    return launch_prune_w<K, CODED, 1>(st, variant, a, grid, lds);
}

// several trees: the lnL-only tip-product variants (the plans pu_batch accepts)
template <int K>
int launch_prune_trees_k(hipStream_t st, int variant, int waves, const TraverseArgs *trees,
                         int n_trees, int blocks, size_t lds, int group) {
    const dim3 grid((unsigned)(n_trees * blocks)), block(kBlock);
    if (variant == TV_PTIP && waves == 7)
        hipLaunchKernelGGL((k_prune_trees<K, true, TV_PTIP, 7>), grid, block, lds, st, trees, blocks,
                           n_trees, group);
    else if (variant == TV_PTIP)
        hipLaunchKernelGGL((k_prune_trees<K, true, TV_PTIP, 1>), grid, block, lds, st, trees, blocks,
                           n_trees, group);
    else if (variant == (TV_PTIP | TV_GENERIC) && waves == 7)
        hipLaunchKernelGGL((k_prune_trees<K, true, TV_PTIP | TV_GENERIC, 7>), grid, block, lds, st,
                           trees, blocks, n_trees, group);
    else if (variant == (TV_PTIP | TV_GENERIC))
        hipLaunchKernelGGL((k_prune_trees<K, true, TV_PTIP | TV_GENERIC, 1>), grid, block, lds, st,
                           trees, blocks, n_trees, group);
    else
        return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
}

}  // namespace

bool traverse_trees_supported(int K, bool coded, int variant) {
    return (K == 2 || K == 4) && coded &&
           (variant == TV_PTIP || variant == (TV_PTIP | TV_GENERIC));
}

int launch_traverse_trees(hipStream_t st, int K, int variant, int waves,
                          const TraverseArgs *trees, int n_trees, int blocks, size_t lds,
                          int group) {
    if (n_trees <= 0 || blocks <= 0) return 0;
    if (K == 2)
        return launch_prune_trees_k<2>(st, variant, waves, trees, n_trees, blocks, lds, group);
    if (K == 4)
        return launch_prune_trees_k<4>(st, variant, waves, trees, n_trees, blocks, lds, group);
    return (int)hipErrorInvalidValue;
}

int launch_pmatrix_trees(hipStream_t st, int K, const PmatArgs *trees, int n_trees,
                         int max_rows) {
    // 256-lane workgroups: 125 trees of 64-lane ones were 6.2k workgroups (10.1 us, r06)
    const unsigned grid = (unsigned)((max_rows + kBlock - 1) / kBlock);
    if (n_trees <= 0 || grid == 0) return 0;
    if (K == 2)
        hipLaunchKernelGGL(k_pmatrix_lane_trees<2>, dim3(grid, n_trees), dim3(kBlock), 0, st, trees);
    else if (K == 4)
        hipLaunchKernelGGL(k_pmatrix_lane_trees<4>, dim3(grid, n_trees), dim3(kBlock), 0, st, trees);
    else
        return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
}

int launch_reduce_trees(hipStream_t st, const ReduceItem *items, int n_trees) {
    if (n_trees <= 0) return 0;
    hipLaunchKernelGGL(k_reduce_trees, dim3(n_trees), dim3(kBlock), 0, st, items);
    return (int)hipGetLastError();
}

bool traverse_supported(int K) { return K == 2 || K == 4 || K == 20; }

size_t traverse_lds_bytes(int K, int C, int n_codes, int max_chunk_uses, bool coded, int n_lds) {
    if (K == 20) return AaLds(20, n_codes, max_chunk_uses, coded, n_lds).total;
    return TravLds(K, n_codes, max_chunk_uses, coded, n_lds, C).total;
}

int launch_traverse(hipStream_t st, int K, bool coded, int variant, const TraverseArgs &a,
                    int grid) {
    int rc;
    const int v = variant & ~TV_KEEP;  // (TV_CHAIN stays: launch_prune_w)
    switch (K) {
        case 2: rc = coded ? launch_prune_k<2, true>(st, v, a, grid) : launch_prune_k<2, false>(st, v, a, grid); break;
        case 4: rc = coded ? launch_prune_k<4, true>(st, v, a, grid) : launch_prune_k<4, false>(st, v, a, grid); break;
        case 20:
            // P into the MFMA A-operand layout (unless k_pmatrix_aa wrote it), then the traversal
            if (!a.pa_ready) {
                hipLaunchKernelGGL(k_pa, dim3(2 * (a.n_ops + 1), a.C), dim3(64), 0, st, a.C, a.P,
                                   a.Pa);
                if ((rc = (int)hipGetLastError())) return rc;
            }
            rc = coded ? launch_mfma<true>(st, variant, a) : launch_mfma<false>(st, variant, a);
            break;
        default: return (int)hipErrorInvalidValue;
    }
    if (rc || !a.cat_lnl || a.lse_ticket) return rc;
    const int64_t nb = (a.S + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_site_lse, dim3((unsigned)nb), dim3(kBlock), 0, st, a.C, a.S,
                       (int64_t)a.n_tiles * kTile, a.cat_lnl, a.pattern_w, a.site_lnl,
                       a.block_sum);
    return (int)hipGetLastError();
}

bool traverse_per_category(int K, int C) { return K == 20 || 4 % C != 0; }

// K = 20: the last of a tile's C workgroups combines its categories in the traversal (r03;
// the k_site_lse launch it replaced and its PU_AA_SITE_LSE A/B switch are gone)
bool traverse_lse_in_kernel(int K) { return K == 20; }

int traverse_block_sums(int K, int C, int64_t S) {
    if (traverse_lse_in_kernel(K)) return (int)tile_count(S);  // one per tile
    return !traverse_per_category(K, C) ? (int)((tile_count(S) * C + kWaves - 1) / kWaves)
                                        : (int)((S + kBlock - 1) / kBlock);
}

int launch_untile(hipStream_t st, int K, int C, int64_t S, int64_t pitch, const double *clv,
                  const double *scale, double *out, double *out_scale) {
    const int64_t n = S * C;
    if (n == 0) return 0;
    const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
    if (K == 20)
        hipLaunchKernelGGL(k_untile_aa, grid, dim3(kBlock), 0, st, C, S, pitch, clv, scale,
                           out, out_scale);
    else
        hipLaunchKernelGGL(k_untile, grid, dim3(kBlock), 0, st, K, C, S, pitch, clv, scale,
                           out, out_scale);
    return (int)hipGetLastError();
}

// K = 20 writes the MFMA A operands in the same launch (k_pmatrix_aa).  (r04: the r01
// per-(side, category) block forms and their PU_PMAT_BLOCK switch are gone -- the block
// k_pmatrix<K> never wrote the tip products PT that an lnL-only coded DNA traversal reads.)
bool pmatrix_writes_pa(int K) { return K == 20; }

int launch_pmatrix(hipStream_t st, const PmatArgs &a) {
    const unsigned lane_grid = (unsigned)((a.n_sides * a.C * a.K + 63) / 64);
    if (lane_grid == 0) return 0;
    if (a.K == 2 || a.K == 4) {
        if (a.PT && (!a.table || a.n_codes < 1)) return (int)hipErrorInvalidValue;
        if (a.K == 2) hipLaunchKernelGGL(k_pmatrix_lane<2>, dim3(lane_grid), dim3(64), 0, st, a);
        else hipLaunchKernelGGL(k_pmatrix_lane<4>, dim3(lane_grid), dim3(64), 0, st, a);
        return (int)hipGetLastError();
    }
    // K = 20: P and the A operands; no tip products (PT is a DNA lnL-only feature)
    if (a.K != 20 || !a.Pa || a.PT) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_pmatrix_aa, dim3(a.n_sides, a.C), dim3(kBlock), 0, st, a);
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
