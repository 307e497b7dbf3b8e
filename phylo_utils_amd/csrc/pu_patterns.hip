// pu_patterns.hip -- site-pattern compression on the GPU (the data format on
// the way into the pruning path): the reference's
//     np.unique(alignment, return_inverse=True, return_counts=True, axis=1)
// (phylo_utils/alignment/alignment.py:40-57) over tip codes instead of [ntaxa][S][K] float
// partials.  A column is the byte string codes[0..n_taxa)[j]; np.unique orders the columns
// lexicographically, taxon 0 first, and numbers them in that order.  With codes whose order
// is the lexicographic order of their partial vectors (alignment.code_table guarantees it),
// the byte order of code columns is the order np.unique gives the float columns, so the
// unique columns, the inverse index and the counts are exactly the reference's.
//
//   k_pack_T    column j -> W = ceil(n_taxa * b / 64) 64-bit words, b bits per code, taxon 0
//               in the top bits of word 0: comparing words as unsigned integers, most
//               significant word first, is the lexicographic byte comparison; stored
//               column-major ([S][W]) so a random column is one contiguous read; the column's
//               dedup hash is computed in the same pass
//   dedup       a 64-bit hash of each column's words; one radix sort by hash; identical
//               columns are adjacent runs, verified word by word (a run whose members differ
//               is a hash collision: retried with another seed); G groups, one representative
//   refine      the G distinct representatives get ranks = their position in lexicographic
//               order, word by word (prefix refinement, as in suffix-array construction):
//               sort by word 0; a run of equal words is a group with rank = its first
//               position; for word w only the members of groups of size > 1 are re-sorted by
//               (rank, word w) -- two stable radix sorts (rocprim) -- and a sub-run's rank is
//               its group's rank + its offset in the group.  Distinct columns separate at
//               their first differing word, so the active set shrinks round by round.
//   k_final     pattern u = rank: its representative column and count; inverse[j] = rank of
//               column j's group
//   k_unpack    unique codes [n_taxa][U] from the packed words of each pattern's column
// (A plain LSD sort of all S columns by every word -- W radix sorts -- was the first form;
// it is 8x slower at 1000 taxa and lost stability somewhere in its 63 passes on
// near-duplicate columns, tests/test_gpu_patterns.py.)
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include <algorithm>
#include <mutex>
#include <vector>

#include "pu_ctx.h"

using namespace pu;

namespace {

constexpr int kPB = 256;

__global__ void __launch_bounds__(kPB) k_iota(int64_t S, uint32_t *__restrict__ perm) {
    const int64_t i = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (i < S) perm[i] = (uint32_t)i;
}

// unique codes: row t of pattern u at out[t * ld + u].  V = 4: a lane unpacks patterns
// 4i..4i+3 and writes one 4-byte word per taxon row (ld % 4 == 0), 256 bytes per wave and
// row instead of 64 single-byte stores
template <int V>
__global__ void __launch_bounds__(kPB) k_unpack(const uint64_t *__restrict__ wordsT, int n_taxa,
                                                int b, int T, int W,
                                                const uint32_t *__restrict__ srep, int64_t U,
                                                int64_t S, uint8_t *__restrict__ out, int64_t ld,
                                                uint32_t *__restrict__ err) {
    const int64_t u0 = ((int64_t)blockIdx.x * kPB + threadIdx.x) * V;
    if (u0 >= U) return;
    size_t col[V];
    bool okc = true;
#pragma unroll
    for (int c = 0; c < V; ++c) {
        const int64_t u = min(u0 + c, U - 1);  // (past U: a copy of the last, not stored)
        col[c] = srep[u];
        okc &= col[c] < (size_t)S;
    }
    if (!okc) {  // a pattern without a column (srep is preset to ~0)
        err[1] = 1u;
        return;
    }
    const uint64_t mask = (b == 64) ? ~0ull : ((1ull << b) - 1);
    for (int w = 0; w < W; ++w) {
        uint64_t v[V];
#pragma unroll
        for (int c = 0; c < V; ++c) v[c] = wordsT[col[c] * W + w];
        const int t0 = w * T, t1 = min(n_taxa, t0 + T);
        for (int t = t0; t < t1; ++t) {
            const int sh = 64 - (t - t0 + 1) * b;
            if constexpr (V == 4) {
                uint32_t x = 0;
#pragma unroll
                for (int c = 0; c < 4; ++c) x |= (uint32_t)((v[c] >> sh) & mask) << (8 * c);
                if (u0 + 4 <= U) {
                    *reinterpret_cast<uint32_t *>(out + (size_t)t * ld + u0) = x;
                } else {
                    for (int c = 0; c < 4 && u0 + c < U; ++c)
                        out[(size_t)t * ld + u0 + c] = (uint8_t)(x >> (8 * c));
                }
            } else {
                out[(size_t)t * ld + u0] = (uint8_t)((v[0] >> sh) & mask);
            }
        }
    }
}

// unique codes through LDS: a workgroup owns 128 consecutive patterns and walks their packed
// words in slices of kSliceW words: it gathers the slice of the 128 columns into LDS (8
// consecutive lanes read one column's 64 contiguous bytes), then writes the slice's rows, one
// 128-byte store per wave instruction (a lane = 2 adjacent patterns, one 2-byte store; byte
// stores when ld is odd).  Small LDS (8 KB) keeps many workgroups resident to hide the gather
// latency.  Measured (cfg4 alignment, r02): the per-lane form above 1.23 ms; all 63 words of
// 64 patterns in LDS with byte stores 0.77 ms; of 128 patterns with 2-byte stores (64 KB LDS,
// 2 workgroups per CU) 0.97 ms.
constexpr int kUnpackCols = 128, kSliceW = 8;
__global__ void __launch_bounds__(kPB) k_unpack_lds(const uint64_t *__restrict__ wordsT,
                                                    int n_taxa, int b, int T, int W,
                                                    const uint32_t *__restrict__ srep,
                                                    int64_t U, int64_t S,
                                                    uint8_t *__restrict__ out, int64_t ld,
                                                    uint32_t *__restrict__ err) {
    __shared__ uint64_t cols[kUnpackCols * (kSliceW + 1)];  // [column][slice word], padded
    __shared__ uint32_t colidx[kUnpackCols];
    const int64_t u0 = (int64_t)blockIdx.x * kUnpackCols;
    const int n = (int)min((int64_t)kUnpackCols, U - u0);
    if (threadIdx.x < kUnpackCols) {
        uint32_t col = 0;
        if ((int)threadIdx.x < n) {
            col = srep[u0 + threadIdx.x];
            if (col >= (uint64_t)S) {
                err[1] = 1u;  // a pattern without a column (srep is preset to ~0)
                col = 0;
            }
        }
        colidx[threadIdx.x] = col;
    }
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int p0 = 2 * l;  // this lane's patterns p0, p0 + 1
    const bool one = p0 < n, two = p0 + 1 < n, pair = two && (((uintptr_t)out | (uintptr_t)ld) & 1) == 0;  // u0 is even
    const uint64_t mask = (b == 64) ? ~0ull : ((1ull << b) - 1);
    uint8_t *o = out + u0 + p0;
    for (int w0 = 0; w0 < W; w0 += kSliceW) {
        const int nw = min(kSliceW, W - w0);
        __syncthreads();  // colidx ready / the previous slice's rows are written
        for (int i = threadIdx.x; i < kUnpackCols * kSliceW; i += kPB) {
            const int c = i / kSliceW, k = i - c * kSliceW;
            if (c < n && k < nw)
                cols[c * (kSliceW + 1) + k] = wordsT[(size_t)colidx[c] * W + w0 + k];
        }
        __syncthreads();
        if (!one) continue;
        for (int k = 0; k < nw; ++k) {
            const int w = w0 + k;
            const uint64_t v0 = cols[p0 * (kSliceW + 1) + k];
            const uint64_t v1 = two ? cols[(p0 + 1) * (kSliceW + 1) + k] : 0;
            const int t0 = w * T, t1 = min(n_taxa, t0 + T);
            for (int t = t0 + wv; t < t1; t += kPB / 64) {
                const int sh = 64 - (t - t0 + 1) * b;
                const uint32_t c0 = (uint32_t)((v0 >> sh) & mask);
                const uint32_t c1 = (uint32_t)((v1 >> sh) & mask);
                uint8_t *q = o + (size_t)t * ld;
                if (pair) {
                    *reinterpret_cast<uint16_t *>(q) = (uint16_t)(c0 | (c1 << 8));
                } else {
                    q[0] = (uint8_t)c0;
                    if (two) q[1] = (uint8_t)c1;
                }
            }
        }
    }
}

// ---- refine form ----
__device__ __forceinline__ uint64_t mix64(uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    return h;
}

// A column's dedup hash: x = mix64(x ^ word_w) + w over its words from the seed.  mix64 and
// "+ w" are bijections, so two columns that differ in exactly one word never collide; any
// collision is caught by k_dup and retried with another seed.

// the hash over the column-major words (another seed after a collision: rare)
__global__ void __launch_bounds__(kPB) k_hash_T(const uint64_t *__restrict__ wordsT, int W,
                                                int64_t S, uint64_t seed,
                                                uint64_t *__restrict__ h) {
    const int64_t j = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (j >= S) return;
    uint64_t x = seed;
    for (int w = 0; w < W; ++w) x = mix64(x ^ wordsT[(size_t)j * W + w]) + (uint64_t)w;
    h[j] = x;
}

// Pack, transpose and hash in one pass (r05; three kernels before: a word-major pack, an LDS
// transpose, a hash pass: 0.38 + 0.26 + 0.12 ms on the cfg4 alignment, now 0.59 ms): a
// workgroup packs kFB * V adjacent columns word by word, keeps each column's hash in registers
// and writes the column-major words ([S][W]) through an LDS tile of kFW words per column, so
// each column's run of kFW words is one 64-byte store segment.  The codes are read once and
// nothing word-major is written.  (Splitting the words over a second grid dimension, with the
// hash as a sum of per-word terms, was slower: 0.63 ms -- its 64-byte runs of a column are
// then written by different workgroups at different times.)
constexpr int kFB = 128, kFW = 8;
template <int V>
__global__ void __launch_bounds__(kFB) k_pack_T(const uint8_t *__restrict__ codes, int n_taxa,
                                                int64_t S, int b, int T, int W, int n_codes,
                                                uint64_t h0, uint64_t *__restrict__ wordsT,
                                                uint64_t *__restrict__ hash,
                                                uint32_t *__restrict__ bad) {
    constexpr int NC = kFB * V;                       // columns per workgroup
    __shared__ uint64_t tile[NC * (kFW + 1)];         // [column][kFW + 1]: odd row pitch
    const int64_t jb = (int64_t)blockIdx.x * NC;      // first column of the workgroup
    const int64_t j = jb + (int64_t)threadIdx.x * V;  // this thread's first column
    const bool live = j < S;                          // (S % V == 0 when V > 1)
    const int ncol = (int)min((int64_t)NC, S - jb);
    uint64_t hx[V];
#pragma unroll
    for (int c = 0; c < V; ++c) hx[c] = h0;
    bool ok = true;
    for (int w0 = 0; w0 < W; w0 += kFW) {
        const int nw = min(kFW, W - w0);
        if (live) {
            for (int wi = 0; wi < nw; ++wi) {
                const int w = w0 + wi, t0 = w * T, t1 = min(n_taxa, t0 + T);
                uint64_t v[V];
#pragma unroll
                for (int c = 0; c < V; ++c) v[c] = 0;
#pragma unroll 8
                for (int t = t0; t < t1; ++t) {
                    uint32_t x;
                    if constexpr (V == 4)
                        x = *reinterpret_cast<const uint32_t *>(codes + (size_t)t * S + j);
                    else
                        x = codes[(size_t)t * S + j];
#pragma unroll
                    for (int c = 0; c < V; ++c) {
                        const uint32_t code = (x >> (8 * c)) & 0xffu;
                        ok &= code < (uint32_t)n_codes;
                        v[c] = (v[c] << b) | code;
                    }
                }
                const int used = (t1 - t0) * b;
#pragma unroll
                for (int c = 0; c < V; ++c) {
                    if (used < 64) v[c] <<= (64 - used);
                    hx[c] = mix64(hx[c] ^ v[c]) + (uint64_t)w;
                    tile[(threadIdx.x * V + c) * (kFW + 1) + wi] = v[c];
                }
            }
        }
        __syncthreads();
        // the tile's columns, nw words each, to wordsT: consecutive threads walk one column's
        // run, then the next column's
        for (int e = threadIdx.x; e < ncol * nw; e += kFB) {
            const int c = e / nw, wi = e - c * nw;
            wordsT[(size_t)(jb + c) * W + w0 + wi] = tile[c * (kFW + 1) + wi];
        }
        __syncthreads();
    }
    if (!ok) *bad = 1u;  // a code outside [0, n_codes): reported, not packed silently
    if (live) {
#pragma unroll
        for (int c = 0; c < V; ++c) hash[j + c] = hx[c];
    }
}

// start of a run of equal hashes; inside a run, the column must equal its predecessor
__global__ void __launch_bounds__(kPB) k_dup(const uint64_t *__restrict__ words, int W,
                                             int64_t S, const uint64_t *__restrict__ hs,
                                             const uint32_t *__restrict__ perm,
                                             uint32_t *__restrict__ start,
                                             uint32_t *__restrict__ collision) {
    const int64_t p = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (p >= S) return;
    const int64_t q = p > 0 ? p - 1 : 0;
    const bool st = (p == 0) | (hs[p] != hs[q]);
    start[p] = st;
    if (!st) {
        const size_t a = perm[p], b = perm[q];
        uint64_t diff = 0;
        for (int w = 0; w < W; ++w) diff |= words[a * W + w] ^ words[b * W + w];
        if (diff) *collision = 1u;
    }
}

__global__ void __launch_bounds__(kPB) k_group(const uint32_t *__restrict__ perm,
                                               const uint32_t *__restrict__ start,
                                               const uint32_t *__restrict__ gid, int64_t S,
                                               uint32_t *__restrict__ colgrp,
                                               uint32_t *__restrict__ rep,
                                               uint32_t *__restrict__ gfirst) {
    const int64_t p = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (p >= S) return;
    const uint32_t g = gid[p] - 1;
    colgrp[perm[p]] = g;
    if (start[p]) {
        rep[g] = perm[p];
        gfirst[g] = (uint32_t)p;
    }
}

// key[g] = word 0 of the representative of group g (column-major words)
__global__ void __launch_bounds__(kPB) k_repkey0(const uint64_t *__restrict__ wordsT, int W,
                                                 const uint32_t *__restrict__ rep, int64_t n,
                                                 uint64_t *__restrict__ key) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a < n) key[a] = wordsT[(size_t)rep[a] * W];
}

__global__ void __launch_bounds__(kPB) k_gather_u32(const uint32_t *__restrict__ src,
                                                    const uint32_t *__restrict__ idx, int64_t n,
                                                    uint32_t *__restrict__ out) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a < n) out[a] = src[idx[a]];
}

// Position p of a group (rank r; R = false: a single group) starts a run of its sorted key.
// Branch-free on purpose: with short-circuit loads (`p == 0 || r[p] != r[p - 1]`) the ROCm
// 7.2 compiler emitted `v_mov v, 0` for every lane of the p != 0 side of the select
// (k_gcand wrote 0 where it had to write p; caught by tests/test_gpu_patterns.py,
// near-duplicate columns), so every load is unconditional and the choices are selects.
template <bool R>
__device__ __forceinline__ bool run_start(const uint32_t *r, const uint64_t *k, int64_t p) {
    const int64_t q = p > 0 ? p - 1 : 0;
    bool s = (p == 0) | (k[p] != k[q]);
    if constexpr (R) s = s | (r[p] != r[q]);
    return s;
}

// first pass of a refinement round: gcand = position of the group start (max-scanned next)
template <bool R>
__global__ void __launch_bounds__(kPB) k_gcand(const uint32_t *__restrict__ r, int64_t n,
                                               uint32_t *__restrict__ gcand) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    bool st = a == 0;
    if constexpr (R) st = st | (r[a] != r[a > 0 ? a - 1 : 0]);
    gcand[a] = st ? (uint32_t)a : 0u;
}

// second pass: a run start's new rank = its group's rank + offset in the group
template <bool R>
__global__ void __launch_bounds__(kPB) k_rcand(const uint32_t *__restrict__ r,
                                               const uint64_t *__restrict__ k,
                                               const uint32_t *__restrict__ gp, int64_t n,
                                               uint32_t *__restrict__ rcand) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    uint32_t base = 0;
    if constexpr (R) base = r[a];
    const uint32_t v = base + ((uint32_t)a - gp[a]);
    rcand[a] = run_start<R>(r, k, a) ? v : 0u;
}

// new ranks; an element stays active while its run has more than one member
// ws: the next round's known-equal word prefix of the element's (sub)group: dg[a] + 1 (dg =
// nullptr: word 0 was the split word)
template <bool R>
__global__ void __launch_bounds__(kPB) k_assign(const uint32_t *__restrict__ r,
                                                const uint64_t *__restrict__ k,
                                                const uint32_t *__restrict__ nr,
                                                const uint32_t *__restrict__ elem, int64_t n,
                                                const uint32_t *__restrict__ dg,
                                                uint32_t *__restrict__ rank,
                                                uint32_t *__restrict__ tied,
                                                uint32_t *__restrict__ ws) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    rank[elem[a]] = nr[a];
    uint32_t next_ws = 1;
    if constexpr (R) next_ws = dg[a] + 1;
    ws[elem[a]] = next_ws;
    const bool next = (a + 1 == n) | run_start<R>(r, k, a + 1 < n ? a + 1 : a);
    tied[a] = !(run_start<R>(r, k, a) & next);
}

// Word skipping: the first word (from the group's known-equal prefix ws) at which element a
// differs from its group's first element; the group's minimum (atomicMin into dmin[group
// start]) is the word that splits it.  (The first form scanned every word with branch-free
// selects, kept as PU_FD_BACKWARD; the early exit took the 5 calls per cfg4 compression from
// 269 to 225 us, r02.)
__global__ void __launch_bounds__(kPB) k_fd(const uint64_t *__restrict__ words, int W, int64_t S,
                                            const uint32_t *__restrict__ rep,
                                            const uint32_t *__restrict__ A,
                                            const uint32_t *__restrict__ gp,
                                            const uint32_t *__restrict__ ws, int64_t n,
                                            uint32_t *__restrict__ dmin) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    const size_t x = rep[A[a]], y = rep[A[gp[a]]];
    const int w0 = (int)ws[A[a]];
    uint32_t fd = (uint32_t)W;
#ifdef PU_FD_BACKWARD
    for (int w = W - 1; w >= w0; --w) {
        const bool d = words[x * W + w] != words[y * W + w];
        fd = d ? (uint32_t)w : fd;
    }
#else
    // forward from the known-equal prefix, leaving at the first difference (most members of
    // a group differ from its first element early; near-duplicates scan further)
    for (int w = w0; w < W; ++w)
        if (words[x * W + w] != words[y * W + w]) {
            fd = (uint32_t)w;
            break;
        }
#endif
    atomicMin(dmin + gp[a], fd);
}

// the group's split word and the element's key in it
__global__ void __launch_bounds__(kPB) k_dkey(const uint64_t *__restrict__ words, int W,
                                              int64_t S, const uint32_t *__restrict__ rep,
                                              const uint32_t *__restrict__ A,
                                              const uint32_t *__restrict__ gp,
                                              const uint32_t *__restrict__ dmin, int64_t n,
                                              uint32_t *__restrict__ dge,
                                              uint64_t *__restrict__ key) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    const uint32_t d = min(dmin[gp[a]], (uint32_t)(W - 1));  // (< W: a group is not all equal)
    dge[a] = d;
    key[a] = words[(size_t)rep[A[a]] * W + d];
}

__global__ void __launch_bounds__(kPB) k_fill(uint32_t v, int64_t n, uint32_t *__restrict__ out) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a < n) out[a] = v;
}

// after the two sorts: element, key and split word in (rank, key) order
__global__ void __launch_bounds__(kPB) k_gather3(const uint32_t *__restrict__ p2,
                                                 const uint32_t *__restrict__ A,
                                                 const uint64_t *__restrict__ key,
                                                 const uint32_t *__restrict__ dge, int64_t n,
                                                 uint32_t *__restrict__ elem,
                                                 uint64_t *__restrict__ keys,
                                                 uint32_t *__restrict__ dg) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    const uint32_t p = p2[a];
    elem[a] = A[p];
    keys[a] = key[p];
    dg[a] = dge[p];
}

__global__ void __launch_bounds__(kPB) k_final(const uint32_t *__restrict__ rank,
                                               const uint32_t *__restrict__ rep,
                                               const uint32_t *__restrict__ gfirst, int64_t G,
                                               int64_t S, uint32_t *__restrict__ srep,
                                               int64_t *__restrict__ counts,
                                               uint32_t *__restrict__ err) {
    const int64_t g = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (g >= G) return;
    const uint32_t r = rank[g];
    if (r >= (uint32_t)G) {  // (ranks are a permutation of [0, G): never taken)
        err[0] = 1u;
        return;
    }
    srep[r] = rep[g];
    counts[r] = (int64_t)(g + 1 < G ? gfirst[g + 1] : (uint32_t)S) - gfirst[g];
}

__global__ void __launch_bounds__(kPB) k_inverse(const uint32_t *__restrict__ rank,
                                                 const uint32_t *__restrict__ colgrp, int64_t S,
                                                 int64_t *__restrict__ inverse) {
    const int64_t j = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (j < S) inverse[j] = rank[colgrp[j]];
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + kPB - 1) / kPB); }

struct PatWs {
    std::mutex mu;
    void *buf = nullptr;
    size_t cap = 0;
};
PatWs g_pat[64];

// Workspace of one compression (S columns, W words per column).
struct Ws {
    uint64_t *wordsT, *key_a, *key_b, *key_c;  // wordsT [S][W] (column-major)
    uint32_t *v[21];   // S-sized u32 scratch arrays
    uint32_t *small;   // [0] bad code, [1] hash collision, [2] selected count
    void *sort_buf, *scan_buf, *sel_buf;
    size_t sort_tmp, scan_tmp, sel_tmp;
    int rounds = 0;    // refinement rounds of the last compression
};

inline unsigned rank_bits(int64_t n) {  // key bits for ranks < n, rounded up to bytes
    unsigned b = 8;
    while (b < 32 && ((int64_t)1 << b) < n) b += 8;
    return b;
}

// dedup + refine (header comment); *collision set when the hash dedup is not exact (the
// caller retries with another seed); returns U
int refine(hipStream_t st, Ws &w, int n_taxa, int64_t S, int b, int T, int W, uint64_t seed,
           bool hashed, uint32_t *srep, int64_t *d_counts, int64_t *d_inverse, int64_t *U_out,
           bool *collision) {
    uint32_t *perm_a = w.v[0], *perm_b = w.v[1], *start = w.v[2], *gid = w.v[3],
             *colgrp = w.v[4], *rep = w.v[5], *gfirst = w.v[6], *rank = w.v[7],
             *act = w.v[8], *e1 = w.v[9], *r1 = w.v[10], *r2 = w.v[11], *e2 = w.v[12],
             *tmp = w.v[13], *dmin = w.v[14], *dge = w.v[15], *p1 = w.v[16], *r1p = w.v[17],
             *p2 = w.v[18], *dg2 = w.v[19], *wsw = w.v[20];
    auto sort64 = [&](const uint64_t *kin, uint64_t *kout, const uint32_t *vin, uint32_t *vout,
                      int64_t n, int word) -> hipError_t {
        const int used = std::min(n_taxa - word * T, T) * b;
        const unsigned begin = word < 0 ? 0u : (unsigned)((64 - used) / 8 * 8);
        size_t need = 0;  // (the temporary storage was sized for S keys over all 64 bits)
        hipError_t e = rocprim::radix_sort_pairs(nullptr, need, kin, kout, vin, vout, (size_t)n,
                                                 begin, 64u, st);
        if (e != hipSuccess) return e;
        if (need > w.sort_tmp) return hipErrorInvalidValue;
        size_t tb = w.sort_tmp;
        return rocprim::radix_sort_pairs(w.sort_buf, tb, kin, kout, vin, vout, (size_t)n, begin,
                                         64u, st);
    };
    auto max_scan = [&](const uint32_t *in, uint32_t *out, int64_t n) -> hipError_t {
        size_t need = 0;
        hipError_t e = rocprim::inclusive_scan(nullptr, need, in, out, (size_t)n,
                                               rocprim::maximum<uint32_t>(), st);
        if (e != hipSuccess) return e;
        if (need > w.scan_tmp) return hipErrorInvalidValue;
        size_t sb = w.scan_tmp;
        return rocprim::inclusive_scan(w.scan_buf, sb, in, out, (size_t)n,
                                       rocprim::maximum<uint32_t>(), st);
    };
    // ---- dedup by hash
    HIPCHK(nullptr, hipMemsetAsync(w.small + 1, 0, 4, st));
    if (!hashed)  // k_pack_T hashed with the first seed
        hipLaunchKernelGGL(k_hash_T, dim3(blocks(S)), dim3(kPB), 0, st, w.wordsT, W, S, seed,
                           w.key_a);
    hipLaunchKernelGGL(k_iota, dim3(blocks(S)), dim3(kPB), 0, st, S, perm_a);
    HIPCHK(nullptr, hipGetLastError());
    HIPCHK(nullptr, sort64(w.key_a, w.key_b, perm_a, perm_b, S, -1));
    hipLaunchKernelGGL(k_dup, dim3(blocks(S)), dim3(kPB), 0, st, w.wordsT, W, S, w.key_b, perm_b,
                       start, w.small + 1);
    HIPCHK(nullptr, hipGetLastError());
    {
        size_t sb = w.scan_tmp;
        HIPCHK(nullptr, rocprim::inclusive_scan(w.scan_buf, sb, start, gid, (size_t)S,
                                                rocprim::plus<uint32_t>(), st));
    }
    hipLaunchKernelGGL(k_group, dim3(blocks(S)), dim3(kPB), 0, st, perm_b, start, gid, S, colgrp,
                       rep, gfirst);
    HIPCHK(nullptr, hipGetLastError());
    uint32_t hb[2] = {0, 0};  // G, collision
    HIPCHK(nullptr, hipMemcpyAsync(hb, gid + (S - 1), 4, hipMemcpyDeviceToHost, st));
    HIPCHK(nullptr, hipMemcpyAsync(hb + 1, w.small + 1, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(nullptr, hipStreamSynchronize(st));
    if (hb[1]) return *collision = true, PU_OK;
    const int64_t G = hb[0];
    const unsigned rbits = rank_bits(G);
    // ---- refinement: word 0 for every group; then each tied group by the first word in
    // which its members differ (word skipping), until every group is a single column
    int64_t n = G;
    const uint32_t *elem_in = nullptr;  // active groups (nullptr: all, as 0..G-1)
    int rounds = 0;
    for (; rounds <= W && n > 0; ++rounds) {
        const uint32_t *r_sorted = nullptr;  // ranks in the sorted order (nullptr: word 0)
        uint32_t *elem;                      // groups in (rank, key) order
        const uint32_t *dg = nullptr;        // split word per element, in that order
        if (rounds == 0) {
            hipLaunchKernelGGL(k_iota, dim3(blocks(G)), dim3(kPB), 0, st, G, e1);
            hipLaunchKernelGGL(k_repkey0, dim3(blocks(G)), dim3(kPB), 0, st, w.wordsT, W, rep, G,
                               w.key_a);
            HIPCHK(nullptr, hipGetLastError());
            HIPCHK(nullptr, sort64(w.key_a, w.key_c, e1, e2, G, 0));
            elem = e2;
        } else {
            const uint32_t *A = elem_in;
            // group start of every active element, then its group's split word and key
            hipLaunchKernelGGL(k_gather_u32, dim3(blocks(n)), dim3(kPB), 0, st, rank, A, n, r1);
            hipLaunchKernelGGL(k_gcand<true>, dim3(blocks(n)), dim3(kPB), 0, st, r1, n, tmp);
            HIPCHK(nullptr, hipGetLastError());
            HIPCHK(nullptr, max_scan(tmp, perm_a, n));
            hipLaunchKernelGGL(k_fill, dim3(blocks(n)), dim3(kPB), 0, st, (uint32_t)W, n, dmin);
            hipLaunchKernelGGL(k_fd, dim3(blocks(n)), dim3(kPB), 0, st, w.wordsT, W, S, rep, A,
                               perm_a, wsw, n, dmin);
            hipLaunchKernelGGL(k_dkey, dim3(blocks(n)), dim3(kPB), 0, st, w.wordsT, W, S, rep, A,
                               perm_a, dmin, n, dge, w.key_a);
            hipLaunchKernelGGL(k_iota, dim3(blocks(n)), dim3(kPB), 0, st, n, e1);
            HIPCHK(nullptr, hipGetLastError());
            // stable by key, then stable by rank: (rank, key) order; p2 = source positions
            HIPCHK(nullptr, sort64(w.key_a, w.key_b, e1, p1, n, -1));
            hipLaunchKernelGGL(k_gather_u32, dim3(blocks(n)), dim3(kPB), 0, st, r1, p1, n, r1p);
            HIPCHK(nullptr, hipGetLastError());
            size_t need = 0;
            HIPCHK(nullptr, rocprim::radix_sort_pairs(nullptr, need, r1p, r2, p1, p2, (size_t)n,
                                                      0u, rbits, st));
            if (need > w.sort_tmp)
                return set_err(nullptr, PU_E_STATE, "compress_patterns: sort storage %zu > %zu",
                               need, w.sort_tmp);
            size_t tb = w.sort_tmp;
            HIPCHK(nullptr, rocprim::radix_sort_pairs(w.sort_buf, tb, r1p, r2, p1, p2, (size_t)n,
                                                      0u, rbits, st));
            hipLaunchKernelGGL(k_gather3, dim3(blocks(n)), dim3(kPB), 0, st, p2, A, w.key_a, dge,
                               n, e2, w.key_c, dg2);
            HIPCHK(nullptr, hipGetLastError());
            r_sorted = r2;
            elem = e2;
            dg = dg2;
        }
        // ranks: group start, then rank + offset of the run start, carried along the run
        const bool has_r = r_sorted != nullptr;
        if (has_r)
            hipLaunchKernelGGL(k_gcand<true>, dim3(blocks(n)), dim3(kPB), 0, st, r_sorted, n, tmp);
        else
            hipLaunchKernelGGL(k_gcand<false>, dim3(blocks(n)), dim3(kPB), 0, st, r_sorted, n, tmp);
        HIPCHK(nullptr, hipGetLastError());
        HIPCHK(nullptr, max_scan(tmp, perm_a, n));  // perm_a: group start positions
        if (has_r)
            hipLaunchKernelGGL(k_rcand<true>, dim3(blocks(n)), dim3(kPB), 0, st, r_sorted, w.key_c,
                               perm_a, n, tmp);
        else
            hipLaunchKernelGGL(k_rcand<false>, dim3(blocks(n)), dim3(kPB), 0, st, r_sorted, w.key_c,
                               perm_a, n, tmp);
        HIPCHK(nullptr, hipGetLastError());
        HIPCHK(nullptr, max_scan(tmp, perm_b, n));  // perm_b: new ranks
        if (has_r)
            hipLaunchKernelGGL(k_assign<true>, dim3(blocks(n)), dim3(kPB), 0, st, r_sorted, w.key_c,
                               perm_b, elem, n, dg, rank, tmp, wsw);
        else
            hipLaunchKernelGGL(k_assign<false>, dim3(blocks(n)), dim3(kPB), 0, st, r_sorted,
                               w.key_c, perm_b, elem, n, dg, rank, tmp, wsw);
        HIPCHK(nullptr, hipGetLastError());
        // the still tied groups, in order
        size_t sel = 0;
        HIPCHK(nullptr, rocprim::select(nullptr, sel, elem, tmp, act, w.small + 2, (size_t)n, st));
        if (sel > w.sel_tmp)
            return set_err(nullptr, PU_E_STATE, "compress_patterns: select storage %zu > %zu",
                           sel, w.sel_tmp);
        sel = w.sel_tmp;
        HIPCHK(nullptr, rocprim::select(w.sel_buf, sel, elem, tmp, act, w.small + 2, (size_t)n,
                                        st));
        uint32_t cnt = 0;
        HIPCHK(nullptr, hipMemcpyAsync(&cnt, w.small + 2, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(nullptr, hipStreamSynchronize(st));
        n = cnt;
        elem_in = act;
    }
    w.rounds = rounds;
    if (n > 0)  // distinct columns always separate by the last word
        return set_err(nullptr, PU_E_STATE, "compress_patterns: %lld groups still tied",
                       (long long)n);
    hipLaunchKernelGGL(k_final, dim3(blocks(G)), dim3(kPB), 0, st, rank, rep, gfirst, G, S, srep,
                       d_counts, w.small + 4);
    hipLaunchKernelGGL(k_inverse, dim3(blocks(S)), dim3(kPB), 0, st, rank, colgrp, S, d_inverse);
    HIPCHK(nullptr, hipGetLastError());
    *U_out = G;
    return PU_OK;
}

// device-side compression; every buffer on the device, `st` the stream.  The host reads back
// a few counts between phases (the group count, each refinement round's active count).
int compress_device(hipStream_t st, int device, const uint8_t *d_codes, int n_taxa, int64_t S,
                    int n_codes, uint8_t *d_unique, int64_t ld_unique, int64_t *d_counts,
                    int64_t *d_inverse, int64_t *n_unique) {
    int b = 1;
    while ((1 << b) < n_codes) ++b;  // n_codes <= 256: b <= 8
    const int T = 64 / b, W = (n_taxa + T - 1) / T;
    Ws w;
    w.sort_tmp = w.scan_tmp = w.sel_tmp = 0;
    size_t t32 = 0, tmax = 0;
    HIPCHK(nullptr, rocprim::radix_sort_pairs(nullptr, w.sort_tmp, (uint64_t *)nullptr,
                                              (uint64_t *)nullptr, (uint32_t *)nullptr,
                                              (uint32_t *)nullptr, (size_t)S, 0, 64, st));
    HIPCHK(nullptr, rocprim::radix_sort_pairs(nullptr, t32, (uint32_t *)nullptr,
                                              (uint32_t *)nullptr, (uint32_t *)nullptr,
                                              (uint32_t *)nullptr, (size_t)S, 0, 32, st));
    HIPCHK(nullptr, rocprim::inclusive_scan(nullptr, w.scan_tmp, (uint32_t *)nullptr,
                                            (uint32_t *)nullptr, (size_t)S,
                                            rocprim::plus<uint32_t>(), st));
    HIPCHK(nullptr, rocprim::inclusive_scan(nullptr, tmax, (uint32_t *)nullptr,
                                            (uint32_t *)nullptr, (size_t)S,
                                            rocprim::maximum<uint32_t>(), st));
    HIPCHK(nullptr, rocprim::select(nullptr, w.sel_tmp, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                    (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)S, st));
    w.sort_tmp = std::max(w.sort_tmp, t32);
    w.scan_tmp = std::max(w.scan_tmp, tmax);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t n_words = al((size_t)W * S * 8), n_keys = al((size_t)S * 8),
                 n_u32 = al((size_t)S * 4);
    const size_t need = n_words + 3 * n_keys + 22 * n_u32 + 256 + al(w.sort_tmp) +
                        al(w.scan_tmp) + al(w.sel_tmp);
    PatWs &ws = g_pat[device];
    if (ws.cap < need) {
        if (ws.buf) (void)hipFree(ws.buf);
        ws.buf = nullptr;
        ws.cap = 0;
        HIPCHK(nullptr, hipMalloc(&ws.buf, need));
        ws.cap = need;
    }
    char *p = (char *)ws.buf;
    w.wordsT = (uint64_t *)p; p += n_words;
    w.key_a = (uint64_t *)p;  p += n_keys;
    w.key_b = (uint64_t *)p;  p += n_keys;
    w.key_c = (uint64_t *)p;  p += n_keys;
    for (int i = 0; i < 21; ++i) w.v[i] = (uint32_t *)p, p += n_u32;
    uint32_t *srep = (uint32_t *)p; p += n_u32;
    w.small = (uint32_t *)p;  p += 256;
    w.sort_buf = p;           p += al(w.sort_tmp);
    w.scan_buf = p;           p += al(w.scan_tmp);
    w.sel_buf = p;

    HIPCHK(nullptr, hipMemsetAsync(w.small, 0, 32, st));
    HIPCHK(nullptr, hipMemsetAsync(srep, 0xff, (size_t)S * 4, st));
    const uint64_t seeds[4] = {0x9e3779b97f4a7c15ull, 0xd1b54a32d192ed03ull,
                               0x8cb92ba72f3d8dd7ull, 0xf1357aea2e62a9c5ull};
    if (S % 4 == 0 && ((uintptr_t)d_codes & 3) == 0)
        hipLaunchKernelGGL(k_pack_T<4>, dim3((unsigned)((S + 4 * kFB - 1) / (4 * kFB))), dim3(kFB),
                           0, st, d_codes, n_taxa, S, b, T, W, n_codes, seeds[0], w.wordsT,
                           w.key_a, w.small);
    else
        hipLaunchKernelGGL(k_pack_T<1>, dim3((unsigned)((S + kFB - 1) / kFB)), dim3(kFB), 0, st,
                           d_codes, n_taxa, S, b, T, W, n_codes, seeds[0], w.wordsT, w.key_a,
                           w.small);
    HIPCHK(nullptr, hipGetLastError());
    uint32_t bad = 0;
    HIPCHK(nullptr, hipMemcpyAsync(&bad, w.small, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(nullptr, hipStreamSynchronize(st));
    if (bad)
        return set_err(nullptr, PU_E_ARG, "compress_patterns: a code is >= n_codes = %d",
                       n_codes);
    int64_t U = 0;
    bool collision = true;
    for (int i = 0; i < 4 && collision; ++i) {
        collision = false;
        int rc = refine(st, w, n_taxa, S, b, T, W, seeds[i], i == 0, srep, d_counts, d_inverse,
                        &U, &collision);
        if (rc) return rc;
    }
    if (collision)
        return set_err(nullptr, PU_E_STATE, "compress_patterns: 64-bit column hashes collided "
                       "under 4 seeds");
    const int64_t ld = ld_unique ? ld_unique : U;
    if (getenv("PU_UNPACK_LANE") == nullptr)  // (set: the per-lane form, for comparison)
        hipLaunchKernelGGL(k_unpack_lds, dim3((unsigned)((U + kUnpackCols - 1) / kUnpackCols)),
                           dim3(kPB), 0, st, w.wordsT, n_taxa, b, T, W, srep, U, S, d_unique, ld,
                           w.small + 4);
    else if (ld % 4 == 0 && ((uintptr_t)d_unique & 3) == 0)
        hipLaunchKernelGGL(k_unpack<4>, dim3(blocks((U + 3) / 4)), dim3(kPB), 0, st, w.wordsT,
                           n_taxa, b, T, W, srep, U, S, d_unique, ld, w.small + 4);
    else
        hipLaunchKernelGGL(k_unpack<1>, dim3(blocks(U)), dim3(kPB), 0, st, w.wordsT, n_taxa, b, T,
                           W, srep, U, S, d_unique, ld, w.small + 4);
    HIPCHK(nullptr, hipGetLastError());
    uint32_t err[2] = {0, 0};
    HIPCHK(nullptr, hipMemcpyAsync(err, w.small + 4, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(nullptr, hipStreamSynchronize(st));
    if (err[0] || err[1])
        return set_err(nullptr, PU_E_STATE, "compress_patterns: inconsistent pattern ranks "
                       "(%u, %u)", err[0], err[1]);
    *n_unique = U;
    return PU_OK;
}

int check_args(const void *codes, int n_taxa, int64_t S, int n_codes, const void *u,
               const void *c, const void *inv, const int64_t *n_unique) {
    if (n_taxa < 1 || n_taxa > 65000 || S < 0 || n_codes < 1 || n_codes > 256)
        return set_err(nullptr, PU_E_ARG, "compress_patterns: n_taxa=%d n_sites=%lld n_codes=%d",
                       n_taxa, (long long)S, n_codes);
    if (S >= (int64_t)1 << 32)
        return set_err(nullptr, PU_E_ARG, "compress_patterns: more than 2^32 - 1 sites");
    if (!n_unique || (S > 0 && (!codes || !u || !c || !inv)))
        return set_err(nullptr, PU_E_ARG, "compress_patterns: null buffer");
    return PU_OK;
}

}  // namespace

extern "C" {

int pu_compress_patterns_device(int device, void *stream, const uint8_t *d_codes, int n_taxa,
                                int64_t n_sites, int n_codes, uint8_t *d_unique,
                                int64_t ld_unique, int64_t *d_counts, int64_t *d_inverse,
                                int64_t *n_unique_out) {
    int rc = check_args(d_codes, n_taxa, n_sites, n_codes, d_unique, d_counts, d_inverse,
                        n_unique_out);
    if (!rc && ld_unique != 0 && ld_unique < n_sites)
        rc = set_err(nullptr, PU_E_ARG, "compress_patterns: ld_unique %lld < n_sites %lld",
                     (long long)ld_unique, (long long)n_sites);
    if (rc || (rc = check_device(device))) return rc;
    if (n_sites == 0) return *n_unique_out = 0, PU_OK;
    DeviceGuard g(device);
    std::lock_guard<std::mutex> lk(g_pat[device].mu);
    return compress_device((hipStream_t)stream, device, d_codes, n_taxa, n_sites, n_codes,
                           d_unique, ld_unique, d_counts, d_inverse, n_unique_out);
}

int pu_compress_patterns(int device, const uint8_t *codes, int n_taxa, int64_t n_sites,
                         int n_codes, uint8_t *unique_out, int64_t *counts_out,
                         int64_t *inverse_out, int64_t *n_unique_out) {
    int rc = check_args(codes, n_taxa, n_sites, n_codes, unique_out, counts_out, inverse_out,
                        n_unique_out);
    if (rc || (rc = check_device(device))) return rc;
    if (n_sites == 0) return *n_unique_out = 0, PU_OK;
    DeviceGuard g(device);
    const size_t nc = (size_t)n_taxa * n_sites;
    uint8_t *d_codes = nullptr, *d_unique = nullptr;
    int64_t *d_counts = nullptr, *d_inv = nullptr;
    hipStream_t st = nullptr;
    auto cleanup = [&]() {
        if (d_codes) (void)hipFree(d_codes);
        if (d_unique) (void)hipFree(d_unique);
        if (d_counts) (void)hipFree(d_counts);
        if (d_inv) (void)hipFree(d_inv);
        if (st) (void)hipStreamDestroy(st);
    };
    hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&d_codes, nc);
    const int64_t ld = (n_sites + 15) / 16 * 16;  // device rows padded: 4-byte stores
    if (e == hipSuccess) e = hipMalloc(&d_unique, (size_t)n_taxa * ld);
    if (e == hipSuccess) e = hipMalloc(&d_counts, n_sites * 8);
    if (e == hipSuccess) e = hipMalloc(&d_inv, n_sites * 8);
    if (e == hipSuccess) e = hipMemcpyAsync(d_codes, codes, nc, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) {
        cleanup();
        return set_err(nullptr, PU_E_HIP, "compress_patterns: %s", hipGetErrorString(e));
    }
    {
        std::lock_guard<std::mutex> lk(g_pat[device].mu);
        rc = compress_device(st, device, d_codes, n_taxa, n_sites, n_codes, d_unique, ld,
                             d_counts, d_inv, n_unique_out);
    }
    if (rc) return cleanup(), rc;
    const int64_t U = *n_unique_out;
    // [n_taxa][U] rows, compact
    e = hipMemcpy2DAsync(unique_out, (size_t)U, d_unique, (size_t)ld, (size_t)U, (size_t)n_taxa,
                         hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(counts_out, d_counts, U * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(inverse_out, d_inv, n_sites * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    cleanup();
    if (e != hipSuccess)
        return set_err(nullptr, PU_E_HIP, "compress_patterns: %s", hipGetErrorString(e));
    return PU_OK;
}

}  // extern "C"
