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
//   k_pack      column j -> W 64-bit words, b bits per code, taxon 0 in the top bits of word
//               0: comparing words as unsigned integers, first word first, is the
//               lexicographic byte comparison; stored column-major ([S][W], W padded to a
//               multiple of 16 past 15 words) so a random column is one contiguous run;
//               word 0 also into the first round's sort keys
//   refine      every column gets a rank = its position in lexicographic order, word by word
//               (prefix refinement, as in suffix-array construction): sort by word 0; a run of
//               equal words is a group with rank = its first position; for later words only
//               the members of groups of size > 1 are re-sorted by (rank, the first word in
//               which the group's members differ from its first member) -- two stable radix
//               sorts (rocPRIM) -- and a sub-run's rank is its group's rank + its offset in the
//               group.  Distinct columns separate at their first differing word; a group none
//               of whose members differs from its first is a run of equal columns (one pattern).
//   k_mark,     the patterns are the distinct final ranks in rank order: marked, numbered by a
//   k_final     scan; inverse[j] = column j's pattern, counts by atomic adds, each pattern's
//               first column as its representative
//   k_unpack_lds unique codes [n_taxa][U] from the packed words of each pattern's column
// (r01-r05 deduplicated first: a 64-bit hash per column, one radix sort by hash, runs verified
// word by word with a retry under another seed on a collision, then the refinement over the
// distinct columns.  Refining all columns directly drops that sort, the verification and the
// host round trip: the exact duplicates cost one more round, which finds no differing word.
// A plain LSD sort of all S columns by every word -- W radix sorts -- was the first form; it is
// 8x slower at 1000 taxa.)
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

// Word w of column col in the packed words: column-major [S][W] (slab = 0), or (r06, W a
// multiple of 16) 16-word slabs [W / 16][S][16]: a column's 16 words of one slab are still one
// 128-byte line (the unpack's gathers and k_fd's 8-word steps as before), and k_pack's flush of
// a slice writes consecutive columns' words contiguously instead of 64 bytes every 512
__device__ __forceinline__ size_t wix(size_t col, int w, int W, int64_t S, int slab) {
    return slab ? ((((size_t)(w >> 4) * (size_t)S + col) << 4) + (size_t)(w & 15))
                : col * (size_t)W + (size_t)w;
}

__global__ void __launch_bounds__(kPB) k_iota(int64_t S, uint32_t *__restrict__ perm) {
    const int64_t i = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (i < S) perm[i] = (uint32_t)i;
}

// unique codes: row t of pattern u at out[t * ld + u].  V = 4: a lane unpacks patterns
// 4i..4i+3 and writes one 4-byte word per taxon row (ld % 4 == 0), 256 bytes per wave and
// row instead of 64 single-byte stores
template <int V>
__global__ void __launch_bounds__(kPB) k_unpack(const uint64_t *__restrict__ wordsT, int n_taxa,
                                                int b, int T, int W, int slab,
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
        for (int c = 0; c < V; ++c) v[c] = wordsT[wix(col[c], w, W, S, slab)];
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
// words in slices of kSliceW words: it gathers the slice of the 128 columns into LDS
// (kSliceW consecutive lanes read one column's contiguous run), then writes the slice's rows,
// one 128-byte store per wave instruction (a lane = 2 adjacent patterns, one 2-byte store;
// byte stores when ld is odd).  Small LDS (17 KB) keeps many workgroups resident to hide the
// gather latency.  Measured (cfg4 alignment, r02): the per-lane form above 1.23 ms; all 63 words of
// 64 patterns in LDS with byte stores 0.77 ms; of 128 patterns with 2-byte stores (64 KB LDS,
// 2 workgroups per CU) 0.97 ms.
// r05 late: 16-word slices.  With 8 (64 bytes of a column) the other half of each 128-byte
// line was fetched again a slice later, after the L2 had dropped it: PMC fetch 985 MB per
// call for 485 MB of columns; 16-word slices fetch 497 MB and run 0.366-0.368 ms against
// 0.378-0.380 for a 4-byte-store form with 8-word slices (256 patterns per workgroup; with
// 16-word slices that one needs 34 KB of LDS and ran 0.404 ms) -- scripts/r05/exp32, exp44.
// (r06: the next slice's 8 words per thread loaded into registers before this slice's rows
// go out: 365.7 vs 364-366 us, scripts/r06/call31.sh -- the gathers are not what waits; not
// kept)
constexpr int kUnpackCols = 128, kSliceW = 16;
// U_dev (nullable): the pattern count on the device (the grid then covers S columns, and
// workgroups past U leave) -- no host round trip between the refinement and the unpack
__global__ void __launch_bounds__(kPB) k_unpack_lds(const uint64_t *__restrict__ wordsT,
                                                    int n_taxa, int b, int T, int W, int slab,
                                                    const uint32_t *__restrict__ srep,
                                                    int64_t U, const uint32_t *__restrict__ U_dev,
                                                    int64_t S, uint8_t *__restrict__ out,
                                                    int64_t ld, uint32_t *__restrict__ err) {
    __shared__ uint64_t cols[kUnpackCols * (kSliceW + 1)];  // [column][slice word], padded
    __shared__ uint32_t colidx[kUnpackCols];
    if (U_dev) U = *U_dev;
    const int64_t u0 = (int64_t)blockIdx.x * kUnpackCols;
    if (u0 >= U) return;
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
                cols[c * (kSliceW + 1) + k] = wordsT[wix(colidx[c], w0 + k, W, S, slab)];
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

// Pack and transpose in one pass (r05): column j -> W words of b-bit codes, taxon 0 in the top
// bits of word 0, stored column-major ([S][W]: a random column is one contiguous run).  A
// workgroup packs kFB * V adjacent columns; the codes a column contributes to a slice of kPW
// words are read kRows rows at a time, every load of a batch issued before the first is used;
// a word is complete after T rows (uniform, so the flush into the LDS tile is a scalar branch);
// the tile goes out as one 64-byte run per column and slice (kPW = 8: with the column pitch a
// multiple of 16 words, half a 128-byte line).  Word 0 also goes to key0, the first
// refinement round's sort key.  Measured on the cfg4 alignment (scripts/r05/exp31, exp32):
// one word's 16 rows per wait and a 37 KB tile (4 workgroups per CU) 0.587 ms; batched loads
// with 4 / 8 / 16-word slices 0.674 / 0.626 / 0.572 ms on the 63-word pitch and, on the
// 64-word pitch, 0.448 ms with 8-word slices (0.570 with 16, 0.463 for the first form).
// (r06: 256 threads of 2-byte loads or 512 of 1-byte loads for the same 512 columns per
// workgroup -- 2 / 4 times the waves per CU -- ran the same, 1.51-1.55 ms per compression on one
// box, scripts/r06/call22.sh: the pass is not short of waves)
// (r06: PF -- the next batch's 64 rows are loaded before this batch is packed, across slice
// boundaries too, so a wave's loads stay in flight while it packs and flushes; the registers
// are there at 2 waves per SIMD, the LDS tile's occupancy)
constexpr int kFB = 128, kPW = 8, kRows = 64;
template <int V, int FB = kFB, bool PF = false, int NR = kRows>
__global__ void __launch_bounds__(FB, 2) k_pack(const uint8_t *__restrict__ codes, int n_taxa,
                                                int64_t S, int b, int T, int W, int slab,
                                                int n_codes,
                                                uint64_t *__restrict__ wordsT,
                                                uint64_t *__restrict__ key0,
                                                uint32_t *__restrict__ bad) {
    constexpr int NC = FB * V;                        // columns per workgroup
    __shared__ uint64_t tile[NC * (kPW + 1)];         // [column][kPW + 1]: odd row pitch
    const int64_t jb = (int64_t)blockIdx.x * NC;
    const int64_t j = jb + (int64_t)threadIdx.x * V;
    const bool live = j < S;                          // (S % V == 0 when V > 1)
    const int ncol = (int)min((int64_t)NC, S - jb);
    const uint8_t *src = codes + (live ? j : 0);
    uint64_t acc[V];
#pragma unroll
    for (int c = 0; c < V; ++c) acc[c] = 0;
    bool ok = true;
    uint32_t xn[PF ? NR : 1];  // PF: the next batch, in flight
    auto load_rows = [&](uint32_t *dst, int r0) {  // rows past the last re-read the last
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const uint8_t *a = src + (size_t)min(r0 + i, n_taxa - 1) * S;
            if constexpr (V == 4)
                dst[i] = *reinterpret_cast<const uint32_t *>(a);
            else
                dst[i] = *a;
        }
    };
    for (int w0 = 0; w0 < W; w0 += kPW) {
        const int nw = min(kPW, W - w0);
        const int r1 = min(n_taxa, (w0 + nw) * T);
        int cnt = 0, wi = 0;  // rows in the current word, word in the slice (uniform)
        auto flush = [&]() {
            const int used = cnt * b;  // 0: a padding word past the last taxon
#pragma unroll
            for (int c = 0; c < V; ++c) {
                const uint64_t v = used == 0 ? 0 : used < 64 ? acc[c] << (64 - used) : acc[c];
                if (w0 + wi == 0 && live) key0[j + c] = v;
                tile[(threadIdx.x * V + c) * (kPW + 1) + wi] = v;
                acc[c] = 0;
            }
            cnt = 0;
            ++wi;
        };
        for (int rb = w0 * T; rb < r1; rb += NR) {
            const int nr = min(NR, r1 - rb);
            uint32_t x[NR];
            if constexpr (PF) {
                // this batch from the prefetch registers (the first: loaded now); then the
                // next batch -- the rest of this slice, or the next slice's first rows
                if (rb == 0) load_rows(xn, rb);
#pragma unroll
                for (int i = 0; i < NR; ++i) x[i] = xn[i];
                const int rn = rb + NR < r1 ? rb + NR : r1;
                if (rn < n_taxa) load_rows(xn, rn);
            } else {  // unconditional: rows past r1 re-read the last
#pragma unroll
                for (int i = 0; i < NR; ++i) {
                    const uint8_t *a = src + (size_t)min(rb + i, r1 - 1) * S;
                    if constexpr (V == 4)
                        x[i] = *reinterpret_cast<const uint32_t *>(a);
                    else
                        x[i] = *a;
                }
            }
#pragma unroll
            for (int i = 0; i < NR; ++i) {
                if (i < nr) {
#pragma unroll
                    for (int c = 0; c < V; ++c) {
                        const uint32_t code = (x[i] >> (8 * c)) & 0xffu;
                        ok &= code < (uint32_t)n_codes;
                        acc[c] = (acc[c] << b) | code;
                    }
                    if (++cnt == T) flush();
                }
            }
        }
        if (cnt > 0) flush();  // the column's last word, part filled
        while (wi < nw) flush();  // padding words (the column pitch), zero
        __syncthreads();
        for (int e = threadIdx.x; e < ncol * nw; e += FB) {
            const int c = e / nw, wj = e - c * nw;
            wordsT[wix(jb + c, w0 + wj, W, S, slab)] = tile[c * (kPW + 1) + wj];
        }
        __syncthreads();
    }
    if (!ok) *bad = 1u;  // a code outside [0, n_codes): reported, not packed silently
}

__global__ void __launch_bounds__(kPB) k_gather_u32(const uint32_t *__restrict__ src,
                                                    const uint32_t *__restrict__ idx, int64_t n,
                                                    uint32_t *__restrict__ out) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a < n) out[a] = src[idx[a]];
}

// Position p of a group (rank r; R = false: a single group) starts a run of its sorted
// (class, key).  Branch-free on purpose: with short-circuit loads (`p == 0 || r[p] != r[p - 1]`)
// the ROCm 7.2 compiler emitted `v_mov v, 0` for every lane of the p != 0 side of the select
// (k_gcand wrote 0 where it had to write p; caught by tests/test_gpu_patterns.py,
// near-duplicate columns), so every load is unconditional and the choices are selects.
template <bool R>
__device__ __forceinline__ bool run_start(const uint32_t *r, const uint32_t *c,
                                          const uint64_t *k, int64_t p) {
    const int64_t q = p > 0 ? p - 1 : 0;
    bool s = (p == 0) | (k[p] != k[q]);
    if constexpr (R) s = s | (r[p] != r[q]) | (c[p] != c[q]);
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
                                               const uint32_t *__restrict__ c,
                                               const uint64_t *__restrict__ k,
                                               const uint32_t *__restrict__ gp, int64_t n,
                                               uint32_t *__restrict__ rcand) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    uint32_t base = 0;
    if constexpr (R) base = r[a];
    const uint32_t v = base + ((uint32_t)a - gp[a]);
    rcand[a] = run_start<R>(r, c, k, a) ? v : 0u;
}

// new ranks; a column stays active while its run has more than one member, unless the run is
// the group's first column and its copies (class W: no differing word, one pattern)
// ws: the next round's known-equal word prefix of the element's run: its first differing word
// + 1 (R = false: word 0 was the key)
template <bool R>
__global__ void __launch_bounds__(kPB) k_assign(const uint32_t *__restrict__ r,
                                                const uint32_t *__restrict__ c,
                                                const uint64_t *__restrict__ k,
                                                const uint32_t *__restrict__ nr,
                                                const uint32_t *__restrict__ elem, int64_t n,
                                                const uint32_t *__restrict__ dg, int W,
                                                uint32_t *__restrict__ rank,
                                                uint32_t *__restrict__ tied,
                                                uint32_t *__restrict__ ws) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    rank[elem[a]] = nr[a];
    uint32_t next_ws = 1;
    bool done = false;
    if constexpr (R) {
        next_ws = dg[a] + 1;
        done = c[a] == (uint32_t)W;
    }
    ws[elem[a]] = next_ws;
    const bool next = (a + 1 == n) | run_start<R>(r, c, k, a + 1 < n ? a + 1 : a);
    tied[a] = !(run_start<R>(r, c, k, a) & next) & !done;
}

// Word skipping: the first word (from the group's known-equal prefix ws) at which element a
// differs from its group's first column f (W: none), and the element's sort class and key
// within its group, which order the group lexicographically in one round:
//   class fd, key word fd        a < f (a[fd] < f[fd]): a smaller fd sorts first
//   class W, key 0               a == f: f and its copies, one pattern
//   class 2W - fd, key word fd   a > f: a larger fd sorts first
// Elements tied on (class, key) agree with each other through word fd and go on to the next
// round.  (r02-r05: one split word per group -- the group's smallest fd -- and one round per
// level: the near-duplicate families of the cfg4 alignment took 6-7 rounds.)
// (The first fd form scanned every word with branch-free selects; the early exit took the 5
// calls per cfg4 compression from 269 to 225 us, r02.)
__global__ void __launch_bounds__(kPB) k_fd(const uint64_t *__restrict__ words, int W, int slab,
                                            int64_t S,
                                            const uint32_t *__restrict__ A,
                                            const uint32_t *__restrict__ gp,
                                            const uint32_t *__restrict__ ws, int64_t n,
                                            uint32_t *__restrict__ fdv,
                                            uint32_t *__restrict__ cls,
                                            uint64_t *__restrict__ key) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    const size_t x = A[a], y = A[gp[a]];
    const int w0 = (int)ws[A[a]];
    uint32_t fd = (uint32_t)W;
    uint64_t xv = 0, yv = 0;
    // forward from the known-equal prefix, leaving at the first difference; eight words of
    // both columns per step, all loads issued before the compare (r05 late: one word per step
    // made every step wait on its own loads; index clamped to the last word, so a step past
    // the end compares copies of a word it has already compared)
    // (from the known-equal prefix rounded down to 8 words -- the words before it are equal,
    // so the first difference is the same -- each step is 8 contiguous words of one slab)
    for (int w = x == y ? W : (w0 & ~7); w < W; w += 8) {  // (the group's first column: itself)
        uint64_t dx[8], dy[8];
        const uint64_t *px = words + wix(x, w, W, S, slab), *py = words + wix(y, w, W, S, slab);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int k = min(i, W - 1 - w);
            dx[i] = px[k];
            dy[i] = py[k];
        }
        int f = 8;
#pragma unroll
        for (int i = 7; i >= 0; --i) f = dx[i] != dy[i] ? i : f;
        if (f < 8) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (i == f) xv = dx[i], yv = dy[i];
            fd = (uint32_t)min(w + f, W - 1);
            break;
        }
    }
    fdv[a] = fd;
    cls[a] = fd == (uint32_t)W ? (uint32_t)W : xv < yv ? fd : 2u * W - fd;
    key[a] = xv;
}


// Small groups settled in place (r06): after k_fd, a group of at most
// kSettleMax members is ordered by one thread -- a stable insertion sort of its members by
// (class, key), exactly the order the round's two radix sorts give it -- which writes the new
// ranks, the known-equal prefixes and the members in sorted order with their "still tied" flags
// (a run of equal (class, key) outside class W, left for the next round).  Larger groups are
// flagged and take the sorts.  On the cfg4 alignment every group of round 1 is a pair or a
// triple of near-duplicates, so the round's sorts over ~600k members go.
constexpr int kSettleMax = 16;
__global__ void __launch_bounds__(kPB) k_settle(const uint32_t *__restrict__ A,
                                                const uint32_t *__restrict__ r,
                                                const uint32_t *__restrict__ gp,
                                                const uint32_t *__restrict__ fdv,
                                                const uint32_t *__restrict__ cls,
                                                const uint64_t *__restrict__ key, int64_t n, int W,
                                                uint32_t *__restrict__ rank,
                                                uint32_t *__restrict__ ws,
                                                uint32_t *__restrict__ out_elem,
                                                uint32_t *__restrict__ out_tied,
                                                uint32_t *__restrict__ big) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    const int64_t g = gp[a];
    // more than kSettleMax members: the member kSettleMax past the start is still in the group
    const bool isbig = g + kSettleMax < n && (int64_t)gp[g + kSettleMax] == g;
    big[a] = isbig ? 1u : 0u;
    if (isbig) {
        out_tied[a] = 0u;
        return;
    }
    if (a != g) return;  // the group's first member's thread orders the group
    uint32_t c[kSettleMax], e[kSettleMax], f[kSettleMax];
    uint64_t k[kSettleMax];
    int m = 0;
    for (; m < kSettleMax && a + m < n && (int64_t)gp[a + m] == g; ++m) {
        c[m] = cls[a + m];
        k[m] = key[a + m];
        e[m] = A[a + m];
        f[m] = fdv[a + m];
        // stable insertion: past every member with a smaller or equal (class, key)
        for (int q = m; q > 0 && (c[q - 1] > c[q] || (c[q - 1] == c[q] && k[q - 1] > k[q])); --q) {
            const uint32_t tc = c[q], te = e[q], tf = f[q];
            const uint64_t tk = k[q];
            c[q] = c[q - 1], e[q] = e[q - 1], f[q] = f[q - 1], k[q] = k[q - 1];
            c[q - 1] = tc, e[q - 1] = te, f[q - 1] = tf, k[q - 1] = tk;
        }
    }
    const uint32_t rr = r[a];
    int s0 = 0;  // start of the current run of equal (class, key)
    for (int p = 0; p < m; ++p) {
        if (p > 0 && (c[p] != c[p - 1] || k[p] != k[p - 1])) s0 = p;
        const bool same_next = p + 1 < m && c[p + 1] == c[p] && k[p + 1] == k[p];
        const bool tied = (p > s0 || same_next) && c[p] != (uint32_t)W;
        rank[e[p]] = rr + (uint32_t)s0;
        ws[e[p]] = f[p] + 1;
        out_elem[a + p] = e[p];
        out_tied[a + p] = tied ? 1u : 0u;
    }
}

// The tail (r06): once at most kTailMax columns are still tied and none of
// their groups needs the sorts, one workgroup runs every remaining round in LDS -- group starts
// by a block scan, k_fd's first differing word, class and key per member, k_settle's in-place
// order per group, the still-tied members compacted by a second scan -- instead of a round of
// ~9 launches and a host round trip each.  small[2] / small[6]: the list's count and the round's
// big-group members (k_settle); small[7] out: 0 not run (too many, or a big group), 1 done,
// 2 stopped before a round that has a big group (the list back in `act`, its count in small[2]).
constexpr int kTail = 1024;  // threads = the most columns the tail takes
__device__ __forceinline__ uint32_t tail_scan(uint32_t v, bool is_max, uint32_t *wsum) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t u = __shfl_up(v, off);
        if (lane >= off) v = is_max ? max(v, u) : v + u;
    }
    if (lane == 63) wsum[wid] = v;
    __syncthreads();
    if (t < kTail / 64) {
        uint32_t x = wsum[t];
        for (int off = 1; off < kTail / 64; off <<= 1) {
            const uint32_t u = __shfl_up(x, off, kTail / 64);
            if (t >= off) x = is_max ? max(x, u) : x + u;
        }
        wsum[t] = x;
    }
    __syncthreads();
    if (wid > 0) v = is_max ? max(v, wsum[wid - 1]) : v + wsum[wid - 1];
    __syncthreads();  // wsum is reused by the next scan
    return v;
}

__global__ void __launch_bounds__(kTail) k_tail(const uint64_t *__restrict__ words, int W,
                                                int slab, int64_t S,
                                                uint32_t *__restrict__ act,
                                                uint32_t *__restrict__ rank,
                                                uint32_t *__restrict__ ws,
                                                uint32_t *__restrict__ small) {
    __shared__ uint32_t col[kTail], rk[kTail], wse[kTail], gp[kTail], fd[kTail], cl[kTail];
    __shared__ uint32_t oc[kTail], orank[kTail], ows[kTail], tf[kTail], wsum[kTail / 64];
    __shared__ uint64_t key[kTail];
    __shared__ uint32_t sh_n;
    const int i = threadIdx.x;
    uint32_t n = small[2];
    if (small[6] != 0 || n > (uint32_t)kTail) {
        if (i == 0) small[7] = 0;
        return;
    }
    if (i < (int)n) {
        col[i] = act[i];
        rk[i] = rank[col[i]];
        wse[i] = ws[col[i]];
    }
    __syncthreads();
    for (int round = 0; round <= W + 1 && n > 0; ++round) {
        const bool live = i < (int)n;
        // group start per member: a max scan of the run starts (ranks are sorted per group)
        // (branch-free, like run_start: see k_gcand's note on the ROCm 7.2 select miscompile)
        const uint32_t prev = rk[i > 0 ? i - 1 : 0];
        const bool s = live & ((i == 0) | (rk[i] != prev));
        const uint32_t st = s ? (uint32_t)i : 0u;
        gp[i] = tail_scan(st, true, wsum);
        __syncthreads();
        const bool big = live && gp[i] == (uint32_t)i && i + kSettleMax < (int)n &&
                         gp[i + kSettleMax] == (uint32_t)i;
        if (__syncthreads_or(big)) {  // a group for the sorts: the host's rounds go on from here
            if (live) act[i] = col[i];
            if (i == 0) {
                small[2] = n;
                small[7] = 2;
            }
            return;
        }
        if (live) {  // k_fd's first differing word, class and key
            const uint32_t x = col[i], y = col[gp[i]];
            uint32_t f = (uint32_t)W;
            uint64_t xv = 0, yv = 0;
            for (int w = x == y ? W : ((int)wse[i] & ~7); w < W; w += 8) {  // k_fd's steps
                uint64_t dx[8], dy[8];
                const uint64_t *px = words + wix(x, w, W, S, slab);
                const uint64_t *py = words + wix(y, w, W, S, slab);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int kq = min(q, W - 1 - w);
                    dx[q] = px[kq];
                    dy[q] = py[kq];
                }
                int d = 8;
#pragma unroll
                for (int q = 7; q >= 0; --q) d = dx[q] != dy[q] ? q : d;
                if (d < 8) {
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if (q == d) xv = dx[q], yv = dy[q];
                    f = (uint32_t)min(w + d, W - 1);
                    break;
                }
            }
            fd[i] = f;
            cl[i] = f == (uint32_t)W ? (uint32_t)W : xv < yv ? f : 2u * W - f;
            key[i] = xv;
        }
        __syncthreads();
        if (live && gp[i] == (uint32_t)i) {  // k_settle's order of this group
            uint32_t c[kSettleMax], e[kSettleMax], fv[kSettleMax];
            uint64_t k[kSettleMax];
            int m = 0;
            for (; m < kSettleMax && i + m < (int)n && gp[i + m] == (uint32_t)i; ++m) {
                c[m] = cl[i + m];
                k[m] = key[i + m];
                e[m] = col[i + m];
                fv[m] = fd[i + m];
                for (int q = m; q > 0 && (c[q - 1] > c[q] || (c[q - 1] == c[q] && k[q - 1] > k[q]));
                     --q) {
                    const uint32_t tc = c[q], te = e[q], tfv = fv[q];
                    const uint64_t tk = k[q];
                    c[q] = c[q - 1], e[q] = e[q - 1], fv[q] = fv[q - 1], k[q] = k[q - 1];
                    c[q - 1] = tc, e[q - 1] = te, fv[q - 1] = tfv, k[q - 1] = tk;
                }
            }
            const uint32_t rr = rk[i];
            int s0 = 0;
            for (int p = 0; p < m; ++p) {
                if (p > 0 && (c[p] != c[p - 1] || k[p] != k[p - 1])) s0 = p;
                const bool same_next = p + 1 < m && c[p + 1] == c[p] && k[p + 1] == k[p];
                const bool tied = (p > s0 || same_next) && c[p] != (uint32_t)W;
                rank[e[p]] = rr + (uint32_t)s0;
                ws[e[p]] = fv[p] + 1;
                oc[i + p] = e[p];
                orank[i + p] = rr + (uint32_t)s0;
                ows[i + p] = fv[p] + 1;
                tf[i + p] = tied ? 1u : 0u;
            }
        }
        __syncthreads();
        const uint32_t flag = live ? tf[i] : 0u;
        const uint32_t pos = tail_scan(flag, false, wsum);  // inclusive
        if (i == kTail - 1) sh_n = pos;
        if (flag) {
            col[pos - 1] = oc[i];
            rk[pos - 1] = orank[i];
            wse[pos - 1] = ows[i];
        }
        __syncthreads();
        n = sh_n;
    }
    if (i == 0) {
        small[2] = n;  // 0 (the round bound past W + 1 is never reached: every round splits)
        small[7] = n == 0 ? 1u : 2u;
    }
    if (n > 0 && i < (int)n) act[i] = col[i];
}

// (rank, class) as one 32-bit sort key, in key order (when both fit 32 bits)
__global__ void __launch_bounds__(kPB) k_rc_key(const uint32_t *__restrict__ r,
                                                const uint32_t *__restrict__ cls,
                                                const uint32_t *__restrict__ p1, int64_t n,
                                                unsigned cbits, uint32_t *__restrict__ out) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    const uint32_t p = p1[a];
    out[a] = (r[p] << cbits) | cls[p];
}

// after the sorts: element, key, class, first differing word and rank in (rank, class, key)
// order
__global__ void __launch_bounds__(kPB) k_gather5(const uint32_t *__restrict__ p2,
                                                 const uint32_t *__restrict__ A,
                                                 const uint64_t *__restrict__ key,
                                                 const uint32_t *__restrict__ cls,
                                                 const uint32_t *__restrict__ fdv,
                                                 const uint32_t *__restrict__ r, int64_t n,
                                                 uint32_t *__restrict__ elem,
                                                 uint64_t *__restrict__ keys,
                                                 uint32_t *__restrict__ cs,
                                                 uint32_t *__restrict__ dg,
                                                 uint32_t *__restrict__ rs) {
    const int64_t a = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (a >= n) return;
    const uint32_t p = p2[a];
    elem[a] = A[p];
    keys[a] = key[p];
    cs[a] = cls[p];
    dg[a] = fdv[p];
    rs[a] = r[p];
}

// The patterns are the distinct final ranks, in rank order.  A final rank is the position of
// its run of equal columns in the lexicographic order of all S columns, so the next pattern's
// rank is this one's + its count.  k_mark: mark[rank] = 1 and the column at that position (any
// of the run: they are equal); an inclusive scan numbers the marks (pattern = scan - 1).
// (The first form took counts by atomic adds and the first column by atomicMin: 86 us on the
// cfg4 alignment.)
__global__ void __launch_bounds__(kPB) k_mark(const uint32_t *__restrict__ rank, int64_t S,
                                              uint32_t *__restrict__ mark,
                                              uint32_t *__restrict__ colat,
                                              uint32_t *__restrict__ err) {
    const int64_t j = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (j >= S) return;
    const uint32_t r = rank[j];
    if (r >= (uint64_t)S) {  // (ranks are positions in [0, S): never taken)
        err[0] = 1u;
        return;
    }
    mark[r] = 1u;
    colat[r] = (uint32_t)j;
}

// index j is a column (its pattern: inverse) and a position (a marked one starts pattern u:
// its representative column and position)
__global__ void __launch_bounds__(kPB) k_final(const uint32_t *__restrict__ rank,
                                               const uint32_t *__restrict__ num,
                                               const uint32_t *__restrict__ mark,
                                               const uint32_t *__restrict__ colat, int64_t S,
                                               int64_t *__restrict__ inverse,
                                               uint32_t *__restrict__ srep,
                                               uint32_t *__restrict__ upos) {
    const int64_t j = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (j >= S) return;
    const uint32_t r = min(rank[j], (uint32_t)(S - 1));  // (out of range: k_mark reported it)
    inverse[j] = (int64_t)num[r] - 1;
    if (mark[j]) {
        const uint32_t u = num[j] - 1;
        srep[u] = colat[j];
        upos[u] = (uint32_t)j;
    }
}

// counts[u] = position of pattern u + 1 (S past the last) - position of u
__global__ void __launch_bounds__(kPB) k_counts(const uint32_t *__restrict__ upos,
                                                const uint32_t *__restrict__ nU, int64_t S,
                                                int64_t *__restrict__ counts,
                                                uint32_t *__restrict__ U_out) {
    const int64_t u = (int64_t)blockIdx.x * kPB + threadIdx.x;
    const uint32_t U = *nU;
    if (u == 0) *U_out = U;
    if (u >= (int64_t)U) return;
    const int64_t next = u + 1 < (int64_t)U ? (int64_t)upos[u + 1] : S;
    counts[u] = next - upos[u];
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + kPB - 1) / kPB); }

template <class K>
hipError_t radix_pairs(void *tmp, size_t &bytes, const K *kin, K *kout, const uint32_t *vin,
                       uint32_t *vout, size_t n, unsigned b0, unsigned b1, hipStream_t st) {
    // (rocPRIM's default: block sort + merge passes up to 2^20 items.  Forcing Onesweep from
    // 64k items was slower here, 2.77-2.88 vs 2.61-2.65 ms per compression: its look-back
    // state fills and eight digit passes over 64-bit keys, scripts/r05/exp33_sorts.sh.)
    return rocprim::radix_sort_pairs(tmp, bytes, kin, kout, vin, vout, n, b0, b1, st);
}

struct PatWs {
    std::mutex mu;
    void *buf = nullptr;
    size_t cap = 0;
    // the flags and counts the host reads between phases: pinned, mapped host memory the
    // kernels (and rocPRIM's selects) write directly -- no copy launch per read-back (r06)
    uint32_t *hsmall = nullptr, *dsmall = nullptr;
};
PatWs g_pat[64];

// Workspace of one compression (S columns, W words per column).
struct Ws {
    uint64_t *wordsT, *key_a, *key_b, *key_c;  // wordsT [S][W] (column-major)
    uint32_t *v[25];   // S-sized u32 scratch arrays
    uint32_t *small;   // [0] bad code, [2] selected count, [4] bad rank, [5] pattern without
                       // column, [6] members of big groups (k_settle), [7] k_tail's state,
                       // [8] pattern count: the device alias of hsmall
    volatile uint32_t *hsmall;
    int slab = 0;      // packed-word layout (wix): 16-word slabs when W % 16 == 0
    void *sort_buf, *scan_buf, *sel_buf;
    size_t sort_tmp, scan_tmp, sel_tmp;
    int rounds = 0;    // refinement rounds of the last compression
};

inline unsigned rank_bits(int64_t n) {  // key bits for ranks < n, rounded up to bytes
    unsigned b = 8;
    while (b < 32 && ((int64_t)1 << b) < n) b += 8;
    return b;
}

// refinement over all S columns (header comment); returns U
// U_out (nullable): the pattern count read back; *U_dev_out: where it is on the device
int refine(hipStream_t st, Ws &w, int n_taxa, int64_t S, int b, int T, int W, uint32_t *srep,
           int64_t *d_counts, int64_t *d_inverse, int64_t *U_out, const uint32_t **U_dev_out) {
    uint32_t *perm_a = w.v[0], *perm_b = w.v[1], *num = w.v[2], *cls = w.v[3], *c1p = w.v[4],
             *c2 = w.v[5], *p1b = w.v[6], *rank = w.v[7], *act = w.v[8], *e1 = w.v[9],
             *r1 = w.v[10], *r2 = w.v[11], *e2 = w.v[12], *tmp = w.v[13], *cs = w.v[14],
             *fdv = w.v[15], *p1 = w.v[16], *r1p = w.v[17], *p2 = w.v[18], *dg2 = w.v[19],
             *wsw = w.v[20], *s_elem = w.v[21], *s_tied = w.v[22], *bigf = w.v[23],
             *bbuf = w.v[24];
    const bool settle = getenv("PU_PAT_NO_SETTLE") == nullptr;  // (set: every group sorted)
    const bool tail = settle && getenv("PU_PAT_NO_TAIL") == nullptr;
    auto sort64 = [&](const uint64_t *kin, uint64_t *kout, const uint32_t *vin, uint32_t *vout,
                      int64_t n, int word) -> hipError_t {
        const int used = std::min(n_taxa - word * T, T) * b;
        const unsigned begin = word < 0 ? 0u : (unsigned)((64 - used) / 8 * 8);
        size_t need = 0;  // (the temporary storage was sized for S keys over all 64 bits)
        hipError_t e = radix_pairs(nullptr, need, kin, kout, vin, vout, (size_t)n, begin, 64u, st);
        if (e != hipSuccess) return e;
        if (need > w.sort_tmp) return hipErrorInvalidValue;
        size_t tb = w.sort_tmp;
        return radix_pairs(w.sort_buf, tb, kin, kout, vin, vout, (size_t)n, begin, 64u, st);
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
    auto sort32 = [&](const uint32_t *kin, uint32_t *kout, const uint32_t *vin, uint32_t *vout,
                      int64_t n, unsigned bits) -> hipError_t {
        size_t need = 0;
        hipError_t e = radix_pairs(nullptr, need, kin, kout, vin, vout, (size_t)n, 0u, bits, st);
        if (e != hipSuccess) return e;
        if (need > w.sort_tmp) return hipErrorInvalidValue;
        size_t tb = w.sort_tmp;
        return radix_pairs(w.sort_buf, tb, kin, kout, vin, vout, (size_t)n, 0u, bits, st);
    };
    const unsigned rbits = rank_bits(S), cbits = rank_bits(2 * (int64_t)W + 1);
    auto bits_for = [](int64_t n) {  // bits of the values 0 .. n - 1
        unsigned b = 1;
        while (((int64_t)1 << b) < n) ++b;
        return b;
    };
    const unsigned rb = bits_for(S), cb = bits_for(2 * (int64_t)W + 1);
    // (cfg4 alignment: 20 + 8 bits; PU_PAT_TWO_SORTS: the two-sort form, for the tests)
    const bool rc32 = rb + cb <= 32 && getenv("PU_PAT_TWO_SORTS") == nullptr;
    // ---- refinement: word 0 for every column; then each tied group by the first word in
    // which its members differ (word skipping), until every group is one column or a run of
    // equal columns (a group none of whose members differs from its first)
    int64_t n = S;
    const uint32_t *elem_in = nullptr;  // active columns (nullptr: all, as 0..S-1)
    int rounds = 0;
    for (; rounds <= W + 1 && n > 0; ++rounds) {
        uint32_t *sel_out = act;  // this round's still-tied columns (after the settled ones)
        uint32_t n_settled = 0;   // of them, from k_settle
        if (rounds > 0 && settle) {
            const uint32_t *A = elem_in;
            hipLaunchKernelGGL(k_gather_u32, dim3(blocks(n)), dim3(kPB), 0, st, rank, A, n, r1);
            hipLaunchKernelGGL(k_gcand<true>, dim3(blocks(n)), dim3(kPB), 0, st, r1, n, tmp);
            HIPCHK(nullptr, hipGetLastError());
            HIPCHK(nullptr, max_scan(tmp, perm_a, n));
            hipLaunchKernelGGL(k_fd, dim3(blocks(n)), dim3(kPB), 0, st, w.wordsT, W, w.slab, S, A, perm_a,
                               wsw, n, fdv, cls, w.key_a);
            hipLaunchKernelGGL(k_settle, dim3(blocks(n)), dim3(kPB), 0, st, A, r1, perm_a, fdv,
                               cls, w.key_a, n, W, rank, wsw, s_elem, s_tied, bigf);
            HIPCHK(nullptr, hipGetLastError());
            // the big groups' members (in order) for the sorts below; the settled groups'
            // still-tied members first in the next round's list
            size_t sel = w.sel_tmp;
            HIPCHK(nullptr, rocprim::select(w.sel_buf, sel, A, bigf, bbuf, w.small + 6, (size_t)n,
                                            st));
            sel = w.sel_tmp;
            HIPCHK(nullptr, rocprim::select(w.sel_buf, sel, s_elem, s_tied, act, w.small + 2,
                                            (size_t)n, st));
            if (tail)  // the remaining rounds in one workgroup when few columns are left
                hipLaunchKernelGGL(k_tail, dim3(1), dim3(kTail), 0, st, w.wordsT, W, w.slab, S, act, rank, wsw,
                                   w.small);
            HIPCHK(nullptr, hipGetLastError());
            HIPCHK(nullptr, hipStreamSynchronize(st));
            uint32_t cnt[6];
            for (int k = 0; k < 6; ++k) cnt[k] = w.hsmall[2 + k];
            if (tail && cnt[5] == 1) {  // the tail finished every round
                n = 0;
                continue;
            }
            if (tail && cnt[5] == 2) {  // the tail stopped at a big group: the host's rounds go on
                n = cnt[0];
                elem_in = act;
                continue;
            }
            n_settled = cnt[0];
            if (cnt[4] == 0) {  // no big group: the round is done
                n = n_settled;
                elem_in = act;
                continue;
            }
            elem_in = bbuf;
            n = cnt[4];
            sel_out = act + n_settled;
        }
        const uint32_t *r_sorted = nullptr;  // ranks in the sorted order (nullptr: word 0)
        uint32_t *elem;                      // columns in (rank, key) order
        const uint32_t *dg = nullptr;        // split word per element, in that order
        if (rounds == 0) {  // key_a: word 0 of every column (k_pack)
            hipLaunchKernelGGL(k_iota, dim3(blocks(S)), dim3(kPB), 0, st, S, e1);
            HIPCHK(nullptr, hipGetLastError());
            HIPCHK(nullptr, sort64(w.key_a, w.key_c, e1, e2, S, 0));
            elem = e2;
        } else {
            const uint32_t *A = elem_in;
            // group start of every active element, then its first differing word, class and key
            hipLaunchKernelGGL(k_gather_u32, dim3(blocks(n)), dim3(kPB), 0, st, rank, A, n, r1);
            hipLaunchKernelGGL(k_gcand<true>, dim3(blocks(n)), dim3(kPB), 0, st, r1, n, tmp);
            HIPCHK(nullptr, hipGetLastError());
            HIPCHK(nullptr, max_scan(tmp, perm_a, n));
            hipLaunchKernelGGL(k_fd, dim3(blocks(n)), dim3(kPB), 0, st, w.wordsT, W, w.slab, S, A, perm_a,
                               wsw, n, fdv, cls, w.key_a);
            hipLaunchKernelGGL(k_iota, dim3(blocks(n)), dim3(kPB), 0, st, n, e1);
            HIPCHK(nullptr, hipGetLastError());
            // stable by key, then by (rank, class): (rank, class, key) order; p2 = sources
            HIPCHK(nullptr, sort64(w.key_a, w.key_b, e1, p1, n, -1));
            if (rc32) {  // one sort by the composite key
                hipLaunchKernelGGL(k_rc_key, dim3(blocks(n)), dim3(kPB), 0, st, r1, cls, p1, n,
                                   cb, c1p);
                HIPCHK(nullptr, hipGetLastError());
                HIPCHK(nullptr, sort32(c1p, c2, p1, p2, n, rb + cb));
            } else {  // by class, then by rank
                hipLaunchKernelGGL(k_gather_u32, dim3(blocks(n)), dim3(kPB), 0, st, cls, p1, n,
                                   c1p);
                HIPCHK(nullptr, hipGetLastError());
                HIPCHK(nullptr, sort32(c1p, c2, p1, p1b, n, cbits));
                hipLaunchKernelGGL(k_gather_u32, dim3(blocks(n)), dim3(kPB), 0, st, r1, p1b, n,
                                   r1p);
                HIPCHK(nullptr, hipGetLastError());
                HIPCHK(nullptr, sort32(r1p, r2, p1b, p2, n, rbits));
            }
            hipLaunchKernelGGL(k_gather5, dim3(blocks(n)), dim3(kPB), 0, st, p2, A, w.key_a, cls,
                               fdv, r1, n, e2, w.key_c, cs, dg2, r2);
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
            hipLaunchKernelGGL(k_rcand<true>, dim3(blocks(n)), dim3(kPB), 0, st, r_sorted, cs,
                               w.key_c, perm_a, n, tmp);
        else
            hipLaunchKernelGGL(k_rcand<false>, dim3(blocks(n)), dim3(kPB), 0, st, r_sorted, cs,
                               w.key_c, perm_a, n, tmp);
        HIPCHK(nullptr, hipGetLastError());
        HIPCHK(nullptr, max_scan(tmp, perm_b, n));  // perm_b: new ranks
        if (has_r)
            hipLaunchKernelGGL(k_assign<true>, dim3(blocks(n)), dim3(kPB), 0, st, r_sorted, cs,
                               w.key_c, perm_b, elem, n, dg, W, rank, tmp, wsw);
        else
            hipLaunchKernelGGL(k_assign<false>, dim3(blocks(n)), dim3(kPB), 0, st, r_sorted, cs,
                               w.key_c, perm_b, elem, n, dg, W, rank, tmp, wsw);
        HIPCHK(nullptr, hipGetLastError());
        // the still tied groups, in order
        size_t sel = 0;
        HIPCHK(nullptr, rocprim::select(nullptr, sel, elem, tmp, sel_out, w.small + 2, (size_t)n,
                                        st));
        if (sel > w.sel_tmp)
            return set_err(nullptr, PU_E_STATE, "compress_patterns: select storage %zu > %zu",
                           sel, w.sel_tmp);
        sel = w.sel_tmp;
        HIPCHK(nullptr, rocprim::select(w.sel_buf, sel, elem, tmp, sel_out, w.small + 2,
                                        (size_t)n, st));
        HIPCHK(nullptr, hipStreamSynchronize(st));
        const uint32_t cnt = w.hsmall[2];
        n = cnt + n_settled;  // groups are contiguous in the list; its order across groups is free
        elem_in = act;
    }
    w.rounds = rounds;
    if (n > 0)  // distinct columns separate by the last word, equal ones finish the round after
        return set_err(nullptr, PU_E_STATE, "compress_patterns: %lld columns still tied",
                       (long long)n);
    // patterns = distinct final ranks; inverse, counts and a representative column of each
    uint32_t *colat = perm_a, *upos = perm_b;
    HIPCHK(nullptr, hipMemsetAsync(tmp, 0, (size_t)S * 4, st));
    hipLaunchKernelGGL(k_mark, dim3(blocks(S)), dim3(kPB), 0, st, rank, S, tmp, colat,
                       w.small + 4);
    HIPCHK(nullptr, hipGetLastError());
    {
        size_t sb = w.scan_tmp;
        HIPCHK(nullptr, rocprim::inclusive_scan(w.scan_buf, sb, tmp, num, (size_t)S,
                                                rocprim::plus<uint32_t>(), st));
    }
    hipLaunchKernelGGL(k_final, dim3(blocks(S)), dim3(kPB), 0, st, rank, num, tmp, colat, S,
                       d_inverse, srep, upos);
    hipLaunchKernelGGL(k_counts, dim3(blocks(S)), dim3(kPB), 0, st, upos, num + (S - 1), S,
                       d_counts, w.small + 8);
    HIPCHK(nullptr, hipGetLastError());
    *U_dev_out = num + (S - 1);
    if (U_out) {
        HIPCHK(nullptr, hipStreamSynchronize(st));
        *U_out = w.hsmall[8];
    }
    return PU_OK;
}

// device-side compression; every buffer on the device, `st` the stream.  The host reads back
// a few counts between phases (the group count, each refinement round's active count).
int compress_device(hipStream_t st, int device, const uint8_t *d_codes, int n_taxa, int64_t S,
                    int n_codes, uint8_t *d_unique, int64_t ld_unique, int64_t *d_counts,
                    int64_t *d_inverse, int64_t *n_unique) {
    int b = 1;
    while ((1 << b) < n_codes) ++b;  // n_codes <= 256: b <= 8
    // W: the column pitch in words.  Past 15 words it is rounded up to 16 (zero padding words,
    // which compare equal and unpack to no rows), so that a column starts on a 128-byte line
    // and k_pack's 8-word slices are half lines (cfg4 alignment, 63 -> 64 words: k_pack_T
    // 0.587 -> 0.463 ms, k_fd and the duplicate check 10-15 % faster, scripts/r05/exp32).
    const int T = 64 / b, Wr = (n_taxa + T - 1) / T, W = Wr < 16 ? Wr : (Wr + 15) / 16 * 16;
    Ws w;
    w.sort_tmp = w.scan_tmp = w.sel_tmp = 0;
    size_t t32 = 0, tmax = 0;
    HIPCHK(nullptr, radix_pairs(nullptr, w.sort_tmp, (uint64_t *)nullptr,
                                              (uint64_t *)nullptr, (uint32_t *)nullptr,
                                              (uint32_t *)nullptr, (size_t)S, 0, 64, st));
    HIPCHK(nullptr, radix_pairs(nullptr, t32, (uint32_t *)nullptr,
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
    const size_t need = n_words + 3 * n_keys + 26 * n_u32 + 256 + al(w.sort_tmp) +
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
    for (int i = 0; i < 25; ++i) w.v[i] = (uint32_t *)p, p += n_u32;
    uint32_t *srep = (uint32_t *)p; p += n_u32;
    p += 256;  // (the flags live in ws.hsmall since r06)
    w.sort_buf = p;           p += al(w.sort_tmp);
    w.scan_buf = p;           p += al(w.scan_tmp);
    w.sel_buf = p;

    if (!ws.hsmall) {
        HIPCHK(nullptr, hipHostMalloc((void **)&ws.hsmall, 256, hipHostMallocMapped));
        HIPCHK(nullptr, hipHostGetDevicePointer((void **)&ws.dsmall, ws.hsmall, 0));
    }
    // (the previous compression on this device has finished: each ends synchronised)
    for (int k = 0; k < 64; ++k) ws.hsmall[k] = 0;
    w.small = ws.dsmall;
    w.hsmall = ws.hsmall;
    HIPCHK(nullptr, hipMemsetAsync(srep, 0xff, (size_t)S * 4, st));
    w.slab = W % 16 == 0 && getenv("PU_PAT_COLMAJOR") == nullptr;  // (set: [S][W], the r05 form)
    const bool v4 = S % 4 == 0 && ((uintptr_t)d_codes & 3) == 0;
    const bool pf = getenv("PU_PACK_PF") == nullptr || atoi(getenv("PU_PACK_PF")) != 0;
    if (v4 && pf)
        hipLaunchKernelGGL((k_pack<4, kFB, true, 32>), dim3((unsigned)((S + 4 * kFB - 1) / (4 * kFB))),
                           dim3(kFB), 0, st, d_codes, n_taxa, S, b, T, W, w.slab, n_codes,
                           w.wordsT, w.key_a, w.small);
    else if (v4)
        hipLaunchKernelGGL(k_pack<4>, dim3((unsigned)((S + 4 * kFB - 1) / (4 * kFB))), dim3(kFB),
                           0, st, d_codes, n_taxa, S, b, T, W, w.slab, n_codes, w.wordsT,
                           w.key_a, w.small);
    else
        hipLaunchKernelGGL(k_pack<1>, dim3((unsigned)((S + kFB - 1) / kFB)), dim3(kFB), 0, st,
                           d_codes, n_taxa, S, b, T, W, w.slab, n_codes, w.wordsT, w.key_a,
                           w.small);
    HIPCHK(nullptr, hipGetLastError());
    // (a code >= n_codes is reported after the last launch, with the rank checks: it only
    // makes the packed words, and so the patterns, wrong -- every index stays in range)
    // The unique rows' stride: the caller's, or U (compact rows: U read back first)
    int64_t U = 0;
    const uint32_t *U_dev = nullptr;
    const bool lane = getenv("PU_UNPACK_LANE") != nullptr;  // (set: the per-lane form)
    if (int rc = refine(st, w, n_taxa, S, b, T, W, srep, d_counts, d_inverse,
                        ld_unique && !lane ? nullptr : &U, &U_dev))
        return rc;
    const int64_t ld = ld_unique ? ld_unique : U;
    const bool aligned4 = ld % 4 == 0 && ((uintptr_t)d_unique & 3) == 0;
    if (!lane && ld_unique)  // the grid covers S columns; U from the device
        hipLaunchKernelGGL(k_unpack_lds, dim3((unsigned)((S + kUnpackCols - 1) / kUnpackCols)),
                           dim3(kPB), 0, st, w.wordsT, n_taxa, b, T, W, w.slab, srep, S, U_dev,
                           S, d_unique, ld, w.small + 4);
    else if (!lane)
        hipLaunchKernelGGL(k_unpack_lds, dim3((unsigned)((U + kUnpackCols - 1) / kUnpackCols)),
                           dim3(kPB), 0, st, w.wordsT, n_taxa, b, T, W, w.slab, srep, U,
                           (const uint32_t *)nullptr, S, d_unique, ld, w.small + 4);
    else if (aligned4)
        hipLaunchKernelGGL(k_unpack<4>, dim3(blocks((U + 3) / 4)), dim3(kPB), 0, st, w.wordsT,
                           n_taxa, b, T, W, w.slab, srep, U, S, d_unique, ld, w.small + 4);
    else
        hipLaunchKernelGGL(k_unpack<1>, dim3(blocks(U)), dim3(kPB), 0, st, w.wordsT, n_taxa, b, T,
                           W, w.slab, srep, U, S, d_unique, ld, w.small + 4);
    HIPCHK(nullptr, hipGetLastError());
    HIPCHK(nullptr, hipStreamSynchronize(st));
    uint32_t sm[9];  // [0] bad code, [4] [5] rank checks, [8] pattern count
    for (int k = 0; k < 9; ++k) sm[k] = w.hsmall[k];
    const uint32_t Ud = sm[8];
    if (sm[0])
        return set_err(nullptr, PU_E_ARG, "compress_patterns: a code is >= n_codes = %d",
                       n_codes);
    if (sm[4] || sm[5])
        return set_err(nullptr, PU_E_STATE, "compress_patterns: inconsistent pattern ranks "
                       "(%u, %u)", sm[4], sm[5]);
    *n_unique = U_dev ? (int64_t)Ud : U;
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
    // an error can leave launches of this call in flight: drained before the next call on
    // this device reuses the workspace and the mapped flags
    rc = compress_device((hipStream_t)stream, device, d_codes, n_taxa, n_sites, n_codes,
                         d_unique, ld_unique, d_counts, d_inverse, n_unique_out);
    if (rc) (void)hipStreamSynchronize((hipStream_t)stream);
    return rc;
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
        if (rc) (void)hipStreamSynchronize(st);  // (as above)
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
