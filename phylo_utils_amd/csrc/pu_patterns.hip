// pu_patterns.hip -- site-pattern compression on the GPU (the data format on
// the way into the pruning path): the reference's
//     np.unique(alignment, return_inverse=True, return_counts=True, axis=1)
// (phylo_utils/alignment/alignment.py:40-57) over tip codes instead of [ntaxa][S][K] float
// partials.  A column is the byte string codes[0..n_taxa)[j]; np.unique orders the columns
// lexicographically, taxon 0 first, and numbers them in that order.  With codes whose order
// is the lexicographic order of their partial vectors (alignment.char_codes guarantees it),
// the byte order of code columns is the order np.unique gives the float columns, so the
// unique columns, the inverse index and the counts are exactly the reference's.
//
//   k_pack      column j -> W = ceil(n_taxa * b / 64) 64-bit words, b bits per code, taxon 0
//               in the top bits of word 0: comparing words as unsigned integers, most
//               significant word first, is the lexicographic byte comparison
//   LSD sort    rocprim::radix_sort_pairs by word W-1, ..., 0 (stable): the permutation that
//               sorts the columns (only the b * taxa bits a word holds are sorted)
//   k_flags     a column starts a new pattern when any word differs from its predecessor's
//   scan        rocprim::inclusive_scan of the flags: pattern number of every sorted column
//   k_scatter   inverse[perm[i]] = pattern; first[pattern] = i at the pattern's first column
//   k_unpack    unique codes [n_taxa][U] from the packed words of each pattern's first column;
//               counts[u] = first[u + 1] - first[u]
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <mutex>
#include <vector>

#include "pu_ctx.h"

using namespace pu;

namespace {

constexpr int kPB = 256;

__global__ void __launch_bounds__(kPB) k_pack(const uint8_t *__restrict__ codes, int n_taxa,
                                              int64_t S, int b, int T, int n_codes,
                                              uint64_t *__restrict__ words,
                                              uint32_t *__restrict__ bad) {
    const int64_t j = (int64_t)blockIdx.x * kPB + threadIdx.x;
    const int w = blockIdx.y;
    if (j >= S) return;
    const int t0 = w * T, t1 = min(n_taxa, t0 + T);
    uint64_t v = 0;
    bool ok = true;
    for (int t = t0; t < t1; ++t) {
        const uint32_t c = codes[(size_t)t * S + j];
        ok &= c < (uint32_t)n_codes;
        v = (v << b) | c;
    }
    if (!ok) *bad = 1u;  // a code outside [0, n_codes): reported, not packed silently
    const int used = (t1 - t0) * b;
    if (used < 64) v <<= (64 - used);
    words[(size_t)w * S + j] = v;
}

__global__ void __launch_bounds__(kPB) k_iota(int64_t S, uint32_t *__restrict__ perm) {
    const int64_t i = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (i < S) perm[i] = (uint32_t)i;
}

__global__ void __launch_bounds__(kPB) k_gather_key(const uint64_t *__restrict__ word,
                                                    const uint32_t *__restrict__ perm, int64_t S,
                                                    uint64_t *__restrict__ key) {
    const int64_t i = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (i < S) key[i] = word[perm[i]];
}

__global__ void __launch_bounds__(kPB) k_flags(const uint64_t *__restrict__ words, int W,
                                               int64_t S, const uint32_t *__restrict__ perm,
                                               uint32_t *__restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (i >= S) return;
    uint32_t f = 1;
    if (i > 0) {
        const size_t a = perm[i], p = perm[i - 1];
        f = 0;
        for (int w = 0; w < W && !f; ++w) f = words[(size_t)w * S + a] != words[(size_t)w * S + p];
    }
    flag[i] = f;
}

__global__ void __launch_bounds__(kPB) k_scatter(const uint32_t *__restrict__ perm,
                                                 const uint32_t *__restrict__ flag,
                                                 const uint32_t *__restrict__ id, int64_t S,
                                                 int64_t *__restrict__ inverse,
                                                 uint32_t *__restrict__ first) {
    const int64_t i = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (i >= S) return;
    const uint32_t u = id[i] - 1;
    inverse[perm[i]] = u;
    if (flag[i]) first[u] = (uint32_t)i;
}

__global__ void __launch_bounds__(kPB) k_unpack(const uint64_t *__restrict__ words, int n_taxa,
                                                int64_t S, int b, int T, int W,
                                                const uint32_t *__restrict__ perm,
                                                const uint32_t *__restrict__ first, int64_t U,
                                                uint8_t *__restrict__ out,
                                                int64_t *__restrict__ counts) {
    const int64_t u = (int64_t)blockIdx.x * kPB + threadIdx.x;
    if (u >= U) return;
    const uint32_t f = first[u];
    counts[u] = (int64_t)(u + 1 < U ? first[u + 1] : (uint32_t)S) - f;
    const size_t col = perm[f];
    const uint64_t mask = (b == 64) ? ~0ull : ((1ull << b) - 1);
    for (int w = 0; w < W; ++w) {
        const uint64_t v = words[(size_t)w * S + col];
        const int t0 = w * T, t1 = min(n_taxa, t0 + T);
        for (int t = t0; t < t1; ++t)
            out[(size_t)t * U + u] = (uint8_t)((v >> (64 - (t - t0 + 1) * b)) & mask);
    }
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + kPB - 1) / kPB); }

struct PatWs {
    std::mutex mu;
    void *buf = nullptr;
    size_t cap = 0;
};
PatWs g_pat[64];

// device-side compression; every buffer on the device, `st` the stream.  n_unique is read
// back (the only host synchronisation).
int compress_device(hipStream_t st, int device, const uint8_t *d_codes, int n_taxa, int64_t S,
                    int n_codes, uint8_t *d_unique, int64_t *d_counts, int64_t *d_inverse,
                    int64_t *n_unique) {
    int b = 1;
    while ((1 << b) < n_codes) ++b;  // n_codes <= 256: b <= 8
    const int T = 64 / b, W = (n_taxa + T - 1) / T;
    // workspace: words [W][S] u64, keys x2 [S] u64, perm x2, flag, id [S] u32, first [S] u32,
    // then the radix sort / scan temporaries
    size_t sort_tmp = 0, scan_tmp = 0;
    HIPCHK(nullptr, rocprim::radix_sort_pairs(nullptr, sort_tmp, (uint64_t *)nullptr,
                                              (uint64_t *)nullptr, (uint32_t *)nullptr,
                                              (uint32_t *)nullptr, (size_t)S, 0, 64, st));
    HIPCHK(nullptr, rocprim::inclusive_scan(nullptr, scan_tmp, (uint32_t *)nullptr,
                                            (uint32_t *)nullptr, (size_t)S,
                                            rocprim::plus<uint32_t>(), st));
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t n_words = al((size_t)W * S * 8), n_keys = al((size_t)S * 8),
                 n_u32 = al((size_t)S * 4);
    const size_t need = n_words + 2 * n_keys + 5 * n_u32 + 256 + al(sort_tmp) + al(scan_tmp);
    PatWs &ws = g_pat[device];
    if (ws.cap < need) {
        if (ws.buf) (void)hipFree(ws.buf);
        ws.buf = nullptr;
        ws.cap = 0;
        HIPCHK(nullptr, hipMalloc(&ws.buf, need));
        ws.cap = need;
    }
    char *p = (char *)ws.buf;
    uint64_t *words = (uint64_t *)p;              p += n_words;
    uint64_t *key_a = (uint64_t *)p;              p += n_keys;
    uint64_t *key_b = (uint64_t *)p;              p += n_keys;
    uint32_t *perm_a = (uint32_t *)p;             p += n_u32;
    uint32_t *perm_b = (uint32_t *)p;             p += n_u32;
    uint32_t *flag = (uint32_t *)p;               p += n_u32;
    uint32_t *id = (uint32_t *)p;                 p += n_u32;
    uint32_t *first = (uint32_t *)p;              p += n_u32;
    uint32_t *bad = (uint32_t *)p;                p += 256;
    void *sort_buf = p;                           p += al(sort_tmp);
    void *scan_buf = p;

    HIPCHK(nullptr, hipMemsetAsync(bad, 0, 4, st));
    hipLaunchKernelGGL(k_pack, dim3(blocks(S), W), dim3(kPB), 0, st, d_codes, n_taxa, S, b, T,
                       n_codes, words, bad);
    HIPCHK(nullptr, hipGetLastError());
    hipLaunchKernelGGL(k_iota, dim3(blocks(S)), dim3(kPB), 0, st, S, perm_a);
    HIPCHK(nullptr, hipGetLastError());
    // least significant word first; each pass is stable, so the last (word 0) decides first
    for (int w = W - 1; w >= 0; --w) {
        const int used = std::min(n_taxa - w * T, T) * b;
        const uint64_t *keys_in = words + (size_t)w * S;
        if (w != W - 1) {  // (the first pass runs on the identity permutation)
            hipLaunchKernelGGL(k_gather_key, dim3(blocks(S)), dim3(kPB), 0, st, keys_in, perm_a,
                               S, key_a);
            HIPCHK(nullptr, hipGetLastError());
            keys_in = key_a;
        }
        // the word's bits are [64 - used, 64); the sorted range starts at a byte boundary
        // below that (the low bits are zero) -- rocPRIM's radix_sort_pairs mis-sorted a
        // 60-bit range [4, 64) (tests/test_gpu_patterns.py, 5-bit codes)
        const unsigned begin = (unsigned)((64 - used) / 8 * 8);
        size_t tb = sort_tmp;
        HIPCHK(nullptr, rocprim::radix_sort_pairs(sort_buf, tb, keys_in, key_b, perm_a, perm_b,
                                                  (size_t)S, begin, 64u, st));
        std::swap(perm_a, perm_b);
    }
    hipLaunchKernelGGL(k_flags, dim3(blocks(S)), dim3(kPB), 0, st, words, W, S, perm_a, flag);
    HIPCHK(nullptr, hipGetLastError());
    size_t sb = scan_tmp;
    HIPCHK(nullptr, rocprim::inclusive_scan(scan_buf, sb, flag, id, (size_t)S,
                                            rocprim::plus<uint32_t>(), st));
    hipLaunchKernelGGL(k_scatter, dim3(blocks(S)), dim3(kPB), 0, st, perm_a, flag, id, S,
                       d_inverse, first);
    HIPCHK(nullptr, hipGetLastError());
    uint32_t hb[2] = {0, 0};  // U, bad
    HIPCHK(nullptr, hipMemcpyAsync(hb, id + (S - 1), 4, hipMemcpyDeviceToHost, st));
    HIPCHK(nullptr, hipMemcpyAsync(hb + 1, bad, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(nullptr, hipStreamSynchronize(st));
    if (hb[1])
        return set_err(nullptr, PU_E_ARG, "compress_patterns: a code is >= n_codes = %d",
                       n_codes);
    const uint32_t U32 = hb[0];
    const int64_t U = U32;
    hipLaunchKernelGGL(k_unpack, dim3(blocks(U)), dim3(kPB), 0, st, words, n_taxa, S, b, T, W,
                       perm_a, first, U, d_unique, d_counts);
    HIPCHK(nullptr, hipGetLastError());
    *n_unique = U;
    return PU_OK;
}

int check_args(const void *codes, int n_taxa, int64_t S, int n_codes, const void *u,
               const void *c, const void *inv, const int64_t *n_unique) {
    if (n_taxa < 1 || S < 0 || n_codes < 1 || n_codes > 256)
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
                                int64_t *d_counts, int64_t *d_inverse, int64_t *n_unique_out) {
    int rc = check_args(d_codes, n_taxa, n_sites, n_codes, d_unique, d_counts, d_inverse,
                        n_unique_out);
    if (rc || (rc = check_device(device))) return rc;
    if (n_sites == 0) return *n_unique_out = 0, PU_OK;
    DeviceGuard g(device);
    std::lock_guard<std::mutex> lk(g_pat[device].mu);
    return compress_device((hipStream_t)stream, device, d_codes, n_taxa, n_sites, n_codes,
                           d_unique, d_counts, d_inverse, n_unique_out);
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
    if (e == hipSuccess) e = hipMalloc(&d_unique, nc);
    if (e == hipSuccess) e = hipMalloc(&d_counts, n_sites * 8);
    if (e == hipSuccess) e = hipMalloc(&d_inv, n_sites * 8);
    if (e == hipSuccess) e = hipMemcpyAsync(d_codes, codes, nc, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) {
        cleanup();
        return set_err(nullptr, PU_E_HIP, "compress_patterns: %s", hipGetErrorString(e));
    }
    {
        std::lock_guard<std::mutex> lk(g_pat[device].mu);
        rc = compress_device(st, device, d_codes, n_taxa, n_sites, n_codes, d_unique, d_counts,
                             d_inv, n_unique_out);
    }
    if (rc) return cleanup(), rc;
    const int64_t U = *n_unique_out;
    // [n_taxa][U] rows, compact
    e = hipMemcpyAsync(unique_out, d_unique, (size_t)n_taxa * U, hipMemcpyDeviceToHost, st);
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
