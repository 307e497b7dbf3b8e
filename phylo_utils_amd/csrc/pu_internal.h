// pu_internal.h -- shared between the HIP kernels (pu_kernels.hip) and the
// C-ABI / planning layer (pu_capi.cpp).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pu {

// Where a child CLV comes from (one 32-bit code per child, wave-uniform).
enum SrcKind : int { SRC_MEM = 0, SRC_TIP = 1, SRC_REG = 2, SRC_LDS = 3 };
__host__ __device__ inline int src_code(int kind, int index) { return (kind << 28) | index; }
__host__ __device__ inline int src_kind(int code) { return (int)((unsigned)code >> 28); }
__host__ __device__ inline int src_index(int code) { return code & 0x0FFFFFFF; }

// One post-order operation as the device walks it (16 bytes).
struct OpDesc {
    int par_slot;  // internal storage slot the parent CLV is written to, -1: not stored
    int src_a;     // child 1 source (P from the op's first matrix set)
    int src_b;     // child 2 source (P from the op's second matrix set)
    int dst;       // on-chip home of the parent until its consumer: -1 none, else
                   // src_code(SRC_REG, slot) or src_code(SRC_LDS, slot)
};

struct TraverseArgs {
    const OpDesc *ops;  // n_ops descriptors followed by the root-combine descriptor
    int n_ops;          // post-order ops, root combine excluded
    int C;              // rate categories
    int chunk;          // ops whose P matrices are staged in LDS at a time
    int n_codes;        // coded tips: rows of code_table
    int64_t S;          // site patterns
    int64_t code_stride;      // row stride of `codes` (S rounded up to 64)
    const double *P;          // [(n_ops+1)][2][C][K][K]
    const double *tips;       // dense tips [n_tips][S][K]
    const uint8_t *codes;     // coded tips [n_tips][S]
    const double *code_table; // [n_codes][K]
    double *clv;              // [n_store][S][C][K]
    double *scale;            // [n_store][S][C]
    double *root_clv;         // [S][C][K]
    double *root_scale;       // [S][C]
    const double *pi;         // [K]
    const double *logw;       // [C] log category weights
    const double *pattern_w;  // [S]
    double *site_lnl;         // [S]
    double *block_sum;        // [n_tiles]
    uint8_t *sflag;           // [n_store + 1][n_tiles * 4]: wave tile may hold non-zero scalers
    int n_tiles;              // site tiles of 256/C patterns (grid may be smaller: tile loop)
    int n_ops_store_rows;     // row of sflag used for the root scaler (= n_store)
    int variant;              // TV_* bits below
};

// k_traverse behaviour bits (TraverseArgs::variant)
enum : int {
    TV_STORE_NT = 2,         // nt stores for every CLV (default: nt only for on-chip-kept ones)
    TV_SKIP_ZERO_SCALE = 8,  // do not rewrite all-zero scaler wave tiles (sflag protocol)
    TV_NOMEM = 32,           // no child is read back from HBM in the op loop (fast path:
                             // no vector-memory loads, hence no waits on in-flight stores)
};

// Padded P row stride: (K*K + 2) doubles puts the C category matrices of one
// op on distinct LDS banks for the 16-lane groups of ds_read_b128.
__host__ __device__ constexpr int p_stride(int K) { return K * K + 2; }

// ---- launchers (pu_kernels.hip) ----
int launch_pmatrix(hipStream_t st, int K, int C, int n_br, const double *evecs,
                   const double *evals, const double *ivecs, const double *brlens,
                   const double *rates, double *P);
int traverse_sites_per_block(int C);
size_t traverse_lds_bytes(int K, int C, int chunk, int n_codes, bool coded, int variant, int L);
int launch_traverse(hipStream_t st, int K, int R, int L, bool coded, const TraverseArgs &a,
                    int grid);
// on-chip slot configurations built for K: register slots R, LDS stash slots L
bool traverse_slots_supported(int K, int R, int L);
void traverse_default_slots(int K, int *R, int *L);
size_t traverse_stash_bytes(int K, int L);
int launch_reduce(hipStream_t st, const double *block_sum, int n, double *out);
int launch_clv(hipStream_t st, int K, int C, int64_t S, const double *p1, const double *p2,
               const double *clv1, const double *clv2, const double *sa, const double *sb,
               double *cml, double *out);
int launch_lnl_node(hipStream_t st, int K, int C, int64_t S, const double *pi,
                    const double *partials, const double *scale, double *out);
int launch_expand_tip(hipStream_t st, int K, int C, int64_t S, int64_t cstride, bool coded,
                      int tip, const double *tips, const uint8_t *codes,
                      const double *code_table, double *out);
bool traverse_supported(int K);

}  // namespace pu
