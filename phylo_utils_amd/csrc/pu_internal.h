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

// One post-order operation as the device walks it (32 bytes).
struct OpDesc {
    int par_slot;  // HBM slot the parent CLV is written to, -1: not stored
    int src_a;     // child 1 source (first side matrix of the op)
    int src_b;     // child 2 source (second side matrix)
    int dst;       // on-chip home of the parent until its consumer: -1 none, else
                   // src_code(SRC_REG, slot) or src_code(SRC_LDS, slot)
    int loff_a;    // LDS offset (doubles, from the chunk's side arena) of side a's matrices
    int loff_b;    // ... of side b
    int pad0, pad1;
};

// Side matrices.  For every (op, side) the device needs, per category c, either the
// transition matrix P[c] (K rows: the child is a CLV, x_i = sum_j P_ij v_j), or -- for a
// coded tip child -- its lookup table LUT[c][code][i] = sum_j P_ij table[code][j]
// (n_codes rows: x = LUT[c][code], no arithmetic).  Each (side, category) block is
// rows*K + 2 doubles (the pad puts the C blocks of a side on distinct LDS banks);
// sides are stored back to back in device op order, so a chunk of ops is one
// contiguous range that is copied to LDS as is.
__host__ __device__ inline int side_block(int rows, int K) { return rows * K + 2; }

struct TraverseArgs {
    const OpDesc *ops;        // n_ops descriptors followed by the root-combine descriptor
    const int *chunk_op;      // [n_chunks + 1] first op of each chunk
    const int *chunk_side;    // [n_chunks + 1] first side-matrix double of each chunk
    int n_chunks;
    int max_chunk_ops;        // LDS layout bounds
    int max_chunk_side;
    int n_ops;                // post-order ops, root combine excluded
    int C;                    // rate categories
    int n_codes;              // coded tips: rows of a tip LUT
    int64_t S;                // site patterns
    int64_t code_stride;      // row stride of `codes` (S rounded up to 64)
    const double *side;       // side matrices (see above)
    const double *tips;       // dense tips [n_tips][S][K]
    const uint8_t *codes;     // coded tips [n_tips][code_stride]
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
    int n_tiles;              // site tiles of 256/C patterns (one workgroup each)
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

// Padded P stride for the stateless k_clv (same idea as side_block).
__host__ __device__ constexpr int p_stride(int K) { return K * K + 2; }

struct PmatArgs {
    int K, C, n_sides, n_codes;
    const double *evecs, *evals, *ivecs;  // [K][K], [K], [K][K] row-major
    const double *brlens;                 // [n_sides]
    const double *rates;                  // [C]
    const int *side_rows;                 // [n_sides]: K (P) or n_codes (tip LUT)
    const int64_t *side_off;              // [n_sides]: first double of the side's blocks
    const double *code_table;             // [n_codes][K]
    double *P;                            // [n_sides][C][K][K] (pu_get_pmatrices)
    double *side;                         // side matrices
};

// ---- launchers (pu_kernels.hip) ----
int launch_pmatrix(hipStream_t st, const PmatArgs &a);
int traverse_sites_per_block(int C);
size_t traverse_lds_bytes(int K, int C, int max_chunk_ops, int max_chunk_side, bool coded,
                          int variant, int L);
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
