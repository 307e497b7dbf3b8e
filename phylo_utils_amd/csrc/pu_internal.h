// pu_internal.h -- shared between the HIP kernels (pu_kernels.hip) and the
// C-ABI / planning layer (pu_capi.cpp).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pu {

// How an op finds its children (pu_capi.cpp canonicalises the child order):
//   PAT_LC  a: a waiting parent in LDS stash slot ia,   b: the previous op's parent
//   PAT_MC  a: a waiting parent read back from HBM,      b: the previous op's parent
//   PAT_CT  a: the previous op's parent,                 b: a tip
//   PAT_TT  a: a tip,                                    b: a tip
//   PAT_MT  a: read back from HBM,                       b: a tip
//   PAT_MM  a: read back from HBM,                       b: read back from HBM
// A DFS post-order only needs LC/MC, CT and TT; MT and MM serve other caller orders.
enum : int { PAT_LC = 0, PAT_CT = 1, PAT_TT = 2, PAT_MT = 3, PAT_MM = 4, PAT_MC = 5 };

// One post-order operation as the device walks it (32 bytes: one s_load_dwordx8).
// The op's two transition matrices are P[2t] (child a) and P[2t+1] (child b).
struct OpDesc {
    int par_slot;  // HBM slot the parent CLV is written to, -1: not stored; | kReadBack when
                   // a later op of the same run reads it back (cached store, else streamed)
    int pat;       // PAT_*
    int ia;        // child a: LDS stash slot (PAT_LC), HBM slot (PAT_M*), tip slot (PAT_TT)
    int ib;        // child b: HBM slot (PAT_MM) or tip slot (PAT_CT, PAT_TT, PAT_MT)
    int dst;       // LDS stash slot the parent waits in for its consumer, -1: none
    int use0;      // the op's first tip use, counted from its staging chunk's first use
                   // (filled by upload_schedule; the DNA kernel indexes the staged codes
                   // with it instead of keeping a running count)
    long long par_off;  // the parent's CLV slot as a byte offset, (par_slot & ~kReadBack) x
                        // slot bytes (0: not stored); its scaler slot is par_off / K.  K = 20:
                        // the scaler slot's byte offset (the CLV slot's is 20 x it).  Filled
                        // by upload_schedule: the kernels add it to their wave's base instead
                        // of a 64-bit multiply on the scalar unit per op
};
static_assert(sizeof(OpDesc) == 32, "one s_load_dwordx8 per descriptor");

constexpr int kReadBack = 1 << 30;
constexpr int kTile = 64;
constexpr int kChunkOps = 64;   // max ops per staging chunk (scaler-flag mask: one 64-bit word)
constexpr int kChunkUses = 32;  // target tip uses per chunk (codes staged in LDS per chunk)

__host__ __device__ inline int64_t tile_count(int64_t S) { return (S + kTile - 1) / kTile; }
// Tiles per (slot, category) row of the tiled CLV / scaler / root layouts: the tile count, plus
// one unused tile when it is a multiple of 256.  Power-of-two tile counts put a workgroup's
// category rows (written together, op by op) at power-of-two distances: 2048 and 4096 tiles
// (131072 / 262144 sites) ran 12-14 % slower per update than one tile fewer or more
// (profiles/r04_sweep_pow2_before_pitch.txt; with the pitch: r04_sweep_pow2.txt).
// Layout only: grids and loops still run tile_count(S) tiles.
__host__ __device__ inline int64_t tile_pitch(int64_t S) {
    const int64_t n = tile_count(S);
    return n % 256 == 0 ? n + 1 : n;
}
// PU_PITCH_EXTRA (an r05 A/B knob, read at pu_ctx_create and latched with the schedule) widens
// a context's rows by up to kPitchPad - 1 unused tiles (pu_ctx::pitch_extra); only a context
// created with the knob set allocates tile_pitch(S) + kPitchPad tiles per row (pu_ctx::pitch_pad)
constexpr int kPitchPad = 8;
// Row (64-site block) of (category, tile) in a slot of the tiled CLV / scaler / root layouts.
// DNA (r04 late): tile-major, tile * C + category -- a workgroup's category blocks are one
// contiguous run per op, so no distance between category rows exists to alias: +3 % geometric
// mean over a 50k-150k-site sweep, +0.4..8 % per size, cfg4 +1.2 % against category-major
// rows (profiles/r04_tile_major_ab/).  Protein: category-major, category * pitch + tile.
// A slot still spans C * tile_pitch(S) rows.
__host__ __device__ constexpr size_t layout_row(int K, int C, int64_t pitch, int cat,
                                                int64_t tile) {
    return K == 20 ? (size_t)(cat * pitch + tile) : (size_t)(tile * C + cat);
}
// Protein (K = 20) CLV of one wave's 16 sites: a lane (g = lane >> 4, site lane & 15) holds
// rows g, g + 4, g + 8, g + 12 and 16 + g (values r = 0..4), stored as [pair 0: r 0, 1]
// [pair 1: r 2, 3] (64 lanes x 16 B each) then [r 4] (64 lanes x 8 B): 2.5 KB per wave, written
// with two 16-byte and one 8-byte store per lane (r04; [r][64 lanes] before: five 8-byte stores)
__host__ __device__ constexpr int aa_row_off(int r, int lane) {
    return r < 4 ? (r >> 1) * 128 + 2 * lane + (r & 1) : 256 + lane;
}
// tiles per workgroup: C*T waves per workgroup
__host__ __device__ inline int tiles_per_block(int C) { return C <= 4 ? 4 / C : 1; }

struct TraverseArgs {
    const OpDesc *ops;        // n_ops descriptors followed by the root-combine descriptor
    const int *chunk_op0;     // [n_chunks + 1] first op of each chunk (last: n_ops + 1)
    const int *chunk_tip0;    // [n_chunks + 1] index of the first tip use of each chunk
    const int *tip_seq;       // [n_uses] tip slot of every tip use, in schedule order
    int n_ops;                // post-order ops, root combine excluded
    int n_chunks;             // staging chunks (host: <= kChunkOps ops, ~kChunkUses tip uses)
    int max_chunk_uses;       // LDS sizing of the staged tip codes
    int C;                    // rate categories
    int T;                    // tiles per workgroup (tiles_per_block(C))
    int n_codes;              // rows of the code table (coded tips)
    int n_tiles;              // tile_count(S)
    int tile_pitch;           // tile_pitch(S): tiles per (slot, category) row of the layouts
    int n_store;              // HBM slots (row n_store of sflag: the root scaler)
    int64_t S;                // site patterns
    int64_t code_stride;      // row stride of `codes` (multiple of 64, zero padded)
    const double *P;          // [2 (n_ops + 1)][C][K][K]
    double *Pa;               // K = 20: P as MFMA A operands [2 (n_ops + 1)][C][5][64][2]
    const double *table;      // [n_codes][K]
    const uint8_t *codes;     // coded tips [n_tips][code_stride]
    const double *tips;       // dense tips [n_tips][S][K]
    double *clv;              // tiled, [n_store] slots
    double *scale;            // tiled
    double *root_clv;         // tiled, one slot
    double *root_scale;
    const double *pi;         // [K]
    const double *logw;       // [C] log category weights
    const double *pattern_w;  // [S]
    double *site_lnl;         // [S]
    double *block_sum;        // [grid]
    uint32_t *sflag;          // [n_store + 1][C * n_tiles]: wave tile may hold non-zero scalers
    double *cat_lnl;          // 4 % C != 0 only: [C][n_tiles * 64] per-category site lnL
    int n_lds;                // LDS stash slots (waiting parents kept on chip)
    int lds_pad;              // extra LDS bytes per workgroup (occupancy experiments)
    int waves;                // kernel build targeting this many waves per SIMD (0: default)
    int pa_ready = 0;         // K = 20: Pa already written by launch_pmatrix (no k_pa launch)
    // K = 20 split plans: {op_lo, op_hi, chunk_lo, chunk_hi} of the n_tasks chain tasks, then
    // of the top task (ops [op_lo, n_ops) and the root combine); block = task * n_tiles * C +
    // tile * C + cat; ticket[n_tiles * C] (zero between launches) elects the workgroup that
    // runs the top task.  nullptr: one whole-tree task per (tile, category)
    const int *tasks = nullptr;
    int n_tasks = 0;
    int *ticket = nullptr;
    // K = 20: per-tile tickets (zero between launches); the last of a tile's C workgroups
    // combines its categories (no k_site_lse).  nullptr: k_site_lse runs after the traversal
    int *lse_ticket = nullptr;
    // K = 20 with lse_ticket: the last arriving tile also adds every tile's sum in k_reduce's
    // order into *lnl_out (lse_ticket[n_tiles] is the grid ticket); nullptr: k_reduce runs
    double *lnl_out = nullptr;
    // r06, DNA single-tree launches without chain tasks (pu_enqueue): each workgroup's block
    // sum into red_slots[2 bid .. 2 bid + 1] as two (32-bit half, 32-bit red_gen) words, and
    // the grid's last workgroup adds the red_n sums in k_reduce's order into *red_out -- no
    // k_reduce launch, no atomics (every earlier workgroup has been dispatched before it, so
    // its wait ends); nullptr: block_sum and k_reduce
    uint64_t *red_slots = nullptr;
    double *red_out = nullptr;
    unsigned red_gen = 0;
    int red_n = 0;
    const double *PT = nullptr;  // TV_PTIP: [2 (n_ops + 1)][C][n_codes][K]
    unsigned long long *timing;  // debug (PU_TIMING): per-phase s_memtime sums of one wave
    // buffer sizes in bytes, for the PU_CHECK diagnostic build (device-side bounds checks)
    size_t pa_bytes, clv_bytes, scale_bytes, root_bytes, root_scale_bytes, lds_bytes;
};

// k_prune behaviour bits (template parameter)
enum : int {
    TV_SKIP_ZERO_SCALE = 8,  // do not rewrite all-zero scaler wave tiles (sflag protocol)
    TV_GENERIC = 16,         // HBM read-backs (PAT_MC / PAT_MT / PAT_MM): stash overflow or
                             // schedules that are not DFS orders
    TV_KEEP = 32,            // every op stores its parent (K = 20 kernel: fixed store count)
    TV_CHAIN = 64,           // split plan: chain tasks + the top task by the last arriver
    TV_PTIP = 128,           // coded tip children read P*table rows (PmatArgs::PT), lnL only
    // 256: TV_PAIR (k_prune_pair, two tiles per wave), measured slower, removed in r05
    TV_RSLOTS = 512,         // KEEP, default build: stash slots n_lds, n_lds + 1 in registers
};

// Padded P stride for the stateless k_clv.
__host__ __device__ constexpr int p_stride(int K) { return K * K + 2; }

struct PmatArgs {
    int K, C, n_sides;
    const double *evecs, *evals, *ivecs;  // [K][K], [K], [K][K] row-major
    const double *brlens;                 // [n_sides]
    const double *rates;                  // [C]
    double *P;                            // [n_sides][C][K][K]
    double *Pa = nullptr;                 // K = 20: also write the MFMA A operands (k_pa layout)
    // K <= 4 lnL-only coded traversals (TV_PTIP): PT[side][cat][code][i] = sum_j P[i][j]
    // table[code][j], the tip child's product, in matvec_s's operation order
    double *PT = nullptr;
    const double *table = nullptr;  // [n_codes][K]
    int n_codes = 0;
};

// ---- edge operations on device-resident CLVs (pu_edge.hip / pu_edge.cpp) ----
// Where one end of an edge (or one child of an update) lives.
enum : int { SRC_CODED = 0, SRC_DENSE = 1, SRC_SLOT = 2 };
struct NodeSrc {
    int kind;  // SRC_*
    int idx;   // tip slot (SRC_CODED / SRC_DENSE) or HBM storage slot (SRC_SLOT)
};
// One in-place partials update: partials[par_slot] = clv(P(t_a), P(t_b), a, b)
// (numba_likelihood_engine.py:35-44; the re-orientation rows of utils.py:137-188).
struct EdgeOp {
    NodeSrc a, b;
    int par_slot;
    int pad;
    double t_a, t_b;
};
constexpr int kEdgeOpsPerLaunch = 8;
constexpr int kEdgeInlineP = 4 * 4 * 4 * 4;  // EdgeArgs::hp: 4 matrices x C <= 4 x 4 x 4
enum : int { EDGE_UPDATE = 0, EDGE_LNL = 1, EDGE_DERIV = 2 };
struct EdgeArgs {
    int K, C, n_tiles, n_ops;     // n_ops: EDGE_UPDATE only (<= kEdgeOpsPerLaunch)
    int tile_pitch;               // tile_pitch(S): tiles per (slot, category) layout row
    int64_t S, code_stride;
    EdgeOp op[kEdgeOpsPerLaunch]; // EDGE_LNL / EDGE_DERIV: op[0] = the edge (a: P(0), b: P(t_b))
    const uint8_t *codes;
    const double *table, *tips;
    double *clv, *scale;          // tiled slots (pu_ctx d_clv / d_scale)
    double *root_clv, *root_scale;
    size_t slot_stride, sstride;  // doubles per CLV slot / scaler slot
    uint32_t *sflag;              // [n_store + 1][C * n_tiles] (k_prune skip-zero protocol)
    int n_store;
    int two_pass;                 // 1: per-workgroup partials + a k_edge_sum launch, 0: ticket,
                                  // 2: partials only (into host memory; the host adds them)
    const double *evecs, *evals, *ivecs, *rates, *pi, *logw, *pattern_w;
    const double *weights;        // [C] category weights (EDGE_DERIV's linear-domain mix)
    // host-supplied matrices instead of the eigen build (pu_set_pmatrix_provider): EDGE_LNL
    // [2][C][K][K] (P(0), P(t)), EDGE_DERIV [4][C][K][K] (+ dP/dt, d2P/dt2), EDGE_UPDATE
    // [n_ops][2][C][K][K]; nullptr: built from evecs / evals / ivecs
    const double *pmats;
    // EDGE_DERIV, K <= 4, C <= 4: P(0), P(t), dP/dt, d2P/dt2 ([m][c][K][K]) computed on the host
    // and passed by value (inline_p = 1); otherwise built per workgroup from the eigen-system
    int inline_p;
    double hp[kEdgeInlineP];
    double *site_lnl;             // EDGE_LNL: [S]
    double *block_part;           // [grid][3] per-workgroup sums
    unsigned int *counter;        // last-workgroup reduction ticket (zero between launches)
    double *result;               // [3]: lnL (, dlnL/dt, d2lnL/dt2); [3]: seq (below)
    double seq;                   // != 0: written to result[3] after the sums (host polls)
};
// Lewis ascertainment-bias correction (tree_model.py:92-98, 151-156, 209-214): the last K
// patterns [first, first + K) are the dummy invariant sites.  mode 1: the reference's form,
// corr = log(1 - exp(logsumexp over (state, category) of lnl_node)), unweighted over
// categories (NaN when that sum exceeds 1, e.g. Gamma with C > 1); mode 2: the weighted
// Lewis form, corr = log(1 - sum_k exp(site_lnl[first + k])).  site_lnl[s < first] -= corr,
// *lnl -= corr * sum_w.
struct AscArgs {
    int K, C, n_tiles, mode;
    int tile_pitch;   // tiles per (category) row of the root layout
    int64_t first;
    const double *root_clv, *root_scale, *pi;
    double *site_lnl;
    double *lnl;      // total to correct (device-visible)
    double *corr;     // [1] out
    double sum_w;     // sum of the real patterns' weights
};
int launch_ascbias(hipStream_t st, const AscArgs &a);
// Device-side Newton-Raphson on one edge length (r06): one persistent launch
// runs the whole loop of pu_edge.cpp's newton() -- its safeguards, bounds and stopping rule --
// with every evaluation a grid-wide reduction, so the host pays one launch and one poll per
// optimisation instead of one per evaluation.  Each wave holds `tpw` tiles' eigen-space
// coefficients in registers (pu_edge.hip k_edge_newton).  After an evaluation every workgroup
// stores its sums into its own 64-byte slot as six 8-byte words, each a 32-bit half beside the
// evaluation's 32-bit generation (single-copy atomic: no drain, one read); workgroup 0, the
// combiner, polls every slot in parallel, adds them in a fixed order, takes newton()'s next
// step (state in its registers) and publishes the next length the same way on 8 lines, one per
// group of pollers (bounded spins: a timeout ends every workgroup and reports an error).
// Generations are monotone across launches (base), so nothing is reset between launches.
// Grid: sized to be co-resident (occupancy API with a margin).
constexpr int kNewtonState = 8;    // NewtonArgs::res doubles
constexpr unsigned kNewtonSpins = 1u << 20;  // bounded polls (a load + s_sleep each): ~1 s
struct NewtonArgs {
    double t0, tol, seq;           // start length, newton()'s tol; seq: res[7] when done
    int max_iter, tpw;             // tpw: tiles per wave
    int plain;                     // 1: an ordinary launch of the co-resident grid (not cooperative)
    int mode;                      // PU_MIN_NEWTON, PU_MIN_BRENT, PU_MIN_DBRENT (pu_minimise.h)
    double lo, hi;                 // brent / dbrent: the bracket (t0: the start, bx)
    unsigned spins;                // polls before a workgroup gives up (kNewtonSpins)
    unsigned base;                 // evaluations of earlier launches since the slots were zeroed
    uint64_t *slots;               // [grid][8]: six (half of a sum, generation) words, 2 spare
    uint64_t *pub;                 // [8][8]: two (half of the next length, 2 gen + done) words
    double *res;                   // mapped host [8]: t, lnL, d1, d2, iterations, evaluations, error, seq
    unsigned long long *timing;    // debug (PU_NT_TIMING): [evaluation][5] s_memrealtime stamps
    int n_timing;                  // rows of timing
};
// workgroups of k_edge_newton one CU holds at once for (K, C) (occupancy API); 0: unsupported
int edge_newton_per_cu(int K, int C, int tpw);
int edge_newton_tiles_per_wg(int tpw);  // tiles one workgroup holds at tpw tiles per wave
int edge_newton_max_tpw();
size_t edge_newton_sync_words(int grid);  // 8-byte words of the slots and publication lines
int launch_edge_newton(hipStream_t st, const EdgeArgs &a, const NewtonArgs &n, int grid);
size_t edge_lds_bytes(int mode, int K, int C);
// after_edge (nullable): recorded between k_edge and the reduction launch (profiling)
int launch_edge(hipStream_t st, int mode, const EdgeArgs &a, hipEvent_t after_edge = nullptr);
// stateless lnl_branch / lnl_branch_derivs (numba_likelihood_engine.py:49-79): E items;
// probs [n_p][M][K][K] (M = 1 or 3), item e uses probs[pidx ? pidx[e] : e % n_p]
int launch_lnl_branch(hipStream_t st, int K, int M, int64_t E, int n_p, const int32_t *pidx,
                      const double *probs, const double *pi, const double *pa,
                      const double *pb, const double *sa, const double *sb, double *out);

// ---- launchers (pu_kernels.hip) ----
int launch_pmatrix(hipStream_t st, const PmatArgs &a);
bool pmatrix_writes_pa(int K);  // launch_pmatrix fills PmatArgs::Pa for this K
size_t traverse_lds_bytes(int K, int C, int n_codes, int max_chunk_uses, bool coded, int n_lds);
int launch_traverse(hipStream_t st, int K, bool coded, int variant, const TraverseArgs &a,
                    int grid);
// categories combined by k_site_lse from a per-category lnl buffer (cat_lnl)
bool traverse_per_category(int K, int C);
// K = 20: the categories are combined inside the traversal (per-tile tickets)
bool traverse_lse_in_kernel(int K);
// number of per-block partial sums launch_traverse writes to block_sum
int traverse_block_sums(int K, int C, int64_t S);
int launch_reduce(hipStream_t st, const double *block_sum, int n, double *out);
// ---- several trees per launch (pu_batch, r05) ----
struct ReduceItem {  // one tree's k_reduce (no padding: pu_batch compares the bytes)
    const double *in;
    double *out;
    int64_t n;
};
// pu_batch accepts plans of these variants (lnL-only coded DNA with tip products)
bool traverse_trees_supported(int K, bool coded, int variant);
// `trees` / `items`: device arrays of n_trees argument blocks; tree t's workgroups are grid
// blocks [t * blocks, (t + 1) * blocks); lds: the largest of the trees' requests
// group > 0: groups of `group` trees, inside a group the trees' workgroups of one tile index
// adjacent; 0: tree-major
int launch_traverse_trees(hipStream_t st, int K, int variant, int waves,
                          const TraverseArgs *trees, int n_trees, int blocks, size_t lds,
                          int group);
// max_rows: the largest tree's P rows (n_sides C K; a tree's lanes past its own rows return)
int launch_pmatrix_trees(hipStream_t st, int K, const PmatArgs *trees, int n_trees,
                         int max_rows);
int launch_reduce_trees(hipStream_t st, const ReduceItem *items, int n_trees);
int launch_clv(hipStream_t st, int K, int C, int64_t S, const double *p1, const double *p2,
               const double *clv1, const double *clv2, const double *sa, const double *sb,
               double *cml, double *out);
int launch_lnl_node(hipStream_t st, int K, int C, int64_t S, const double *pi,
                    const double *partials, const double *scale, double *out);
int launch_expand_tip(hipStream_t st, int K, int C, int64_t S, int64_t cstride, bool coded,
                      int tip, const double *tips, const uint8_t *codes,
                      const double *code_table, double *out);
// tiled [cat][tile][K/2][64][2] (+ scale [cat][tile][64]) -> [S][C][K] (+ [S][C])
int launch_untile(hipStream_t st, int K, int C, int64_t S, int64_t pitch, const double *clv,
                  const double *scale, double *out, double *out_scale);
bool traverse_supported(int K);

}  // namespace pu

struct pu_ctx;
namespace pu {
// the HIP stream a context launches on (pu_group.cpp orders its RCCL all-reduce after it)
void *ctx_stream(pu_ctx *c);
}  // namespace pu
