// pu_ctx.h -- the device context behind the C ABI and the helpers every C-ABI translation
// unit shares (pu_capi.cpp: contexts, planner, traversal; pu_edge.cpp: edge likelihoods,
// derivatives and branch-length optimisation).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/phylo_hip.h"
#include "pu_internal.h"

namespace pu {

// process-wide last error (pu_last_error(NULL)); defined in pu_capi.cpp
extern thread_local std::string g_err;

inline int set_err(std::string *dst, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    if (dst) *dst = buf;
    return code;
}

#define HIPCHK(ctxerr, expr)                                                              \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return pu::set_err(ctxerr, PU_E_HIP, "%s: %s (%s:%d)", #expr,                \
                               hipGetErrorString(e_), __FILE__, __LINE__);                \
    } while (0)

template <class T>
int dalloc(std::string *err, T **p, size_t n) {
    *p = nullptr;
    if (n == 0) return PU_OK;
    hipError_t e = hipMalloc((void **)p, n * sizeof(T));
    if (e != hipSuccess) {
        *p = nullptr;
        (void)hipGetLastError();
        return set_err(err, PU_E_NOMEM, "hipMalloc of %zu bytes failed: %s", n * sizeof(T),
                       hipGetErrorString(e));
    }
    return PU_OK;
}

template <class T>
void dfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// coded tips, code table and pattern weights held by several contexts (pu_share_tips): freed
// with the last context that holds them
struct TipStore {
    int device = 0;
    const void *first = nullptr;  // the context that uploaded them
    uint8_t *codes = nullptr;
    double *table = nullptr, *pattern_w = nullptr;
    ~TipStore() {
        DeviceGuard g(device);
        dfree(codes);
        dfree(table);
        dfree(pattern_w);
    }
};

}  // namespace pu

struct pu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int n_nodes = 0, n_tips = 0, C = 0, K = 0, flags = 0;
    int64_t S = 0;
    std::string err;

    // tips
    std::vector<int> tip_slot;      // node -> tip slot (-1: not a tip)
    std::vector<int> tip_kind;      // slot -> 0 unset, 1 dense, 2 coded
    std::vector<uint8_t> h_codes;   // host copy of coded tips [n_tips][S]
    std::vector<double> h_table;    // [n_codes][K]
    int n_codes = 0, n_tips_used = 0;
    int64_t code_stride = 0;        // device row stride of coded tips (S rounded up to 64)
    bool dense_dirty = false;
    double *d_tips = nullptr;
    uint8_t *d_codes = nullptr;
    double *d_table = nullptr;
    // set once the coded tips are shared (pu_share_tips): d_codes, d_table and d_pattern_w
    // then alias the store's buffers and are frozen
    std::shared_ptr<pu::TipStore> tip_store;

    // model
    bool have_model = false;
    // host-supplied transition matrices (pu_set_pmatrices): k_pmatrix is skipped; p_fresh
    // turns false when branch lengths or the schedule change
    bool host_p = false, p_fresh = false;
    pu_pmat_provider pm_fn = nullptr;  // host matrices for edge operations (host_p only)
    void *pm_user = nullptr;
    std::vector<double> h_eig;         // host copy of evecs [K*K], evals [K], ivecs [K*K]
    std::vector<double> h_rates;       // host copy of the category rates [C]
    std::vector<double> h_brlens;      // device-order branch lengths [2 (n_ops + 1)]
    bool lengths_dirty = false;        // up_len moved past h_brlens / d_brlens (pu_optimise_edge)
    double *d_edge_pm = nullptr;       // provider matrices of one edge launch
    double *d_evecs = nullptr, *d_evals = nullptr, *d_ivecs = nullptr, *d_pi = nullptr,
           *d_rates = nullptr, *d_logw = nullptr;

    // schedule
    bool have_sched = false;
    int n_ops = 0, n_store = 0, grid = 0, n_tiles = 0, variant = 0, n_mem = 0, n_lds = 0;
    int lds_pad = 0, waves = 0, n_cu = 256;
    int n_store_ops = 0, n_tip_uses = 0;  // ops that write their parent; tip children (plan)
    std::vector<char> swap;       // device op: children exchanged w.r.t. the caller's op
    // tip uses in schedule order, grouped by staging chunk (pu_internal.h kChunkOps)
    int n_chunks = 0, max_chunk_uses = 0;
    int chunk_cap = 0;  // tip uses per staging chunk (0: kChunkUses), set with the schedule
    int *d_chunk_op0 = nullptr, *d_chunk_tip0 = nullptr, *d_tip_seq = nullptr;
    // split plan (K = 20): n_tasks chain tasks + the top task, {op_lo, op_hi, chunk_lo,
    // chunk_hi} each; 0: one whole-tree launch
    int n_tasks = 0;
    int *d_tasks = nullptr;
    int *d_ticket = nullptr;  // [n_tiles * C] top-task election, zero between launches
    uint32_t *d_sflag = nullptr;  // [clv_cap + 1][C * n_tiles] scaler dirty flags
    double *d_cat_lnl = nullptr;  // [C][n_tiles * 64] when 4 % C != 0
    int *d_lse_ticket = nullptr;  // K = 20: [n_tiles] category-combine election, zero between launches
    // the last arriver of each launch re-zeroes its ticket; a launch that failed or did not
    // complete leaves counters off by k, so the next pu_enqueue re-zeroes both ticket arrays
    bool tickets_dirty = false;
    std::vector<int> perm;        // device op -> caller op
    std::vector<int> store_slot;  // node -> storage slot (-1: not stored)
    std::vector<int32_t> ops_in;  // caller ops (par,c1,c2)
    int root_a = -1, root_b = -1;
    pu::OpDesc *d_ops = nullptr;
    double *d_brlens = nullptr, *d_P = nullptr;
    double *d_Pa = nullptr;  // K = 20: P as MFMA A operands
    double *d_PT = nullptr;  // K <= 4 lnL-only coded: tip products (TV_PTIP)
    size_t pt_cap = 0;       // doubles allocated
    unsigned long long *d_timing = nullptr;  // debug: PU_TIMING
    int n_timed = 0;
    // layout (r05): tiles per layout row = tile_pitch(S) + pitch_extra (PU_PITCH_EXTRA, an A/B
    // knob latched with the schedule, at most pitch_pad - 1); buffers are allocated for
    // tile_pitch(S) + pitch_pad tiles per row, pitch_pad = kPitchPad only when the knob is set
    // at pu_ctx_create, else 0
    int pitch_extra = 0, pitch_pad = 0;

    // partials / outputs
    double *d_clv = nullptr, *d_scale = nullptr;
    size_t clv_cap = 0;  // slots allocated
    double *d_root = nullptr, *d_root_scale = nullptr, *d_site_lnl = nullptr,
           *d_pattern_w = nullptr, *d_block = nullptr, *d_lnl = nullptr;
    int block_cap = 0;
    uint64_t *d_red_slots = nullptr;  // TraverseArgs::red_slots (r06), 2 words per block sum
    int red_cap = 0;                  // block sums the slots hold
    unsigned red_gen = 0;             // the last launch's generation (monotone; 0: zeroed)
    double *h_lnl = nullptr;  // pinned
    bool ran = false;
    bool root_stale = false;  // last run by pu_batch, which does not write the root partials

    hipStream_t own_stream = nullptr;
    double *d_lnl_ext = nullptr;  // caller's device output for the lnL
    // the last evaluation was a pu_batch_enqueue into the caller's lnl_dev: this tree's entry
    const double *lnl_batch = nullptr;

    // edge operations (pu_edge.cpp): the unrooted topology of the schedule -- parent[v] is
    // v's neighbour towards the root edge (the two root-edge ends point at each other) and
    // up_len[v] the length of that edge (Traversal.brlens, traversal.py:24-25,
    // utils.py:202-213)
    std::vector<int> parent;
    std::vector<double> up_len;
    double *d_edge_part = nullptr;      // [n_tiles][3] per-workgroup sums
    unsigned int *d_edge_ctr = nullptr; // last-workgroup ticket
    double *d_edge_res = nullptr;       // [3]
    double *h_edge_res = nullptr;       // pinned, mapped [4]: 3 sums + sequence number
    // EDGE_DERIV partials written straight into pinned mapped host memory and summed by the
    // host (no k_edge_sum launch): two buffers [3 * edge_tiles], sentinel-filled when free
    double *h_edge_part[2] = {nullptr, nullptr};
    double *d_edge_part_host[2] = {nullptr, nullptr};  // their device addresses
    int edge_part_buf = 0;
    double edge_seq = 0.0;              // last sequence number handed to k_edge_sum
    double *d_edge_res_host = nullptr;  // its device address (the kernels write the sums)
    int edge_tiles = 0;
    // device-side Newton (k_edge_newton): tickets + generation word, the step state, the
    // result in mapped host memory; nt_per_cu: co-resident workgroups per CU (-1: not asked)
    uint64_t *d_nt_slots = nullptr;  // k_edge_newton's slots and publication lines
    size_t nt_slots_cap = 0;
    double *h_nt_res = nullptr, *d_nt_res_host = nullptr;
    double nt_seq = 0.0;
    int nt_per_cu_t[3] = {-1, -1, -1}, nt_launches = 0, nt_evals = 0, nt_timeouts = 0;
    // the tickets and the generation word run on across launches (zeroed when nt_fresh is off:
    // first use, another grid, a failed launch, or far along)
    unsigned nt_base = 0;
    int nt_grid = 0;
    bool nt_fresh = false;
    std::vector<hipEvent_t> edge_ev;  // profiling: event pairs around edge reductions
    int n_edge_prof = 0;

    // Lewis ascertainment-bias correction (tree_model.py:92-98, 151-156, 209-214): mode 0 off,
    // 1 the reference's form, 2 weighted; the dummy invariant sites are [asc_first, S)
    int asc_mode = 0;
    int64_t asc_first = 0;
    double *d_asc_corr = nullptr;
    std::vector<double> h_pattern_w;  // host copy of the pattern weights

    // profiling: event triples per recorded run
    bool profile = false;
    std::vector<hipEvent_t> ev;
    int n_prof = 0;
};

namespace pu {
// tiles per layout row of a context's tiled CLV / scaler / root buffers
inline int64_t ctx_pitch(const pu_ctx *c) { return tile_pitch(c->S) + c->pitch_extra; }
// shared by the C-ABI translation units (pu_capi.cpp)
int check_ready(pu_ctx *c);
// one traversal launch of a context, prepared (pu_enqueue, pu_batch_enqueue): checks, provider
// refresh, tip sync, tip-product buffer, then the P and traversal arguments
struct LaunchPlan {
    PmatArgs pa;
    TraverseArgs a;
    int variant = 0;
    bool coded = true;
    size_t lds = 0;
    double *lnl_dst = nullptr;  // where the lnL lands (the caller's device output or d_lnl)
};
int prepare_launch(pu_ctx *c, LaunchPlan &L);
int flush_lengths(pu_ctx *c);  // pu_edge.cpp: upload up_len when pu_optimise_edge moved it
bool any_dense(const pu_ctx *c);
int sync_tips(pu_ctx *c);
int check_device(int device);
// host_p contexts with a provider: matrices d^order/dt^order P(t[i] r) for n lengths into out
int provide(pu_ctx *c, int order, int n, const double *t, double *out);
// host_p contexts: regenerate the traversal's P from the provider when the lengths moved
int refresh_host_p(pu_ctx *c);
// host_p contexts: the plain-P buffer (not allocated for the protein eigen path)
int ensure_host_p(pu_ctx *c);
// pu_edge.cpp: release the edge-operation buffers of a context
void edge_free(pu_ctx *c);
// enqueue the ascertainment-bias correction of site_lnl and *lnl (no-op when off)
int enqueue_ascbias(pu_ctx *c, double *lnl);
// stateless seam calls (pu_clv, pu_lnl_node, pu_lnl_branch*): one scratch buffer and stream
// per device, guarded by ws_mutex(device)
std::mutex &ws_mutex(int device);
int ws_get(int device, size_t doubles, double **out, hipStream_t *st);
}  // namespace pu
