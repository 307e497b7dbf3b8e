// pu_batch.cpp -- several trees' lnL in one launch of each kernel (r05, SURVEY 8(e) G2:
// "batch several trees per launch if a single tree underfills the GPU").  The workload is
// BASELINE cfg5's: many candidate / bootstrap trees on one alignment, i.e. the reference's
// set_tree + compute_partials + likelihood loop over trees (tree_model.py:87-89, 160-176).
// Every tree keeps its own context (schedule, branch lengths, P, buffers); a batch launches
// one k_pmatrix_lane_trees (every tree's P and tip products), one k_prune_trees (tree t's
// workgroups are grid blocks [t * blocks, (t + 1) * blocks), each exactly k_prune's work for
// that tree) and one k_reduce_trees (tree t's block sums in k_reduce's order), so each lnL is
// bitwise the one pu_enqueue gives.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "pu_ctx.h"

struct pu_batch {
    int device = 0;
    std::vector<pu_ctx *> ctx;
    hipStream_t stream = nullptr, own_stream = nullptr;
    pu::TraverseArgs *d_t = nullptr;
    pu::PmatArgs *d_p = nullptr;
    pu::ReduceItem *d_r = nullptr;
    std::vector<pu::TraverseArgs> h_t;
    std::vector<pu::PmatArgs> h_p;
    std::vector<pu::ReduceItem> h_r;
    bool uploaded = false, uploaded_dbg = false;
    std::vector<hipEvent_t> ev;  // joins of context streams other than the batch's
    hipEvent_t done = nullptr;   // ... and of the batch's launches back into those streams
    // profiling (pu_batch_profile): 4 events per enqueue -- before P, around the traversal,
    // after the reduction
    bool profile = false;
    int n_prof = 0;
    std::vector<hipEvent_t> pev;
    std::string err;
};

namespace {
constexpr int kMaxBatchProf = 4096;
}

using pu::set_err;

namespace {

template <class T>
bool same_bytes(const std::vector<T> &a, const std::vector<T> &b) {
    return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(T)) == 0;
}

}  // namespace

extern "C" {

int pu_batch_create(pu_batch **out, int n, pu_ctx *const *ctxs) {
    if (!out || n < 1 || !ctxs) return set_err(nullptr, PU_E_ARG, "pu_batch_create: bad arguments");
    *out = nullptr;
    for (int i = 0; i < n; ++i)
        if (!ctxs[i]) return set_err(nullptr, PU_E_ARG, "pu_batch_create: context %d is null", i);
    const int dev = ctxs[0]->device;
    for (int i = 1; i < n; ++i)
        if (ctxs[i]->device != dev)
            return set_err(nullptr, PU_E_ARG, "pu_batch_create: contexts on devices %d and %d",
                           dev, ctxs[i]->device);
    pu_batch *b = new pu_batch;
    b->device = dev;
    b->ctx.assign(ctxs, ctxs + n);
    pu::DeviceGuard g(dev);
    int rc;
    if (hipStreamCreateWithFlags(&b->own_stream, hipStreamNonBlocking) != hipSuccess ||
        (rc = pu::dalloc(&b->err, &b->d_t, (size_t)n)) ||
        (rc = pu::dalloc(&b->err, &b->d_p, (size_t)n)) ||
        (rc = pu::dalloc(&b->err, &b->d_r, (size_t)n))) {
        pu_batch_destroy(b);
        return set_err(nullptr, PU_E_NOMEM, "pu_batch_create: device allocation failed");
    }
    b->stream = b->own_stream;
    *out = b;
    return PU_OK;
}

void pu_batch_destroy(pu_batch *b) {
    if (!b) return;
    pu::DeviceGuard g(b->device);
    if (b->stream) (void)hipStreamSynchronize(b->stream);
    pu::dfree(b->d_t);
    pu::dfree(b->d_p);
    pu::dfree(b->d_r);
    for (hipEvent_t e : b->ev) (void)hipEventDestroy(e);
    if (b->done) (void)hipEventDestroy(b->done);
    for (hipEvent_t e : b->pev) (void)hipEventDestroy(e);
    if (b->own_stream) (void)hipStreamDestroy(b->own_stream);
    delete b;
}

const char *pu_batch_last_error(const pu_batch *b) { return b ? b->err.c_str() : ""; }

int pu_batch_set_stream(pu_batch *b, void *st) {
    if (!b) return set_err(nullptr, PU_E_ARG, "null batch");
    pu::DeviceGuard g(b->device);
    HIPCHK(&b->err, hipStreamSynchronize(b->stream));
    b->stream = st == PU_OWN_STREAM ? b->own_stream : (hipStream_t)st;
    return PU_OK;
}

int pu_batch_enqueue(pu_batch *b, double *lnl_dev) {
    if (!b) return set_err(nullptr, PU_E_ARG, "null batch");
    pu::DeviceGuard g(b->device);
    const int n = (int)b->ctx.size();
    std::vector<pu::LaunchPlan> L(n);
    for (int i = 0; i < n; ++i)
        if (int rc = pu::prepare_launch(b->ctx[i], L[i]))
            return set_err(&b->err, rc, "tree %d: %s", i, b->ctx[i]->err.c_str());
    // one kernel build for every tree: same shape, the lnL-only tip-product plans.  A tree
    // whose plan reads parents back from HBM needs the read-back build (TV_GENERIC); the
    // others run it too (same arithmetic, bitwise: test_kernel_builds_and_plans_bitwise_equal)
    const pu_ctx *c0 = b->ctx[0];
    size_t lds = 0;
    int max_rows = 0;  // the largest tree's P rows (k_pmatrix_lane_trees)
    int variant = 0;
    for (int i = 0; i < n; ++i) variant |= L[i].variant;
    for (int i = 0; i < n; ++i) {
        const pu_ctx *c = b->ctx[i];
        const pu::LaunchPlan &l = L[i];
        if (c->K != c0->K || c->C != c0->C || c->S != c0->S || c->grid != c0->grid ||
            (l.variant | pu::TV_GENERIC) != (variant | pu::TV_GENERIC) || l.coded != L[0].coded)
            return set_err(&b->err, PU_E_ARG,
                           "tree %d: K %d C %d S %lld grid %d variant %d differ from tree 0's "
                           "(K %d C %d S %lld grid %d variant %d)", i, c->K, c->C,
                           (long long)c->S, c->grid, l.variant, c0->K, c0->C, (long long)c0->S,
                           c0->grid, L[0].variant);
        if (!(c->flags & PU_LNL_ONLY) || c->host_p || c->asc_mode ||
            !pu::traverse_trees_supported(c->K, l.coded, variant))
            return set_err(&b->err, PU_E_ARG,
                           "tree %d: a batch takes lnL-only DNA contexts with coded tips, the "
                           "model's eigen-system on the device and no ascertainment correction "
                           "(variant %d)", i, l.variant);
        // a category count that does not divide 4 leaves the categories to a separate
        // k_site_lse launch per tree (launch_traverse), which the batch does not have
        if (pu::traverse_per_category(c->K, c->C))
            return set_err(&b->err, PU_E_ARG,
                           "tree %d: a batch takes C = 1, 2 or 4 rate categories (C = %d: use "
                           "pu_enqueue per context)", i, c->C);
        lds = std::max(lds, l.lds + (size_t)l.a.lds_pad);
        max_rows = std::max(max_rows, l.pa.n_sides * l.pa.C * l.pa.K);
    }
    if (lds > 160 * 1024)
        return set_err(&b->err, PU_E_ARG, "LDS request %zu exceeds 160 KiB", lds);
    std::vector<pu::TraverseArgs> ht(n);
    std::vector<pu::PmatArgs> hp(n);
    std::vector<pu::ReduceItem> hr(n);
    const int n_block = pu::traverse_block_sums(c0->K, c0->C, c0->S);
    const bool skip_root = !(getenv("PU_BATCH_ROOT") && atoi(getenv("PU_BATCH_ROOT")) == 1);
    for (int i = 0; i < n; ++i) {
        ht[i] = L[i].a;
        // the root partials are not written by a batch (pu_get_root refuses until the
        // context's next pu_enqueue / pu_run); PU_BATCH_ROOT=1 writes them (the r06 A/B)
        if (skip_root) {
            ht[i].root_clv = nullptr;
            ht[i].root_scale = nullptr;
            ht[i].root_bytes = ht[i].root_scale_bytes = 0;
        }
        hp[i] = L[i].pa;
        hr[i] = pu::ReduceItem{L[i].a.block_sum, lnl_dev ? lnl_dev + i : L[i].lnl_dst, n_block};
    }
    // the argument blocks change only with a context's schedule, tips or output: uploaded
    // then, after the batch's earlier launches that read them
    if (!b->uploaded || !same_bytes(ht, b->h_t) || !same_bytes(hp, b->h_p) ||
        !same_bytes(hr, b->h_r)) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        HIPCHK(&b->err, hipStreamIsCapturing(b->stream, &cs));
        if (cs != hipStreamCaptureStatusNone)
            return set_err(&b->err, PU_E_STATE,
                           "pu_batch_enqueue: arguments changed during stream capture (enqueue "
                           "once before capturing)");
        HIPCHK(&b->err, hipStreamSynchronize(b->stream));
        HIPCHK(&b->err, hipMemcpy(b->d_t, ht.data(), n * sizeof(ht[0]), hipMemcpyHostToDevice));
        HIPCHK(&b->err, hipMemcpy(b->d_p, hp.data(), n * sizeof(hp[0]), hipMemcpyHostToDevice));
        HIPCHK(&b->err, hipMemcpy(b->d_r, hr.data(), n * sizeof(hr[0]), hipMemcpyHostToDevice));
        b->h_t.swap(ht);
        b->h_p.swap(hp);
        b->h_r.swap(hr);
        b->uploaded = true;
    }
    // work a context queued on its own stream (tip or length uploads) comes first
    std::vector<hipStream_t> others;
    for (const pu_ctx *c : b->ctx)
        if (c->stream != b->stream &&
            std::find(others.begin(), others.end(), c->stream) == others.end())
            others.push_back(c->stream);
    while (b->ev.size() < others.size()) {
        hipEvent_t e;
        HIPCHK(&b->err, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        b->ev.push_back(e);
    }
    for (size_t k = 0; k < others.size(); ++k) {
        HIPCHK(&b->err, hipEventRecord(b->ev[k], others[k]));
        HIPCHK(&b->err, hipStreamWaitEvent(b->stream, b->ev[k], 0));
    }
    hipEvent_t *evs = nullptr;
    if (b->profile && b->n_prof < kMaxBatchProf) {
        while (b->pev.size() < 4 * (size_t)(b->n_prof + 1)) {
            hipEvent_t e;
            HIPCHK(&b->err, hipEventCreate(&e));
            b->pev.push_back(e);
        }
        evs = &b->pev[4 * (size_t)b->n_prof++];
    }
    if (evs) HIPCHK(&b->err, hipEventRecord(evs[0], b->stream));
    HIPCHK(&b->err, (hipError_t)pu::launch_pmatrix_trees(b->stream, c0->K, b->d_p, n, max_rows));
    if (evs) HIPCHK(&b->err, hipEventRecord(evs[1], b->stream));
    // the 7-wave build when the batch needs more than one dispatch round of the default
    // build's 6 workgroups per CU (as pick_waves decides for one launch): cfg5's 125 trees 442
    // vs 351 G updates/s (profiles/r05_batch_ab/), one tree alone 0.088 vs 0.078 ms
    int waves = (int64_t)n * c0->grid > 6 * (int64_t)c0->n_cu ? 7 : 1;
    if (const char *wv = getenv("PU_BATCH_WAVES")) waves = atoi(wv) == 7 ? 7 : 1;  // A/B
    if (getenv("PU_DEBUG_PLAN") && !b->uploaded_dbg) {
        b->uploaded_dbg = true;
        size_t lmin = L[0].lds, lmax = 0;
        for (int i = 0; i < n; ++i) lmin = std::min(lmin, L[i].lds), lmax = std::max(lmax, L[i].lds);
        fprintf(stderr, "[pu batch] %d trees, %d blocks each, variant %d, LDS %zu..%zu -> %zu, "
                "waves %d\n", n, c0->grid, variant, lmin, lmax, lds, waves);
    }
    // groups of 24 trees, the group's workgroups of one tile index adjacent: the dispatcher's
    // round-robin over the 8 XCDs keeps a tree on one XCD, three trees per XCD at a time, and
    // the workgroups a CU holds belong to different trees (not in lockstep).  cfg5 bench,
    // same box (profiles/r05_batch_ab/exp25_groups.txt, exp27_group_sweep.txt): tree-major
    // 442 G updates/s, groups of 8 / 16 / 20 / 24 / 28 / 40 502 / 507-512 / 511 / 515-518 /
    // 508-511 / 521-523, but 32 455-461 and 48 486 -- sizes whose workgroups of one tree land
    // on the same CUs.  r06, with one shared alignment (profiles/r06_cfg5_groups.txt, two
    // rounds): 16 / 24 / 32 / 40 / 48 / 64 -> 526 / 534 / 486-489 / 544-545 / 504-506 / 436 G,
    // so 40 (24 before).  Without the root-partial stores (r06, scripts/r06/call43.sh, two
    // rounds): 24 / 40 / 56 / 72 / tree-major -> 541-542 / 551 / 556 / 454 / 454 G, so 56.
    // PU_BATCH_GROUP=g for the A/B (0: tree-major)
    int group = 56;
    if (const char *gv = getenv("PU_BATCH_GROUP")) group = std::max(0, atoi(gv));
    HIPCHK(&b->err, (hipError_t)pu::launch_traverse_trees(b->stream, c0->K, variant, waves,
                                                           b->d_t, n, c0->grid, lds, group));
    if (evs) HIPCHK(&b->err, hipEventRecord(evs[2], b->stream));
    HIPCHK(&b->err, (hipError_t)pu::launch_reduce_trees(b->stream, b->d_r, n));
    if (evs) HIPCHK(&b->err, hipEventRecord(evs[3], b->stream));
    for (int i = 0; i < n; ++i) {
        pu_ctx *c = b->ctx[i];
        if (!lnl_dev && !c->d_lnl_ext)  // pu_synchronize(ctx, &lnl) after pu_batch_synchronize
            HIPCHK(&b->err, hipMemcpyAsync(c->h_lnl, c->d_lnl, sizeof(double),
                                           hipMemcpyDeviceToHost, b->stream));
        c->lnl_batch = lnl_dev ? lnl_dev + i : nullptr;
        c->ran = true;
        c->root_stale = skip_root;
    }
    // and the batch's launches (which read and write each context's lengths, P, block sums,
    // sitewise lnL and lnL) come before anything queued on a context's own stream from here
    // on: length updates, pu_enqueue, pu_get_site_lnl
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIPCHK(&b->err, hipStreamIsCapturing(b->stream, &cap));
    if (!others.empty() && cap == hipStreamCaptureStatusNone) {  // (a capture joins itself)
        if (!b->done) HIPCHK(&b->err, hipEventCreateWithFlags(&b->done, hipEventDisableTiming));
        HIPCHK(&b->err, hipEventRecord(b->done, b->stream));
        for (hipStream_t st : others) HIPCHK(&b->err, hipStreamWaitEvent(st, b->done, 0));
    }
    return PU_OK;
}

int pu_batch_profile(pu_batch *b, int on) {
    if (!b) return set_err(nullptr, PU_E_ARG, "null batch");
    pu::DeviceGuard g(b->device);
    HIPCHK(&b->err, hipStreamSynchronize(b->stream));
    b->profile = on != 0;
    b->n_prof = 0;
    return PU_OK;
}

int pu_batch_kernel_times(pu_batch *b, double *trav, double *total, int cap, int *n) {
    if (!b || cap < 0 || (cap > 0 && (!trav || !total)))
        return set_err(b ? &b->err : nullptr, PU_E_ARG, "bad arguments");
    pu::DeviceGuard g(b->device);
    const int k = std::min(cap, b->n_prof);
    for (int i = 0; i < k; ++i) {
        hipEvent_t *e = &b->pev[4 * (size_t)i];
        HIPCHK(&b->err, hipEventSynchronize(e[3]));
        float t_tr = 0.f, t_all = 0.f;
        HIPCHK(&b->err, hipEventElapsedTime(&t_tr, e[1], e[2]));
        HIPCHK(&b->err, hipEventElapsedTime(&t_all, e[0], e[3]));
        trav[i] = t_tr;
        total[i] = t_all;
    }
    if (n) *n = k;
    return PU_OK;
}

int pu_batch_synchronize(pu_batch *b) {
    if (!b) return set_err(nullptr, PU_E_ARG, "null batch");
    pu::DeviceGuard g(b->device);
    HIPCHK(&b->err, hipStreamSynchronize(b->stream));
    return PU_OK;
}

}  // extern "C"
