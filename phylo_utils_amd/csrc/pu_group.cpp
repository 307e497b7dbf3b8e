// pu_group.cpp -- one process driving several GPUs (SURVEY 8(b) B2 `pu_group_create`,
// 8(e) G1 site sharding): one context per device over a contiguous range of the site
// patterns, and an RCCL communicator over the devices (ncclCommInitAll).  An evaluation
// enqueues every shard's traversal on its own stream, then all-reduces the per-device lnL
// (8 bytes) on the same streams -- the only data-path collective; the sitewise output is
// a gather of the shards' slices.  (The torch.distributed path -- one process per GPU,
// parallel.py / bench.py -- is the other way to shard; both reduce the same sums.)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/phylo_hip.h"
#include "pu_internal.h"

struct pu_group {
    int n = 0;
    std::vector<int> dev;
    std::vector<pu_ctx *> ctx;
    std::vector<int64_t> first, count;  // pattern shard of each device
    std::vector<double *> d_lnl;        // per-device lnL (all-reduced in place)
    std::vector<ncclComm_t> comm;
    int64_t S = 0;
    int K = 0;
    std::string err;
};

namespace {

int gfail(pu_group *g, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (g) g->err = buf;
    return code;
}

// a shard call failed: keep its context's message
int from_ctx(pu_group *g, int i, int rc) {
    if (rc) g->err = std::string("device ") + std::to_string(g->dev[i]) + ": " +
                     pu_last_error(g->ctx[i]);
    return rc;
}

}  // namespace

extern "C" {

int pu_group_create(pu_group **out, int n_dev, const int *devices, int n_nodes, int n_tips,
                    int64_t n_patterns, int n_cat, int n_states, int flags) {
    if (!out || n_dev < 1 || n_patterns < n_dev) return PU_E_ARG;
    *out = nullptr;
    pu_group *g = new pu_group();
    g->n = n_dev;
    g->S = n_patterns;
    g->K = n_states;
    for (int i = 0; i < n_dev; ++i) g->dev.push_back(devices ? devices[i] : i);
    // contiguous shards, sizes differing by at most one pattern
    for (int i = 0; i < n_dev; ++i) {
        g->first.push_back(n_patterns * i / n_dev);
        g->count.push_back(n_patterns * (i + 1) / n_dev - g->first.back());
    }
    g->ctx.assign(n_dev, nullptr);
    g->d_lnl.assign(n_dev, nullptr);
    int rc = PU_OK;
    for (int i = 0; i < n_dev && !rc; ++i) {
        rc = pu_ctx_create(&g->ctx[i], g->dev[i], n_nodes, n_tips, g->count[i], n_cat,
                           n_states, flags);
        if (rc) {
            gfail(g, rc, "device %d: %s", g->dev[i], pu_last_error(nullptr));
            break;
        }
        if (hipSetDevice(g->dev[i]) != hipSuccess ||
            hipMalloc(&g->d_lnl[i], sizeof(double)) != hipSuccess) {
            rc = gfail(g, PU_E_NOMEM, "device %d: lnL buffer", g->dev[i]);
            break;
        }
        rc = from_ctx(g, i, pu_set_lnl_device_output(g->ctx[i], g->d_lnl[i]));
    }
    if (!rc) {
        g->comm.assign(n_dev, nullptr);
        const ncclResult_t r = ncclCommInitAll(g->comm.data(), n_dev, g->dev.data());
        if (r != ncclSuccess) {
            g->comm.clear();
            rc = gfail(g, PU_E_COMM, "ncclCommInitAll: %s", ncclGetErrorString(r));
        }
    }
    *out = g;  // also on failure: pu_group_last_error / pu_group_destroy
    return rc;
}

void pu_group_destroy(pu_group *g) {
    if (!g) return;
    for (ncclComm_t c : g->comm)
        if (c) (void)ncclCommDestroy(c);
    for (int i = 0; i < g->n; ++i) {
        if (g->ctx[i]) pu_ctx_destroy(g->ctx[i]);
        if (g->d_lnl[i]) {
            (void)hipSetDevice(g->dev[i]);
            (void)hipFree(g->d_lnl[i]);
        }
    }
    delete g;
}

const char *pu_group_last_error(const pu_group *g) {
    return g && !g->err.empty() ? g->err.c_str() : pu_last_error(nullptr);
}

int pu_group_size(const pu_group *g) { return g ? g->n : 0; }

int pu_group_shard(const pu_group *g, int i, int64_t *first, int64_t *count) {
    if (!g || i < 0 || i >= g->n) return PU_E_ARG;
    if (first) *first = g->first[i];
    if (count) *count = g->count[i];
    return PU_OK;
}

pu_ctx *pu_group_ctx(pu_group *g, int i) {
    return g && i >= 0 && i < g->n ? g->ctx[i] : nullptr;
}

int pu_group_set_tips(pu_group *g, int n_tips, const int32_t *nodes, int n_codes,
                      const double *code_table, const uint8_t *codes, const double *partials,
                      const double *pattern_weights) {
    if (!g || (!codes == !partials)) return gfail(g, PU_E_ARG, "exactly one of codes/partials");
    for (int i = 0; i < g->n; ++i) {
        const int64_t f = g->first[i], m = g->count[i];
        // each shard's slice of every tip row, made contiguous
        std::vector<uint8_t> c8;
        std::vector<double> pd;
        if (codes) {
            c8.resize((size_t)n_tips * m);
            for (int t = 0; t < n_tips; ++t)
                std::copy(codes + (size_t)t * g->S + f, codes + (size_t)t * g->S + f + m,
                          c8.begin() + (size_t)t * m);
        } else {
            const size_t K = g->K;
            pd.resize((size_t)n_tips * m * K);
            for (int t = 0; t < n_tips; ++t)
                std::copy(partials + ((size_t)t * g->S + f) * K,
                          partials + ((size_t)t * g->S + f + m) * K,
                          pd.begin() + (size_t)t * m * K);
        }
        const int rc = pu_set_tips(g->ctx[i], n_tips, nodes, n_codes, code_table,
                                   codes ? c8.data() : nullptr, codes ? nullptr : pd.data(),
                                   pattern_weights ? pattern_weights + f : nullptr);
        if (rc) return from_ctx(g, i, rc);
    }
    return PU_OK;
}

int pu_group_set_model(pu_group *g, const double *evecs, const double *evals,
                       const double *ivecs, const double *freqs, const double *rates,
                       const double *weights) {
    if (!g) return PU_E_ARG;
    for (int i = 0; i < g->n; ++i)
        if (int rc = pu_set_model(g->ctx[i], evecs, evals, ivecs, freqs, rates, weights))
            return from_ctx(g, i, rc);
    return PU_OK;
}

int pu_group_set_schedule(pu_group *g, int n_ops, const int32_t *ops, const double *brlens,
                          int root_a, int root_b, double root_len) {
    if (!g) return PU_E_ARG;
    for (int i = 0; i < g->n; ++i)
        if (int rc = pu_set_schedule(g->ctx[i], n_ops, ops, brlens, root_a, root_b, root_len))
            return from_ctx(g, i, rc);
    return PU_OK;
}

int pu_group_set_branch_lengths(pu_group *g, const double *brlens, double root_len) {
    if (!g) return PU_E_ARG;
    for (int i = 0; i < g->n; ++i)
        if (int rc = pu_set_branch_lengths(g->ctx[i], brlens, root_len))
            return from_ctx(g, i, rc);
    return PU_OK;
}

int pu_group_set_model_p(pu_group *g, const double *freqs, const double *rates,
                         const double *weights) {
    if (!g) return PU_E_ARG;
    for (int i = 0; i < g->n; ++i)
        if (int rc = pu_set_model_p(g->ctx[i], freqs, rates, weights)) return from_ctx(g, i, rc);
    return PU_OK;
}

int pu_group_set_pmatrices(pu_group *g, const double *P) {
    if (!g) return PU_E_ARG;
    for (int i = 0; i < g->n; ++i)
        if (int rc = pu_set_pmatrices(g->ctx[i], P)) return from_ctx(g, i, rc);
    return PU_OK;
}

int pu_group_run(pu_group *g, double *lnl_out, double *sitewise_out) {
    if (!g || g->comm.empty()) return gfail(g, PU_E_STATE, "group not initialised");
    for (int i = 0; i < g->n; ++i)
        if (int rc = pu_enqueue(g->ctx[i])) return from_ctx(g, i, rc);
    // sum of the shards' lnL, stream-ordered after each traversal
    ncclResult_t r = ncclGroupStart();
    for (int i = 0; i < g->n && r == ncclSuccess; ++i)
        r = ncclAllReduce(g->d_lnl[i], g->d_lnl[i], 1, ncclFloat64, ncclSum, g->comm[i],
                          (hipStream_t)pu::ctx_stream(g->ctx[i]));
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
        return gfail(g, PU_E_COMM, "ncclAllReduce: %s",
                     ncclGetErrorString(r != ncclSuccess ? r : r2));
    for (int i = 0; i < g->n; ++i) {
        double v = 0.0;
        if (int rc = pu_synchronize(g->ctx[i], &v)) return from_ctx(g, i, rc);
        if (i == 0 && lnl_out) *lnl_out = v;
        if (sitewise_out)
            if (int rc = pu_get_site_lnl(g->ctx[i], sitewise_out + g->first[i]))
                return from_ctx(g, i, rc);
    }
    return PU_OK;
}

}  // extern "C"
