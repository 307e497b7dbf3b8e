// pu_edge.cpp -- C ABI of the edge operations (include/phylo_hip.h):
//   pu_edge_lnl          compute_partials_at_edge + compute_likelihood_at_edge on any edge
//                        (phylo_utils/tree_model.py:178-217)
//   pu_edge_derivs       lnL and d/dt, d2/dt2 of the edge length (lnl_branch_derivs,
//                        likelihood/numba_likelihood_engine.py:49-57, over the rate mixture)
//   pu_update_partials   in-place clv updates (numba_likelihood_engine.py:35-44) on any nodes
//   pu_optimise_edge     Newton-Raphson on one edge length, every evaluation on the GPU
//   pu_optimise_sweep    the optimising traversal (utils.py:137-188, Traversal
//                        .optimising_traversal traversal.py:29,34-35): re-orient, optimise
//                        each edge in turn, restore -- one pass over the 2N-3 edges
//   pu_lnl_branch[_derivs]  the stateless numba gufuncs (numba_likelihood_engine.py:49-79)
#include <math.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>

#include "pu_ctx.h"
#include "pu_minimise.h"

using namespace pu;

namespace {

// MIN_BRANCH_LENGTH of the reference is 2^-16 (substitution_models/abstract.py:8, unused
// there); the optimiser bounds lengths to [kMinLen, kMaxLen]
constexpr double kMinLen = 1e-8;
constexpr double kMaxLen = 100.0;

int node_src(pu_ctx *c, int node, NodeSrc *out) {
    if (node < 0 || node >= c->n_nodes)
        return set_err(&c->err, PU_E_ARG, "node %d out of range [0,%d)", node, c->n_nodes);
    const int t = c->tip_slot[node];
    if (t >= 0) {
        if (c->tip_kind[t] == 0) return set_err(&c->err, PU_E_STATE, "tip %d has no data", node);
        out->kind = any_dense(c) ? SRC_DENSE : SRC_CODED;
        out->idx = t;
        return PU_OK;
    }
    if (c->flags & PU_LNL_ONLY)
        return set_err(&c->err, PU_E_STATE, "edge operations on internal node %d need "
                       "PU_KEEP_PARTIALS (PU_LNL_ONLY reuses CLV storage)", node);
    if (!c->ran) return set_err(&c->err, PU_E_STATE, "pu_run first");
    const int s = c->store_slot[node];
    if (s < 0) return set_err(&c->err, PU_E_ARG, "node %d is not in the schedule", node);
    out->kind = SRC_SLOT;
    out->idx = s;
    return PU_OK;
}

// the edge (u, v) of the current topology -- BranchLengths lookup (utils.py:191-199)
int edge_of(pu_ctx *c, int u, int v, int *key) {
    if (u >= 0 && u < c->n_nodes && v >= 0 && v < c->n_nodes && u != v) {
        if (c->parent[u] == v) return *key = u, PU_OK;
        if (c->parent[v] == u) return *key = v, PU_OK;
    }
    // tree_model.py:184-187
    return set_err(&c->err, PU_E_ARG, "There is no edge connecting nodes %d and %d", u, v);
}

void set_len(pu_ctx *c, int key, double len) {
    c->up_len[key] = len;
    const int p = c->parent[key];
    if (p >= 0 && c->parent[p] == key) c->up_len[p] = len;  // the root edge is stored twice
}

// The PU_EDGE_* switches are read at every evaluation (a getenv is ~0.1 us against ~25 us),
// so a test can compare the paths in one process
int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    return v ? atoi(v) : dflt;
}

// Host-summed partials: a free slot holds this NaN payload (the device never produces it:
// its NaNs are the canonical quiet NaN); k_edge overwrites every slot of its launch
constexpr uint64_t kPartSentinel = 0x7ff4deadbeef0000ull;

void fill_sentinel(double *h, size_t n) {
    uint64_t *u = reinterpret_cast<uint64_t *>(h);
    for (size_t i = 0; i < n; ++i) u[i] = kPartSentinel;
}

int prepare(pu_ctx *c) {
    int rc = check_ready(c);
    if (rc) return rc;
    if (!c->ran) return set_err(&c->err, PU_E_STATE, "pu_run first");
    // the edge kernels build P, dP/dt and d2P/dt2 from the eigen-decomposition per workgroup,
    // or take them from the host's provider (non-reversible models on host matrices)
    if (c->host_p && !c->pm_fn)
        return set_err(&c->err, PU_E_STATE, "edge operations on host transition matrices need "
                       "pu_set_pmatrix_provider (or an eigen-decomposed model, pu_set_model)");
    if (c->host_p && !c->d_edge_pm) {
        const size_t n = (size_t)std::max(4, 2 * kEdgeOpsPerLaunch) * c->C * c->K * c->K;
        if ((rc = dalloc(&c->err, &c->d_edge_pm, n))) return rc;
    }
    if ((rc = sync_tips(c))) return rc;
    if (c->edge_tiles < c->n_tiles) {
        dfree(c->d_edge_part);
        if ((rc = dalloc(&c->err, &c->d_edge_part, 3 * (size_t)c->n_tiles))) return rc;
        for (int b = 0; b < 2; ++b) {
            double *&h = c->h_edge_part[b];
            if (h) (void)hipHostFree(h);
            h = nullptr;
            HIPCHK(&c->err, hipHostMalloc((void **)&h, 3 * (size_t)c->n_tiles * sizeof(double),
                                          hipHostMallocMapped));
            HIPCHK(&c->err, hipHostGetDevicePointer((void **)&c->d_edge_part_host[b], h, 0));
            fill_sentinel(h, 3 * (size_t)c->n_tiles);
        }
        c->edge_tiles = c->n_tiles;
    }
    if (!c->d_edge_ctr) {
        if ((rc = dalloc(&c->err, &c->d_edge_ctr, 1)) ||
            (rc = dalloc(&c->err, &c->d_edge_res, 3)))
            return rc;
        HIPCHK(&c->err, hipMemset(c->d_edge_ctr, 0, sizeof(unsigned int)));
        HIPCHK(&c->err, hipHostMalloc((void **)&c->h_edge_res, 4 * sizeof(double),
                                      hipHostMallocMapped));
        c->h_edge_res[3] = 0.0;
        HIPCHK(&c->err, hipHostGetDevicePointer((void **)&c->d_edge_res_host, c->h_edge_res, 0));
    }
    return PU_OK;
}

void fill_args(const pu_ctx *c, EdgeArgs &a) {
    memset(&a, 0, sizeof a);
    const size_t padS = (size_t)ctx_pitch(c) * kTile;  // layout rows
    a.K = c->K;
    a.C = c->C;
    a.n_tiles = c->n_tiles;
    a.tile_pitch = (int)ctx_pitch(c);
    a.S = c->S;
    a.code_stride = c->code_stride;
    a.codes = c->d_codes;
    a.table = c->d_table;
    a.tips = c->d_tips;
    a.clv = c->d_clv;
    a.scale = c->d_scale;
    a.root_clv = c->d_root;
    a.root_scale = c->d_root_scale;
    a.slot_stride = padS * c->C * c->K;
    a.sstride = padS * c->C;
    a.sflag = c->d_sflag;
    a.n_store = (int)c->clv_cap;
    a.evecs = c->d_evecs;
    a.evals = c->d_evals;
    a.ivecs = c->d_ivecs;
    a.rates = c->d_rates;
    a.pi = c->d_pi;
    a.logw = c->d_logw;
    a.weights = c->d_logw + c->C;  // d_logw = [log w][w]
    a.pattern_w = c->d_pattern_w;
    a.site_lnl = c->d_site_lnl;
    a.block_part = c->d_edge_part;
    a.counter = c->d_edge_ctr;
    // the 3 sums land directly in mapped pinned host memory (no copy command per evaluation)
    a.result = c->d_edge_res_host;
    // Reduction of the lnL / derivative sums: per-workgroup partials and a second one-block
    // launch (default), or a last-workgroup ticket in the same launch (PU_EDGE_TWO_PASS=0).
    // The ticket needs an agent-scope release fence per workgroup, i.e. an L2 write-back on
    // every XCD for each of the ~1.6k workgroups: measured 40 us per launch against 19 us for
    // both launches of the two-pass form (cfg2, profiles/r01_edges_cfg2.json).
    const int two_pass = env_int("PU_EDGE_TWO_PASS", 1);
    a.two_pass = two_pass;
}

// one reduction launch (EDGE_LNL / EDGE_DERIV) and its 3 results back on the host
// host_p: the provider's matrices of one launch to the device, in the kernel's order
int upload_pm(pu_ctx *c, const std::vector<double> &m, EdgeArgs &a) {
    HIPCHK(&c->err, hipMemcpyAsync(c->d_edge_pm, m.data(), m.size() * 8, hipMemcpyHostToDevice,
                                   c->stream));
    // (pageable source: the copy has left the host buffer when the call returns)
    a.pmats = c->d_edge_pm;
    return PU_OK;
}

// n_mat matrices per category on the host, matrix m at length ts[m] and derivative order
// ord[m], in build_p's [m][c][K][K] order and arithmetic (evecs diag(x^ord e^{l t r}) ivecs,
// x = l r), for EdgeArgs::hp
void host_p_mats(const pu_ctx *c, int n_mat, const double *ts, const int *ord, double *hp) {
    const int K = c->K, C = c->C;
    const double *ev = c->h_eig.data(), *el = ev + K * K, *iv = el + K;
    double e[4];
    for (int m = 0; m < n_mat; ++m)
        for (int q = 0; q < C; ++q) {
            const double r = c->h_rates[q];
            const double tt = ts[m] * r;
            for (int k = 0; k < K; ++k) {
                e[k] = exp(el[k] * tt);
                if (ord[m] > 0) {
                    const double x = el[k] * r;
                    e[k] = ord[m] == 1 ? x * e[k] : (x * x) * e[k];
                }
            }
            double *P = hp + (size_t)(m * C + q) * K * K;
            for (int i = 0; i < K; ++i)
                for (int j = 0; j < K; ++j) {
                    double acc = 0.0;
                    for (int k = 0; k < K; ++k) acc = fma(ev[i * K + k] * e[k], iv[k * K + j], acc);
                    P[i * K + j] = acc;
                }
        }
}

// matrices in the launch: eigen-decomposed DNA models with at most 4 categories
bool inline_ok(const pu_ctx *c) {
    return !c->host_p && c->K <= 4 && c->C <= 4 &&
           c->h_eig.size() == (size_t)(2 * c->K * c->K + c->K) &&
           c->h_rates.size() == (size_t)c->C;
}

int run_reduce(pu_ctx *c, int mode, const NodeSrc &sa, const NodeSrc &sb, double t, double *r3) {
    EdgeArgs a;
    fill_args(c, a);
    a.op[0] = EdgeOp{sa, sb, -1, 0, 0.0, t};
    // derivative matrices by value in the launch (PU_EDGE_INLINE_P=0: built on the device)
    const int inline_env = env_int("PU_EDGE_INLINE_P", 1);
    if (inline_env && mode == EDGE_DERIV && inline_ok(c)) {
        const double ts[4] = {0.0, t, t, t};
        const int ord[4] = {0, 0, 1, 2};
        host_p_mats(c, 4, ts, ord, a.hp);
        a.inline_p = 1;
    }
    if (c->host_p) {  // P(0), P(t) (, dP/dt, d2P/dt2) from the provider
        const size_t one = (size_t)c->C * c->K * c->K;
        std::vector<double> m((mode == EDGE_DERIV ? 4 : 2) * one);
        const double ts[2] = {0.0, t};
        int rc = pu::provide(c, 0, 2, ts, m.data());
        if (!rc && mode == EDGE_DERIV) rc = pu::provide(c, 1, 1, &t, m.data() + 2 * one);
        if (!rc && mode == EDGE_DERIV) rc = pu::provide(c, 2, 1, &t, m.data() + 3 * one);
        if (!rc) rc = upload_pm(c, m, a);
        if (rc) return rc;
    }
    if (edge_lds_bytes(mode, c->K, c->C) > 160 * 1024)
        return set_err(&c->err, PU_E_ARG, "edge operation: C=%d categories of K=%d states "
                       "exceed the LDS of one workgroup", c->C, c->K);
    hipEvent_t *ev = nullptr;
    if (c->profile && c->n_edge_prof < 65536) {
        if (c->edge_ev.size() < 3 * (size_t)(c->n_edge_prof + 1)) {
            const size_t old = c->edge_ev.size();
            c->edge_ev.resize(3 * (size_t)(c->n_edge_prof + 1), nullptr);
            for (size_t i = old; i < c->edge_ev.size(); ++i)
                HIPCHK(&c->err, hipEventCreate(&c->edge_ev[i]));
        }
        ev = &c->edge_ev[3 * (size_t)c->n_edge_prof++];
        HIPCHK(&c->err, hipEventRecord(ev[0], c->stream));
    }
    // EDGE_DERIV: every workgroup writes its 3 partial sums straight into pinned host memory
    // and the host adds them in workgroup order once every slot has left the sentinel
    // (PU_EDGE_HOST_SUM=0: the k_edge_sum launch below)
    const int host_sum_env = env_int("PU_EDGE_HOST_SUM", 1);
    if (host_sum_env && mode == EDGE_DERIV && a.two_pass == 1) {
        const int b = c->edge_part_buf ^= 1;
        double *hp = c->h_edge_part[b];
        a.block_part = c->d_edge_part_host[b];
        a.two_pass = 2;  // partials only, no k_edge_sum
        const size_t n = 3 * (size_t)c->n_tiles;
        // every way out of here leaves the buffer sentinel-filled again: a stale value left in
        // it would pass for a result two evaluations later
        auto fail = [&](hipError_t e, const char *what) {
            (void)hipStreamSynchronize(c->stream);
            fill_sentinel(hp, n);
            return set_err(&c->err, PU_E_HIP, "edge evaluation: %s (%s)", what,
                           hipGetErrorString(e));
        };
        hipError_t e = (hipError_t)launch_edge(c->stream, mode, a, ev ? ev[2] : nullptr);
        if (e != hipSuccess) return fail(e, "launch");
        if (ev && (e = hipEventRecord(ev[1], c->stream)) != hipSuccess) return fail(e, "event");
        volatile uint64_t *u = reinterpret_cast<volatile uint64_t *>(hp);
        for (size_t i = 0; i < n; ++i)
            for (unsigned long spin = 0; u[i] == kPartSentinel; ++spin) {
                if ((spin & 0xffff) == 0xffff && hipStreamQuery(c->stream) != hipErrorNotReady) {
                    // the launch has ended: its writes are visible, or it failed
                    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess)
                        return fail(e, "kernel");
                    if (u[i] == kPartSentinel)
                        return fail(hipErrorUnknown, "partial sums never arrived");
                    break;
                }
                __builtin_ia32_pause();
            }
        std::atomic_thread_fence(std::memory_order_acquire);
        double s0 = 0.0, s1 = 0.0, s2 = 0.0;
        for (size_t w = 0; w < (size_t)c->n_tiles; ++w) {
            s0 += hp[3 * w];
            s1 += hp[3 * w + 1];
            s2 += hp[3 * w + 2];
        }
        fill_sentinel(hp, n);
        r3[0] = s0;
        r3[1] = s1;
        r3[2] = s2;
        return PU_OK;
    }
    // Completion: the host polls the sequence number k_edge_sum writes into mapped memory
    // after the sums (PU_EDGE_POLL=0: hipStreamSynchronize).  Not with the ascertainment
    // correction, which rewrites the lnL in a later launch.
    const int poll_env = env_int("PU_EDGE_POLL", 1);
    const bool poll = poll_env && a.two_pass == 1 && !(mode == EDGE_LNL && c->asc_mode);
    a.seq = poll ? (c->edge_seq += 1.0) : 0.0;
    HIPCHK(&c->err, (hipError_t)launch_edge(c->stream, mode, a, ev ? ev[2] : nullptr));
    if (mode == EDGE_LNL) {
        int rc = enqueue_ascbias(c, c->d_edge_res_host);
        if (rc) return rc;
    }
    if (ev) HIPCHK(&c->err, hipEventRecord(ev[1], c->stream));
    bool done = false;
    if (poll) {
        volatile double *flag = c->h_edge_res + 3;
        for (unsigned long spin = 0; !done; ++spin) {
            if (*flag == a.seq) {
                done = true;
            } else if ((spin & 0xffff) == 0xffff && hipStreamQuery(c->stream) != hipErrorNotReady) {
                break;  // finished without the flag (or failed): synchronise for the status
            } else {
                __builtin_ia32_pause();
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    }
    if (!done) HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    for (int k = 0; k < 3; ++k) r3[k] = c->h_edge_res[k];
    return PU_OK;
}

int derivs_at(pu_ctx *c, const NodeSrc &sa, const NodeSrc &sb, double t, double *r3) {
    if (c->asc_mode)
        return set_err(&c->err, PU_E_STATE, "branch-length derivatives with the ascertainment-"
                       "bias correction are not implemented");
    return run_reduce(c, EDGE_DERIV, sa, sb, t, r3);
}

// The whole Newton loop below in one persistent launch (k_edge_newton, r06): DNA models on
// the device's eigen-system, C <= 4, no ascertainment correction, and a grid the device holds
// at once at <= 2 tiles per wave (about 390k sites on MI355X).  Returns 1 (nothing done) when not
// eligible, so newton() runs the host loop.  PU_EDGE_DEVICE_NEWTON=0: always the host loop.
std::mutex g_newton_mu[64];

// mode PU_MIN_BRENT / PU_MIN_DBRENT: the reference's minimisers instead (pu_minimise.h) over
// [lo, hi] from t0; then t_out = x, r_out[0] = lnL(x), it_out = the reference's iteration count
int device_newton(pu_ctx *c, const NodeSrc &sa, const NodeSrc &sb, double t0, double tol,
                  int max_iter, double *t_out, double *r_out, int *it_out,
                  int mode = PU_MIN_NEWTON, double lo = 0.0, double hi = 0.0) {
    const auto h_in = std::chrono::steady_clock::now();
    if (!env_int("PU_EDGE_DEVICE_NEWTON", 1) || c->host_p || c->asc_mode ||
        (c->K != 2 && c->K != 4) || c->C > 4 ||
        c->h_eig.size() != (size_t)(2 * c->K * c->K + c->K))
        return 1;
    // tiles per wave: 1 (4 workgroups per CU) when the grid fits, else 2; the occupancy API
    // can admit one workgroup per CU too many (MI355X_MICROARCH.md): margin of one
    int tpw = 0, grid = 0;
    const int tpw_min = std::max(1, std::min(edge_newton_max_tpw(), env_int("PU_NT_TPW", 1)));
    for (int k = tpw_min; k <= edge_newton_max_tpw() && !tpw; ++k) {
        if (c->nt_per_cu_t[k] < 0) c->nt_per_cu_t[k] = edge_newton_per_cu(c->K, c->C, k);
        const int pc = c->nt_per_cu_t[k];
        const int64_t cap = (int64_t)(pc > 1 ? pc - 1 : pc) * c->n_cu;
        const int per = edge_newton_tiles_per_wg(k);
        const int64_t need = ((int64_t)c->n_tiles + per - 1) / per;
        if (cap >= 1 && need <= cap) {
            tpw = k;
            grid = (int)need;
        }
    }
    if (!tpw) return 1;
    const size_t words = edge_newton_sync_words(grid);
    int rc;
    if (c->nt_slots_cap < words) {
        dfree(c->d_nt_slots);
        if ((rc = dalloc(&c->err, &c->d_nt_slots, words))) return rc;
        c->nt_slots_cap = words;
        c->nt_fresh = false;
    }
    if (!c->h_nt_res) {
        HIPCHK(&c->err, hipHostMalloc((void **)&c->h_nt_res, kNewtonState * sizeof(double),
                                      hipHostMallocMapped));
        c->h_nt_res[7] = 0.0;
        HIPCHK(&c->err, hipHostGetDevicePointer((void **)&c->d_nt_res_host, c->h_nt_res, 0));
    }
    EdgeArgs a;
    fill_args(c, a);
    a.op[0] = EdgeOp{sa, sb, -1, 0, 0.0, t0};
    NewtonArgs n;
    n.t0 = t0;
    n.tol = tol;
    n.seq = (c->nt_seq += 1.0);
    n.max_iter = max_iter;
    n.tpw = tpw;
    // an ordinary launch: the grid fits the device at once (occupancy API with a margin), so on
    // an otherwise idle device every workgroup is resident.  hipLaunchCooperativeKernel
    // guarantees it, but costs ~65 us per launch (r06: 64.8 vs 130.5 us per optimisation);
    // work on other streams only delays workgroups, and a wait that never ends (another
    // persistent grid holding the CUs) times out and falls back to the host loop below
    n.mode = mode;
    n.lo = lo;
    n.hi = hi;
    n.plain = !env_int("PU_NT_COOPERATIVE", 0);
    n.spins = (unsigned)std::max(1, env_int("PU_NT_SPINS", (int)kNewtonSpins));  // tests: 1
    n.slots = c->d_nt_slots;
    n.pub = c->d_nt_slots + 8 * (size_t)grid;
    n.res = c->d_nt_res_host;
    n.timing = nullptr;
    n.n_timing = 0;
    // debug: per-evaluation stamps, printed after the launch (PU_NT_TIMING=1)
    // (per device: a process may optimise on several GPUs)
    static unsigned long long *d_tm_dev[64] = {};
    unsigned long long *&d_tm = d_tm_dev[c->device & 63];
    constexpr int kTm = 64;
    if (env_int("PU_NT_TIMING", 0)) {
        if (!d_tm && (rc = dalloc(&c->err, &d_tm, (size_t)8 * kTm))) return rc;
        HIPCHK(&c->err, hipMemsetAsync(d_tm, 0, 8 * kTm * 8, c->stream));
        n.timing = d_tm;
        n.n_timing = kTm;
    }
    // the generations are monotone across launches: the slots are zeroed only when they start
    // afresh (a memset is a launch of its own, about as long as an evaluation)
    if (!c->nt_fresh || c->nt_grid != grid || c->nt_base > (1u << 30)) {
        HIPCHK(&c->err, hipMemsetAsync(c->d_nt_slots, 0, words * sizeof(uint64_t), c->stream));
        c->nt_base = 0;
        c->nt_grid = grid;
        c->nt_fresh = true;
    }
    n.base = c->nt_base;
    // one device Newton grid per device at a time in this process: two partly resident grids
    // would each wait for the other's CUs until the timeout
    std::lock_guard<std::mutex> lk(g_newton_mu[c->device & 63]);
    c->h_nt_res[6] = 0.0;  // the error word (the previous launch has left: its result was seen)
    const auto h0 = std::chrono::steady_clock::now();
    hipError_t e = (hipError_t)launch_edge_newton(c->stream, a, n, grid);
    const auto h1 = std::chrono::steady_clock::now();
    if (e != hipSuccess) {
        (void)hipGetLastError();
        c->nt_fresh = false;
        if (e == hipErrorCooperativeLaunchTooLarge || e == hipErrorNotSupported) return 1;
        return set_err(&c->err, PU_E_HIP, "k_edge_newton launch: %s", hipGetErrorString(e));
    }
    ++c->nt_launches;
    // completion: the combiner writes the result, then the sequence number (mapped memory); a
    // workgroup that timed out sets the error word alone
    volatile double *flag = c->h_nt_res + 7, *fail = c->h_nt_res + 6;
    bool done = false;
    for (unsigned long spin = 0; !done; ++spin) {
        if (*flag == n.seq) {
            done = true;
        } else if (*fail != 0.0) {
            break;
        } else if ((spin & 0xffff) == 0xffff && hipStreamQuery(c->stream) != hipErrorNotReady) {
            break;
        } else {
            __builtin_ia32_pause();
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    const auto h2 = std::chrono::steady_clock::now();
    // The result is final when its sequence number is: the rest of the grid only leaves (after
    // the last generation) and reads nothing else, and later work on the stream is ordered
    // after it, so the host does not wait for the drain -- unless the result never came
    // (synchronise for the status) or the debug stamps are to be read
    if (!done || n.timing || *fail != 0.0) {
        if (hipError_t es = hipStreamSynchronize(c->stream); es != hipSuccess) {
            c->nt_fresh = false;
            return set_err(&c->err, PU_E_HIP, "k_edge_newton: %s", hipGetErrorString(es));
        }
    }
    if (n.timing) {
        const auto h3 = std::chrono::steady_clock::now();
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        fprintf(stderr, "[pu newton] host: entry to launch %.1f us, launch call %.1f us, to result "
                "%.1f us, drain %.1f us\n", us(h_in, h0), us(h0, h1), us(h1, h2), us(h2, h3));
    }
    if (!done && *flag != n.seq && *fail == 0.0) {
        c->nt_fresh = false;
        return set_err(&c->err, PU_E_HIP, "k_edge_newton ended without a result");
    }
    if (*fail != 0.0) {
        // a workgroup timed out waiting for the grid (not all resident): every workgroup leaves,
        // the slots start afresh, and this optimisation runs on the host loop
        c->nt_fresh = false;
        ++c->nt_timeouts;
        HIPCHK(&c->err, hipStreamSynchronize(c->stream));
        return 1;
    }
    c->nt_base += (unsigned)c->h_nt_res[5];
    if (n.timing) {
        unsigned long long h[8 * kTm];
        HIPCHK(&c->err, hipMemcpy(h, d_tm, sizeof h, hipMemcpyDeviceToHost));
        const int ne = std::min(kTm, (int)c->h_nt_res[5]);
        fprintf(stderr, "[pu newton] grid %d tpw %d: per evaluation (us) tiles (= factors+barrier, "
                "sites+wave sums, barrier), slot->all slots seen, seen->published, published->seen "
                "(workgroup 1), seen->next start\n", grid, tpw);
        for (int i = 0; i < ne; ++i) {
            const unsigned long long *r = h + 8 * i;
            auto us = [](unsigned long long a, unsigned long long b) {
                return a && b ? ((double)b - (double)a) * 0.01 : -1.0;
            };
            fprintf(stderr, "[pu newton] ev %d: %.2f (%.2f %.2f %.2f) %.2f %.2f %.2f %.2f\n", i,
                    us(r[0], r[1]), us(r[0], r[5]), us(r[5], r[6]), us(r[6], r[7]), us(r[1], r[2]),
                    us(r[2], r[3]), us(r[3], r[4]), i + 1 < ne ? us(r[4], r[8]) : -1.0);
        }
    }
    *t_out = c->h_nt_res[0];
    for (int k = 0; k < 3; ++k) r_out[k] = c->h_nt_res[1 + k];
    *it_out = (int)c->h_nt_res[4];
    c->nt_evals += (int)c->h_nt_res[5];
    return PU_OK;
}

// Newton-Raphson on one edge length with a monotone safeguard: a step that lowers the lnL
// is halved (up to 30 times); a non-concave point moves by expansion (d1 > 0) or halving.
int newton(pu_ctx *c, int na, int nb, int key, double tol, int max_iter, double *len_io,
           double *lnl_out, int *iters_out) {
    NodeSrc sa, sb;
    int rc;
    if ((rc = node_src(c, na, &sa)) || (rc = node_src(c, nb, &sb))) return rc;
    double t = std::min(std::max(*len_io, kMinLen), kMaxLen);
    {
        double td, rd[3];
        int itd;
        rc = device_newton(c, sa, sb, t, tol, max_iter, &td, rd, &itd);
        if (rc < 0) return rc;
        if (rc == 0) {
            *len_io = td;
            set_len(c, key, td);
            if (lnl_out) *lnl_out = rd[0];
            if (iters_out) *iters_out = itd;
            return PU_OK;
        }
    }
    double r[3];
    if ((rc = derivs_at(c, sa, sb, t, r))) return rc;
    int it = 0;
    for (; it < max_iter; ++it) {
        const double l = r[0], d1 = r[1], d2 = r[2];
        if (!std::isfinite(l)) break;
        double step = d2 < 0.0 ? -d1 / d2 : (d1 > 0.0 ? t + 0.1 : -0.5 * t);
        double tn = std::min(std::max(t + step, kMinLen), kMaxLen);
        if (tn == t) break;
        double rn[3];
        bool ok = false;
        for (int h = 0; h < 30; ++h) {
            if ((rc = derivs_at(c, sa, sb, tn, rn))) return rc;
            if (rn[0] >= l - 1e-13 * fabs(l)) {
                ok = true;
                break;
            }
            tn = 0.5 * (t + tn);
        }
        if (!ok) break;  // no ascent along this direction: t is (numerically) optimal
        const double dt = fabs(tn - t);
        t = tn;
        r[0] = rn[0];
        r[1] = rn[1];
        r[2] = rn[2];
        if (dt <= tol * (1.0 + t)) {
            ++it;
            break;
        }
    }
    *len_io = t;
    set_len(c, key, t);
    if (lnl_out) *lnl_out = r[0];
    if (iters_out) *iters_out = it;
    return PU_OK;
}

// rebuild the device branch lengths (caller op order) from parent / up_len
int push_lengths(pu_ctx *c) {
    std::vector<double> bl(2 * (size_t)c->n_ops);
    for (int o = 0; o < c->n_ops; ++o) {
        bl[2 * o] = c->up_len[c->ops_in[3 * o + 1]];
        bl[2 * o + 1] = c->up_len[c->ops_in[3 * o + 2]];
    }
    return pu_set_branch_lengths(c, bl.data(), c->up_len[c->root_a]);
}

int update_ops(pu_ctx *c, int n, const int32_t *ops, const double *brlens) {
    EdgeArgs a;
    fill_args(c, a);
    if (edge_lds_bytes(EDGE_UPDATE, c->K, c->C) > 160 * 1024)
        return set_err(&c->err, PU_E_ARG, "edge operation: too many categories for LDS");
    int k = 0;
    for (int o = 0; o < n; ++o) {
        const int p = ops[3 * o], x = ops[3 * o + 1], y = ops[3 * o + 2];
        if (p == x || p == y || x == y)
            return set_err(&c->err, PU_E_ARG, "update %d (%d,%d,%d): repeated node", o, p, x, y);
        NodeSrc sp, sx, sy;
        int rc;
        if ((rc = node_src(c, p, &sp)) || (rc = node_src(c, x, &sx)) || (rc = node_src(c, y, &sy)))
            return rc;
        if (sp.kind != SRC_SLOT)
            return set_err(&c->err, PU_E_ARG, "update %d: parent %d is a tip", o, p);
        a.op[k++] = EdgeOp{sx, sy, sp.idx, 0, brlens[2 * o], brlens[2 * o + 1]};
        if (k == kEdgeOpsPerLaunch || o == n - 1) {
            a.n_ops = k;
            // one or two ops (the sweep's re-orientations): their P in the launch
            a.inline_p = 0;
            if (k <= 2 && env_int("PU_EDGE_INLINE_P", 1) && inline_ok(c)) {
                for (int q = 0; q < k; ++q) {
                    const double ts[2] = {a.op[q].t_a, a.op[q].t_b};
                    const int ord[2] = {0, 0};
                    host_p_mats(c, 2, ts, ord, a.hp + (size_t)q * 2 * c->C * c->K * c->K);
                }
                a.inline_p = 1;
            }
            if (c->host_p) {  // P(t_a), P(t_b) of every op of the launch from the provider
                std::vector<double> ts(2 * (size_t)k), m(2 * (size_t)k * c->C * c->K * c->K);
                for (int q = 0; q < k; ++q) {
                    ts[2 * q] = a.op[q].t_a;
                    ts[2 * q + 1] = a.op[q].t_b;
                }
                if ((rc = pu::provide(c, 0, 2 * k, ts.data(), m.data()))) return rc;
                // the previous launch may still read d_edge_pm
                HIPCHK(&c->err, hipStreamSynchronize(c->stream));
                if ((rc = upload_pm(c, m, a))) return rc;
            }
            HIPCHK(&c->err, (hipError_t)launch_edge(c->stream, EDGE_UPDATE, a));
            k = 0;
        }
    }
    return PU_OK;
}

}  // namespace

int pu::flush_lengths(pu_ctx *c) { return c->lengths_dirty ? push_lengths(c) : PU_OK; }

int pu::enqueue_ascbias(pu_ctx *c, double *lnl) {
    if (!c->asc_mode) return PU_OK;
    if (!c->d_asc_corr) {
        int rc = dalloc(&c->err, &c->d_asc_corr, 1);
        if (rc) return rc;
    }
    AscArgs a;
    a.K = c->K;
    a.C = c->C;
    a.n_tiles = c->n_tiles;
    a.tile_pitch = (int)ctx_pitch(c);
    a.mode = c->asc_mode;
    a.first = c->asc_first;
    a.root_clv = c->d_root;
    a.root_scale = c->d_root_scale;
    a.pi = c->d_pi;
    a.site_lnl = c->d_site_lnl;
    a.lnl = lnl;
    a.corr = c->d_asc_corr;
    a.sum_w = 0.0;
    for (int64_t s = 0; s < c->asc_first; ++s) a.sum_w += c->h_pattern_w[s];
    HIPCHK(&c->err, (hipError_t)launch_ascbias(c->stream, a));
    return PU_OK;
}

void pu::edge_free(pu_ctx *c) {
    dfree(c->d_asc_corr);
    dfree(c->d_edge_pm);
    for (hipEvent_t e : c->edge_ev) (void)hipEventDestroy(e);
    c->edge_ev.clear();
    dfree(c->d_edge_part);
    dfree(c->d_edge_ctr);
    dfree(c->d_edge_res);
    if (c->h_edge_res) (void)hipHostFree(c->h_edge_res);
    c->h_edge_res = nullptr;
    dfree(c->d_nt_slots);
    c->nt_slots_cap = 0;
    if (c->h_nt_res) (void)hipHostFree(c->h_nt_res);
    c->h_nt_res = nullptr;
    for (double *&h : c->h_edge_part) {
        if (h) (void)hipHostFree(h);
        h = nullptr;
    }
    c->edge_tiles = 0;
}

extern "C" {

int pu_edge_lnl(pu_ctx *c, int node_a, int node_b, double *lnl_out, double *sitewise_out) {
    int rc = prepare(c);
    if (rc) return rc;
    DeviceGuard g(c->device);
    int key;
    NodeSrc sa, sb;
    if ((rc = edge_of(c, node_a, node_b, &key)) || (rc = node_src(c, node_a, &sa)) ||
        (rc = node_src(c, node_b, &sb)))
        return rc;
    double r[3];
    if ((rc = run_reduce(c, EDGE_LNL, sa, sb, c->up_len[key], r))) return rc;
    if (lnl_out) *lnl_out = r[0];
    if (sitewise_out)
        HIPCHK(&c->err, hipMemcpy(sitewise_out, c->d_site_lnl, (size_t)c->S * 8,
                                  hipMemcpyDeviceToHost));
    return PU_OK;
}

int pu_edge_derivs(pu_ctx *c, int node_a, int node_b, double length, double *out3) {
    if (!out3) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null output");
    int rc = prepare(c);
    if (rc) return rc;
    DeviceGuard g(c->device);
    int key;
    NodeSrc sa, sb;
    if ((rc = edge_of(c, node_a, node_b, &key)) || (rc = node_src(c, node_a, &sa)) ||
        (rc = node_src(c, node_b, &sb)))
        return rc;
    if (length < 0.0) length = c->up_len[key];
    return derivs_at(c, sa, sb, length, out3);
}

int pu_update_partials(pu_ctx *c, int n_ops, const int32_t *ops, const double *brlens) {
    if (n_ops < 0 || (n_ops > 0 && (!ops || !brlens)))
        return set_err(c ? &c->err : nullptr, PU_E_ARG, "bad update arguments");
    int rc = prepare(c);
    if (rc) return rc;
    DeviceGuard g(c->device);
    if ((rc = update_ops(c, n_ops, ops, brlens))) return rc;
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    return PU_OK;
}

int pu_optimise_edge(pu_ctx *c, int node_a, int node_b, double tol, int max_iter,
                     double *length_out, double *lnl_out) {
    int rc = prepare(c);
    if (rc) return rc;
    DeviceGuard g(c->device);
    int key;
    if ((rc = edge_of(c, node_a, node_b, &key))) return rc;
    double t = c->up_len[key];
    if ((rc = newton(c, node_a, node_b, key, tol, max_iter, &t, lnl_out, nullptr))) return rc;
    if (length_out) *length_out = t;
    if (c->host_p) return push_lengths(c);  // the provider's matrices follow h_brlens now
    // the device copy of the lengths is rebuilt by the next launch that reads it
    // (pu::prepare_launch): a run of edge optimisations does not wait for each Newton drain
    c->lengths_dirty = true;
    return PU_OK;
}

int pu_optimise_sweep(pu_ctx *c, int n_rows, const int32_t *rows, double tol, int max_iter,
                      double *lnl_out, int *evals_out) {
    if (n_rows < 1 || !rows) return set_err(c ? &c->err : nullptr, PU_E_ARG, "no rows");
    int rc = prepare(c);
    if (rc) return rc;
    DeviceGuard g(c->device);
    int total_iters = 0;
    for (int r = 0; r < n_rows; ++r) {
        const int32_t *row = rows + 5 * (size_t)r;
        if (row[0] >= 0) {
            // re-orient (rows (PAR, SIB, GPA, NOD, PAR)) or restore (NOD, CH1, CH2, -1, -1)
            int k1, k2;
            if ((rc = edge_of(c, row[0], row[1], &k1)) || (rc = edge_of(c, row[0], row[2], &k2)))
                return rc;
            const double bl[2] = {c->up_len[k1], c->up_len[k2]};
            if ((rc = update_ops(c, 1, row, bl))) return rc;
        }
        if (row[3] >= 0) {
            int key, it = 0;
            if ((rc = edge_of(c, row[3], row[4], &key))) return rc;
            double t = c->up_len[key];
            if ((rc = newton(c, row[3], row[4], key, tol, max_iter, &t, nullptr, &it))) return rc;
            total_iters += it;
        }
    }
    if (evals_out) *evals_out = total_iters;
    // every node is back in its post-order orientation; one traversal with the new lengths
    if ((rc = push_lengths(c))) return rc;
    return pu_run(c, lnl_out, nullptr);
}

int pu_minimise_edge(pu_ctx *c, int node_a, int node_b, int method, double lo, double t0,
                     double hi, double tol, double *out3) {
    if (!out3) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null output");
    if (method != PU_MIN_BRENT && method != PU_MIN_DBRENT)
        return set_err(c ? &c->err : nullptr, PU_E_ARG, "method %d: 1 (brent) or 2 (dbrent)",
                       method);
    if (!(lo < hi) || !(tol > 0.0))
        return set_err(c ? &c->err : nullptr, PU_E_ARG, "bracket [%g, %g], tol %g", lo, hi, tol);
    int rc = prepare(c);
    if (rc) return rc;
    if (c->asc_mode)
        return set_err(&c->err, PU_E_STATE, "branch-length derivatives with the ascertainment-"
                       "bias correction are not implemented");
    DeviceGuard g(c->device);
    int key;
    NodeSrc sa, sb;
    if ((rc = edge_of(c, node_a, node_b, &key)) || (rc = node_src(c, node_a, &sa)) ||
        (rc = node_src(c, node_b, &sb)))
        return rc;
    double x = 0.0, r[3] = {0.0, 0.0, 0.0};
    int it = 0;
    // the whole minimisation in one persistent launch, else one k_edge launch per evaluation;
    // both drive the same state machine (pu_minimise.h)
    rc = device_newton(c, sa, sb, t0, tol, 0, &x, r, &it, method, lo, hi);
    if (rc < 0) return rc;
    if (rc == 1) {
        MinState ms;
        double t = min_start(ms, method, lo, t0, hi, tol);
        while (!ms.done) {
            if ((rc = derivs_at(c, sa, sb, t, r))) return rc;
            t = min_step(ms, -r[0], -r[1]);
        }
        x = ms.res_x;
        r[0] = -ms.res_f;
        it = ms.res_it;
    }
    out3[0] = x;
    out3[1] = -r[0];  // the reference's out[1]: the minimised objective f(x) = -lnL(x)
    out3[2] = (double)it;
    set_len(c, key, x);
    if (c->host_p) return push_lengths(c);
    c->lengths_dirty = true;
    return PU_OK;
}

int pu_ctx_newton_stats(pu_ctx *c, int *launches, int *evaluations) {
    if (!c) return set_err(nullptr, PU_E_ARG, "null context");
    if (launches) *launches = c->nt_launches;
    if (evaluations) *evaluations = c->nt_evals;
    return PU_OK;
}

int pu_set_ascertainment(pu_ctx *c, int mode, int64_t first_dummy) {
    if (!c) return set_err(nullptr, PU_E_ARG, "null context");
    if (mode < 0 || mode > 2) return set_err(&c->err, PU_E_ARG, "ascertainment mode %d", mode);
    if (mode && first_dummy + c->K != c->S)
        return set_err(&c->err, PU_E_ARG, "the %d dummy invariant sites must be the last "
                       "patterns: first_dummy %lld + K != S %lld", c->K, (long long)first_dummy,
                       (long long)c->S);
    if (mode && c->C > 64) return set_err(&c->err, PU_E_ARG, "too many categories");
    c->asc_mode = mode;
    c->asc_first = mode ? first_dummy : 0;
    return PU_OK;
}

int pu_get_ascertainment_correction(pu_ctx *c, double *corr_out) {
    if (!c || !corr_out) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (!c->asc_mode || !c->d_asc_corr)
        return set_err(&c->err, PU_E_STATE, "no ascertainment correction computed");
    DeviceGuard g(c->device);
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    HIPCHK(&c->err, hipMemcpy(corr_out, c->d_asc_corr, sizeof(double), hipMemcpyDeviceToHost));
    return PU_OK;
}

int pu_get_branch_lengths(pu_ctx *c, double *brlens_out, double *root_len_out) {
    if (!c || (!brlens_out && c->n_ops > 0))
        return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (!c->have_sched) return set_err(&c->err, PU_E_STATE, "pu_set_schedule first");
    for (int o = 0; o < c->n_ops; ++o) {
        brlens_out[2 * o] = c->up_len[c->ops_in[3 * o + 1]];
        brlens_out[2 * o + 1] = c->up_len[c->ops_in[3 * o + 2]];
    }
    if (root_len_out) *root_len_out = c->up_len[c->root_a];
    return PU_OK;
}

int pu_ctx_edge_kernel_ms(pu_ctx *c, double *kernel_ms_avg, int *n) {
    return pu_ctx_edge_kernel_ms2(c, kernel_ms_avg, nullptr, n);
}

int pu_ctx_edge_kernel_ms2(pu_ctx *c, double *kernel_ms_avg, double *edge_ms_avg, int *n) {
    if (!c) return set_err(nullptr, PU_E_ARG, "null context");
    DeviceGuard g(c->device);
    double acc = 0.0, acc_e = 0.0;
    for (int k = 0; k < c->n_edge_prof; ++k) {
        hipEvent_t *e = &c->edge_ev[3 * (size_t)k];
        float ms = 0.f, ms_e = 0.f;
        HIPCHK(&c->err, hipEventSynchronize(e[1]));
        HIPCHK(&c->err, hipEventElapsedTime(&ms, e[0], e[1]));
        HIPCHK(&c->err, hipEventElapsedTime(&ms_e, e[0], e[2]));
        acc += ms;
        acc_e += ms_e;
    }
    if (kernel_ms_avg) *kernel_ms_avg = c->n_edge_prof ? acc / c->n_edge_prof : 0.0;
    if (edge_ms_avg) *edge_ms_avg = c->n_edge_prof ? acc_e / c->n_edge_prof : 0.0;
    if (n) *n = c->n_edge_prof;
    return PU_OK;
}

static int lnl_branch_impl(int device, int M, int K, int64_t E, int n_p, const int32_t *pidx,
                           const double *probs, const double *pi, const double *pa,
                           const double *pb, const double *sa, const double *sb, double *out) {
    if (K < 1 || K > 64 || E < 0 || n_p < 1)
        return set_err(nullptr, PU_E_ARG, "lnl_branch: bad shape K=%d E=%lld n_p=%d", K,
                       (long long)E, n_p);
    if (!probs || !pi || (E > 0 && (!pa || !pb || !sa || !sb || !out)))
        return set_err(nullptr, PU_E_ARG, "lnl_branch: null buffer");
    int rc = check_device(device);
    if (rc) return rc;
    if (E == 0) return PU_OK;
    if (pidx)
        for (int64_t e = 0; e < E; ++e)
            if (pidx[e] < 0 || pidx[e] >= n_p)
                return set_err(nullptr, PU_E_ARG, "lnl_branch: probs index %d out of range",
                               pidx[e]);
    DeviceGuard g(device);
    std::lock_guard<std::mutex> lk(ws_mutex(device));
    const size_t nP = (size_t)n_p * M * K * K, nV = (size_t)E * K, nI = pidx ? (E + 1) / 2 : 0;
    double *w;
    hipStream_t st;
    if ((rc = ws_get(device, nP + K + 2 * nV + 2 * E + (size_t)M * E + nI, &w, &st))) return rc;
    double *dP = w, *dpi = dP + nP, *da = dpi + K, *db = da + nV, *dsa = db + nV, *dsb = dsa + E,
           *dout = dsb + E;
    int32_t *didx = pidx ? reinterpret_cast<int32_t *>(dout + (size_t)M * E) : nullptr;
    HIPCHK(nullptr, hipMemcpyAsync(dP, probs, nP * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(dpi, pi, K * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(da, pa, nV * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(db, pb, nV * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(dsa, sa, E * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(dsb, sb, E * 8, hipMemcpyHostToDevice, st));
    if (didx) HIPCHK(nullptr, hipMemcpyAsync(didx, pidx, E * 4, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, (hipError_t)launch_lnl_branch(st, K, M, E, n_p, didx, dP, dpi, da, db, dsa,
                                                   dsb, dout));
    HIPCHK(nullptr, hipMemcpyAsync(out, dout, (size_t)M * E * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(nullptr, hipStreamSynchronize(st));
    return PU_OK;
}

int pu_lnl_branch(int device, int K, int64_t E, int n_p, const int32_t *pidx,
                  const double *probs, const double *pi, const double *pa, const double *pb,
                  const double *sa, const double *sb, double *out) {
    return lnl_branch_impl(device, 1, K, E, n_p, pidx, probs, pi, pa, pb, sa, sb, out);
}

int pu_lnl_branch_derivs(int device, int K, int64_t E, int n_p, const int32_t *pidx,
                         const double *probs, const double *pi, const double *pa,
                         const double *pb, const double *sa, const double *sb, double *out) {
    return lnl_branch_impl(device, 3, K, E, n_p, pidx, probs, pi, pa, pb, sa, sb, out);
}

}  // extern "C"
