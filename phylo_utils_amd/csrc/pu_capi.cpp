// pu_capi.cpp -- C ABI (include/phylo_hip.h), device contexts and the schedule planner.
//
// A context is the device-resident counterpart of one TreeModel
// (phylo_utils/tree_model.py:12-217): tips, substitution/rate model, the
// flattened post-order (Traversal.postorder_traversal, traversal.py:28,36) and
// all conditional-likelihood buffers live in HBM; one pu_run = P matrices for
// every branch + the whole post-order + root combine + lnL reduction, enqueued
// on the context's stream as three kernels.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <cmath>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "pu_ctx.h"

using pu::OpDesc;

namespace pu {
thread_local std::string g_err;
}  // namespace pu

using namespace pu;

namespace {

constexpr int kMaxProf = 4096;


// ------------------------------------------------------------------ planner
// Evaluate the post-order so that the subtree with the larger register need
// goes first (Strahler / Sethi-Ullman), then keep as many parent CLVs in
// registers as R slots allow: among overlapping lifetimes the value whose
// consumer comes last is the one left in memory (optimal for intervals).
struct Plan {
    std::vector<int> order;          // device op -> caller op
    std::vector<OpDesc> descs;       // n_ops + root
    std::vector<int> store_slot;     // node -> storage slot
    int n_store = 0;
    std::vector<char> swap;          // device op: children exchanged w.r.t. the caller's op
    int n_mem = 0;                   // children read back from HBM
    int n_lds = 0;                   // children from the LDS stash
    int n_tip = 0, n_cur = 0;        // children that are tips / the previous op's parent
    int max_live = 0;                // peak number of waiting parents (stack depth)
    // split plan (K = 20 KEEP): device ops [tasks[i].first, tasks[i].second) are chain i, an
    // independent subtree; the ops from top_lo on and the root combine form the top task
    std::vector<std::pair<int, int>> tasks;
    int top_lo = 0;
};

int make_plan(pu_ctx *c, int n_ops, const int32_t *ops, int root_a, int root_b, int L,
              bool reorder, bool keep_all, Plan &pl, int split = 0) {
    const int N = c->n_nodes;
    std::vector<int> prod(N, -1), cons_count(N, 0);
    for (int o = 0; o < n_ops; ++o) {
        const int p = ops[3 * o], a = ops[3 * o + 1], b = ops[3 * o + 2];
        if (p < 0 || p >= N || a < 0 || a >= N || b < 0 || b >= N || a == b || p == a ||
            p == b)
            return set_err(&c->err, PU_E_SCHED, "op %d (%d,%d,%d): node index out of range "
                           "or repeated (n_nodes=%d)", o, p, a, b, N);
        if (prod[p] >= 0)
            return set_err(&c->err, PU_E_SCHED, "node %d is the parent of ops %d and %d", p,
                           prod[p], o);
        prod[p] = o;
        cons_count[a]++;
        cons_count[b]++;
    }
    if (root_a < 0 || root_a >= N || root_b < 0 || root_b >= N || root_a == root_b)
        return set_err(&c->err, PU_E_SCHED, "bad root edge (%d,%d)", root_a, root_b);
    cons_count[root_a]++;
    cons_count[root_b]++;
    for (int v = 0; v < N; ++v) {
        if (prod[v] >= 0 && cons_count[v] != 1)
            return set_err(&c->err, PU_E_SCHED, "internal node %d is consumed %d times "
                           "(expected once)", v, cons_count[v]);
        if (prod[v] < 0 && cons_count[v] > 1)
            return set_err(&c->err, PU_E_SCHED, "tip node %d is consumed %d times", v,
                           cons_count[v]);
    }
    // order
    pl.order.clear();
    if (!reorder) {
        for (int o = 0; o < n_ops; ++o) {
            for (int k = 1; k <= 2; ++k) {
                const int ch = ops[3 * o + k];
                if (prod[ch] >= o)
                    return set_err(&c->err, PU_E_SCHED, "op %d reads node %d before it is "
                                   "computed (not a post-order)", o, ch);
            }
            pl.order.push_back(o);
        }
    } else {
        // need[] bottom-up without recursion (depth can reach N for caterpillars)
        std::vector<int> need(N, 0), state(N, 0);
        std::vector<int> stack;
        auto visit_need = [&](int root) -> int {
            stack.push_back(root);
            while (!stack.empty()) {
                const int v = stack.back();
                if (prod[v] < 0) {
                    need[v] = 0;
                    state[v] = 2;
                    stack.pop_back();
                    continue;
                }
                const int o = prod[v], a = ops[3 * o + 1], b = ops[3 * o + 2];
                if (state[v] == 0) {
                    state[v] = 1;
                    if (state[a] == 1 || state[b] == 1) return -1;  // cycle
                    if (state[a] == 0) stack.push_back(a);
                    if (state[b] == 0) stack.push_back(b);
                    continue;
                }
                stack.pop_back();
                if (state[v] == 2) continue;
                const int na = need[a], nb = need[b];
                need[v] = na == nb ? na + 1 : std::max(na, nb);
                state[v] = 2;
            }
            return 0;
        };
        if (visit_need(root_a) < 0 || visit_need(root_b) < 0)
            return set_err(&c->err, PU_E_SCHED, "schedule contains a cycle");
        int reached = 0;
        // emit post-order, larger-need child first
        auto emit = [&](int root) {
            std::vector<std::pair<int, int>> st;  // (node, phase)
            st.push_back({root, 0});
            while (!st.empty()) {
                auto [v, ph] = st.back();
                st.pop_back();
                if (prod[v] < 0) continue;
                const int o = prod[v], a = ops[3 * o + 1], b = ops[3 * o + 2];
                if (ph == 0) {
                    st.push_back({v, 1});
                    const int first = need[a] >= need[b] ? a : b;
                    const int second = first == a ? b : a;
                    st.push_back({second, 0});
                    st.push_back({first, 0});
                } else {
                    pl.order.push_back(o);
                    ++reached;
                }
            }
        };
        const int fa = need[root_a] >= need[root_b] ? root_a : root_b;
        emit(fa);
        emit(fa == root_a ? root_b : root_a);
        if (reached != n_ops)
            return set_err(&c->err, PU_E_SCHED, "%d of %d ops are not below the root edge",
                           n_ops - reached, n_ops);
    }
    // Split into tasks.  The post-order is one dependency chain per (tile, category) wave;
    // with few waves per SIMD its length sets the time of the SIMDs that carry one wave more
    // than the average.  Disjoint subtrees ("chains", about n_ops / split ops each) are
    // independent: a first launch runs every chain as a wave task of its own, a second the ops
    // above them (the "top": ancestors of the cut nodes, then the root combine), reading the
    // chain roots back from HBM.  Cuts: starting from the root's children, the largest subtree
    // is replaced by its children's while it exceeds the target (bounded top and task count).
    std::vector<int> region(n_ops + 1, 0);  // device op -> task (the top task is the last)
    pl.tasks.clear();
    pl.top_lo = 0;
    if (split > 1 && reorder && n_ops > 2) {
        std::vector<int> size(N, 0), parent(N, -1);
        for (int o : pl.order) {
            const int p = ops[3 * o], a = ops[3 * o + 1], b = ops[3 * o + 2];
            size[p] = 1 + size[a] + size[b];
            parent[a] = parent[b] = p;
        }
        std::vector<int> cuts;
        for (int r : {root_a, root_b})
            if (prod[r] >= 0) cuts.push_back(r);
        std::vector<char> is_top(N, 0);
        const int target = (n_ops + split - 1) / split;
        // at most n_ops / 16 top ops and 32 chains (r03 sweeps: no better value; cfg4 8 / 16 / 32
        // / 64 chains 3.70 / 3.44 / 3.37 / 3.38 ms)
        const int max_top = std::max(1, n_ops / 16);
        const size_t max_chains = 32;
        int n_top = 0;
        while (!cuts.empty()) {
            auto it = std::max_element(cuts.begin(), cuts.end(),
                                       [&](int x, int y) { return size[x] < size[y]; });
            if (size[*it] <= target || n_top >= max_top || cuts.size() >= max_chains) break;
            const int v = *it;
            cuts.erase(it);
            is_top[v] = 1;
            ++n_top;
            for (int k = 1; k <= 2; ++k) {
                const int ch = ops[3 * prod[v] + k];
                if (prod[ch] >= 0) cuts.push_back(ch);
            }
        }
        if (cuts.size() >= 2) {
            // longest chain first: the dispatcher hands out workgroups in block order
            std::stable_sort(cuts.begin(), cuts.end(),
                             [&](int x, int y) { return size[x] > size[y]; });
            std::vector<int> chain_of(N, -1), rank(N, -1);
            for (size_t k = 0; k < cuts.size(); ++k) rank[cuts[k]] = (int)k;
            for (int t = n_ops - 1; t >= 0; --t) {  // parents before children
                const int v = ops[3 * pl.order[t]];
                chain_of[v] = is_top[v] ? -1 : rank[v] >= 0 ? rank[v] : chain_of[parent[v]];
            }
            std::vector<int> order;
            order.reserve(n_ops);
            for (size_t k = 0; k < cuts.size(); ++k) {
                const int lo = (int)order.size();
                for (int o : pl.order)
                    if (chain_of[ops[3 * o]] == (int)k) order.push_back(o);
                pl.tasks.push_back({lo, (int)order.size()});
            }
            pl.top_lo = (int)order.size();
            for (int o : pl.order)
                if (chain_of[ops[3 * o]] < 0) order.push_back(o);
            pl.order = std::move(order);
            for (size_t k = 0; k < pl.tasks.size(); ++k)
                for (int t = pl.tasks[k].first; t < pl.tasks[k].second; ++t) region[t] = (int)k;
            for (int t = pl.top_lo; t <= n_ops; ++t) region[t] = (int)pl.tasks.size();
        }
    }
    const bool split_on = !pl.tasks.empty();
    const int top_region = (int)pl.tasks.size();
    // lifetimes in device order (root combine = time n_ops)
    std::vector<int> t_prod(N, -1), t_cons(N, -1);
    for (int t = 0; t < n_ops; ++t) {
        const int o = pl.order[t];
        t_prod[ops[3 * o]] = t;
        t_cons[ops[3 * o + 1]] = t;
        t_cons[ops[3 * o + 2]] = t;
    }
    t_cons[root_a] = n_ops;
    t_cons[root_b] = n_ops;
    // Child kinds: a tip, the previous op's parent (the kernel's "current" registers), a
    // waiting parent in an LDS stash slot, or one read back from HBM.  A parent waits when
    // its consumer is not the next op; at each production, if more parents wait than
    // there are L stash slots, the one whose consumer is latest stays in HBM (Belady,
    // optimal for intervals); stash slots are then assigned by interval colouring.
    std::vector<char> waits(N, 0), in_lds(N, 0);
    for (int t = 0; t < n_ops; ++t) {
        const int v = ops[3 * pl.order[t]];
        waits[v] = t_cons[v] != t + 1 || region[t_cons[v]] != region[t];
    }
    // the LDS stash serves values produced and consumed inside one chain task (the top task
    // reads every waiting parent back from HBM)
    auto stashable = [&](int v) {
        return !split_on || (region[t_prod[v]] != top_region &&
                             region[t_cons[v]] == region[t_prod[v]]);
    };
    // The stash serves DFS orders, where a waiting parent is always paired with the
    // current one (PAT_LC).  Other caller orders read every waiting parent back from HBM.
    auto dfs_pair = [&](int t, int a, int b) {
        for (int x : {a, b})
            if (prod[x] >= 0 && waits[x]) {
                const int y = x == a ? b : a;
                if (prod[y] < 0 || t_prod[y] != t - 1) return false;
            }
        return true;
    };
    for (int t = 0; t <= n_ops && L > 0; ++t) {
        if (split_on && region[t] == top_region) continue;
        const int a = t < n_ops ? ops[3 * pl.order[t] + 1] : root_a;
        const int b = t < n_ops ? ops[3 * pl.order[t] + 2] : root_b;
        if (!dfs_pair(t, a, b)) L = 0;
    }
    pl.max_live = 0;
    {
        std::vector<int> waiting, live;
        for (int t = 0; t < n_ops; ++t) {
            auto gone = [&](int x) { return t_cons[x] <= t; };
            waiting.erase(std::remove_if(waiting.begin(), waiting.end(), gone), waiting.end());
            live.erase(std::remove_if(live.begin(), live.end(), gone), live.end());
            const int v = ops[3 * pl.order[t]];
            if (!waits[v]) continue;
            waiting.push_back(v);
            pl.max_live = std::max(pl.max_live, (int)waiting.size());
            if (L == 0 || !stashable(v)) continue;
            live.push_back(v);
            in_lds[v] = 1;
            if ((int)live.size() > L) {
                auto it = std::max_element(live.begin(), live.end(), [&](int x, int y) {
                    return t_cons[x] < t_cons[y];
                });
                in_lds[*it] = 0;
                live.erase(it);
            }
        }
    }
    std::vector<int> lds_slot(N, -1);
    {
        std::vector<int> busy(std::max(L, 1), -1);
        for (int t = 0; t < n_ops; ++t) {
            const int v = ops[3 * pl.order[t]];
            if (!in_lds[v]) continue;
            for (int r = 0; r < L; ++r)
                if (busy[r] <= t) {  // the previous occupant was read at op busy[r]
                    busy[r] = t_cons[v];
                    lds_slot[v] = r;
                    break;
                }
            if (lds_slot[v] < 0)
                return set_err(&c->err, PU_E_SCHED, "LDS stash planner overflow");
        }
    }
    // storage slots: KEEP -- every internal node; LNL_ONLY -- only parents read back from
    // HBM, slots reused by interval colouring
    pl.store_slot.assign(N, -1);
    if (keep_all) {
        int s = 0;
        for (int v = 0; v < N; ++v)
            if (prod[v] >= 0) pl.store_slot[v] = s++;
        pl.n_store = s;
    } else {
        // interval colouring; a split plan colours each task apart (disjoint slot ranges):
        // chain tasks run concurrently, so no slot may pass from one chain's value to another's
        int base = 0;
        const int n_regions = split_on ? top_region + 1 : 1;
        for (int r = 0; r < n_regions; ++r) {
            std::vector<int> busy_until;
            for (int t = 0; t < n_ops; ++t) {
                if (split_on && region[t] != r) continue;
                const int v = ops[3 * pl.order[t]];
                if (!waits[v] || in_lds[v]) continue;
                int slot = -1;
                for (size_t k = 0; k < busy_until.size(); ++k)
                    if (busy_until[k] <= t) {  // the op that reads it writes after its reads
                        slot = (int)k;
                        break;
                    }
                if (slot < 0) {
                    slot = (int)busy_until.size();
                    busy_until.push_back(0);
                }
                busy_until[slot] = t_cons[v];
                pl.store_slot[v] = base + slot;
            }
            base += (int)busy_until.size();
        }
        pl.n_store = base;
    }
    // descriptors: canonical child order -- waiting parent first, then the current parent,
    // then tips; swap[t] records that the caller's (child 1, child 2) became (b, a)
    enum { K_WAIT, K_CUR, K_TIP };
    auto kind_at = [&](int node, int t) {
        if (prod[node] < 0) return (int)K_TIP;
        return t_prod[node] == t - 1 && region[t - 1] == region[t] ? (int)K_CUR : (int)K_WAIT;
    };
    pl.n_mem = pl.n_tip = pl.n_cur = pl.n_lds = 0;
    pl.descs.assign(n_ops + 1, OpDesc{-1, 0, 0, 0, -1, 0, 0});
    pl.swap.assign(n_ops + 1, 0);
    auto describe = [&](int t, int a, int b, int par_slot, int dst) -> int {
        int ka = kind_at(a, t), kb = kind_at(b, t);
        const bool swp = kb < ka;
        if (swp) {
            std::swap(a, b);
            std::swap(ka, kb);
        }
        int pat, ia = 0, ib = 0;
        if (ka == K_WAIT && kb == K_CUR) {
            pat = in_lds[a] ? pu::PAT_LC : pu::PAT_MC;
            ia = in_lds[a] ? lds_slot[a] : pl.store_slot[a];
        } else if (ka == K_CUR && kb == K_TIP) {
            pat = pu::PAT_CT;
            ib = c->tip_slot[b];
        } else if (ka == K_TIP && kb == K_TIP) {
            pat = pu::PAT_TT;
            ia = c->tip_slot[a];
            ib = c->tip_slot[b];
        } else if (ka == K_WAIT && !in_lds[a] && kb == K_TIP) {
            pat = pu::PAT_MT;
            ia = pl.store_slot[a];
            ib = c->tip_slot[b];
        } else if (ka == K_WAIT && !in_lds[a] && kb == K_WAIT && !in_lds[b]) {
            pat = pu::PAT_MM;
            ia = pl.store_slot[a];
            ib = pl.store_slot[b];
        } else {
            // a stashed parent that is not paired with the current one (not a DFS order)
            return set_err(&c->err, PU_E_SCHED, "op %d: child pair not supported", t);
        }
        for (int k : {ka, kb}) {
            if (k == K_TIP) pl.n_tip++;
            if (k == K_CUR) pl.n_cur++;
        }
        for (int n : {a, b})
            if (prod[n] >= 0 && kind_at(n, t) == K_WAIT) (in_lds[n] ? pl.n_lds : pl.n_mem)++;
        pl.descs[t] = OpDesc{par_slot, pat, ia, ib, dst, 0, 0};
        pl.swap[t] = swp;
        return PU_OK;
    };
    for (int t = 0; t < n_ops; ++t) {
        const int o = pl.order[t];
        const int p = ops[3 * o], a = ops[3 * o + 1], b = ops[3 * o + 2];
        int slot = pl.store_slot[p];
        // a stored value that a later op reads back from HBM is written through the
        // caches; everything else is streamed
        if (slot >= 0 && waits[p] && !in_lds[p]) slot |= pu::kReadBack;
        if (int rc = describe(t, a, b, slot, lds_slot[p])) return rc;
    }
    if (int rc = describe(n_ops, root_a, root_b, -1, -1)) return rc;
    return PU_OK;
}

}  // namespace

int pu::check_ready(pu_ctx *c) {
    if (!c) return set_err(nullptr, PU_E_ARG, "null context");
    if (!c->have_model) return set_err(&c->err, PU_E_STATE, "pu_set_model not called");
    if (!c->have_sched) return set_err(&c->err, PU_E_STATE, "pu_set_schedule not called");
    for (int v = 0; v < c->n_nodes; ++v) {
        const int t = c->tip_slot[v];
        if (t >= 0 && c->tip_kind[t] == 0)
            return set_err(&c->err, PU_E_STATE, "tip node %d has no data", v);
    }
    return PU_OK;
}

bool pu::any_dense(const pu_ctx *c) {
    for (int k : c->tip_kind)
        if (k == 1) return true;
    return false;
}

// bring dense tip storage up to date when coded and dense tips are mixed
int pu::sync_tips(pu_ctx *c) {
    if (!any_dense(c) || !c->dense_dirty) return PU_OK;
    // an evaluation already enqueued on the context's stream may still read d_tips
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    std::vector<double> row((size_t)c->S * c->K);
    for (int t = 0; t < c->n_tips_used; ++t) {
        if (c->tip_kind[t] != 2) continue;
        const uint8_t *cd = c->h_codes.data() + (size_t)t * c->S;
        for (int64_t s = 0; s < c->S; ++s)
            memcpy(&row[(size_t)s * c->K], &c->h_table[(size_t)cd[s] * c->K],
                   sizeof(double) * c->K);
        HIPCHK(&c->err, hipMemcpy(c->d_tips + (size_t)t * c->S * c->K, row.data(),
                                  row.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    c->dense_dirty = false;
    return PU_OK;
}

namespace {

int tip_slot_for(pu_ctx *c, int node) {
    if (node < 0 || node >= c->n_nodes)
        return set_err(&c->err, PU_E_ARG, "node %d out of range [0,%d)", node, c->n_nodes);
    if (c->tip_slot[node] >= 0) return c->tip_slot[node];
    if (c->n_tips_used >= c->n_tips)
        return set_err(&c->err, PU_E_ARG, "more than n_tips=%d tip nodes", c->n_tips);
    if (c->have_sched)
        return set_err(&c->err, PU_E_STATE, "declare every tip before pu_set_schedule");
    c->tip_slot[node] = c->n_tips_used;
    return c->n_tips_used++;
}

// Tip uses in device op order (child a before child b), grouped into staging chunks of at
// most kChunkOps ops and about kChunkUses tip uses: the traversal stages one chunk's tip
// codes in LDS at a time, and the fewer bytes that takes, the more workgroups fit a CU.
// the chunking: tip uses in order (seq), first use and first op of every chunk; returns the
// largest number of uses in a chunk (>= 1)
// (a task of a split plan starts a chunk: `breaks`, ascending op indices)
// (cap: the uses target, 0 = kChunkUses; PU_CHUNK_USES overrides both)
int chunk_schedule(const std::vector<OpDesc> &descs, std::vector<int> &seq,
                   std::vector<int> &tip0, std::vector<int> &op0,
                   const std::vector<int> &breaks = {}, int cap = 0) {
    const int n = (int)descs.size();
    int maxu = 0, start = 0;
    size_t nb = 0;
    int cap_uses = cap > 0 ? cap : pu::kChunkUses;
    if (const char *env = getenv("PU_CHUNK_USES")) cap_uses = std::max(2, atoi(env));
    for (int t = 0; t < n; ++t) {
        const OpDesc &d = descs[t];
        const int uses = d.pat == pu::PAT_TT ? 2
                         : (d.pat == pu::PAT_CT || d.pat == pu::PAT_MT) ? 1 : 0;
        const bool brk = nb < breaks.size() && breaks[nb] == t;
        if (brk) ++nb;
        if (t == 0 || brk || t - start == pu::kChunkOps ||
            (int)seq.size() - tip0.back() + uses > cap_uses) {
            if (t > 0) maxu = std::max(maxu, (int)seq.size() - tip0.back());
            op0.push_back(t);
            tip0.push_back((int)seq.size());
            start = t;
        }
        if (d.pat == pu::PAT_TT) seq.push_back(d.ia);
        if (uses > 0) seq.push_back(d.ib);
    }
    maxu = std::max(maxu, (int)seq.size() - tip0.back());
    op0.push_back(n);
    tip0.push_back((int)seq.size());
    return std::max(maxu, 1);
}

// the task boundaries of a split plan (chunk breaks), ascending
std::vector<int> task_breaks(const Plan &pl) {
    std::vector<int> b;
    for (const auto &r : pl.tasks) b.push_back(r.first);
    if (!pl.tasks.empty()) b.push_back(pl.top_lo);
    return b;
}

int upload_schedule(pu_ctx *c, const Plan &pl) {
    const std::vector<OpDesc> &descs = pl.descs;
    std::vector<int> seq, tip0, op0;
    const int maxu = chunk_schedule(descs, seq, tip0, op0, task_breaks(pl), c->chunk_cap);
    c->n_chunks = (int)op0.size() - 1;
    c->max_chunk_uses = maxu;
    // tasks [chains..., top]: {op_lo, op_hi, chunk_lo, chunk_hi} (kernel: TraverseArgs::tasks)
    c->n_tasks = (int)pl.tasks.size();
    dfree(c->d_tasks);
    if (c->n_tasks > 0) {
        auto chunk_at = [&](int t) {
            return (int)(std::lower_bound(op0.begin(), op0.end(), t) - op0.begin());
        };
        std::vector<int> tk;
        for (const auto &r : pl.tasks)
            tk.insert(tk.end(), {r.first, r.second, chunk_at(r.first), chunk_at(r.second)});
        tk.insert(tk.end(), {pl.top_lo, (int)descs.size() - 1, chunk_at(pl.top_lo), c->n_chunks});
        for (size_t k = 0; k + 1 < tk.size() / 4; ++k)
            if (op0[tk[4 * k + 2]] != tk[4 * k] || op0[tk[4 * k + 3]] != tk[4 * k + 1])
                return set_err(&c->err, PU_E_SCHED, "split plan: task %zu does not start a chunk",
                               k);
        if (int rc = dalloc(&c->err, &c->d_tasks, tk.size())) return rc;
        HIPCHK(&c->err, hipMemcpy(c->d_tasks, tk.data(), tk.size() * 4, hipMemcpyHostToDevice));
        const size_t n_wt = (size_t)pu::tile_count(c->S) * c->C;
        dfree(c->d_ticket);
        if (int rc = dalloc(&c->err, &c->d_ticket, n_wt)) return rc;
        HIPCHK(&c->err, hipMemset(c->d_ticket, 0, n_wt * 4));
    }
    dfree(c->d_chunk_op0);
    if (int rc = dalloc(&c->err, &c->d_chunk_op0, op0.size())) return rc;
    HIPCHK(&c->err, hipMemcpy(c->d_chunk_op0, op0.data(), op0.size() * 4,
                              hipMemcpyHostToDevice));
    dfree(c->d_chunk_tip0);
    dfree(c->d_tip_seq);
    int rc;
    if ((rc = dalloc(&c->err, &c->d_chunk_tip0, tip0.size())) ||
        (rc = dalloc(&c->err, &c->d_tip_seq, std::max<size_t>(seq.size(), 1))))
        return rc;
    HIPCHK(&c->err, hipMemcpy(c->d_chunk_tip0, tip0.data(), tip0.size() * 4,
                              hipMemcpyHostToDevice));
    if (!seq.empty())
        HIPCHK(&c->err, hipMemcpy(c->d_tip_seq, seq.data(), seq.size() * 4,
                                  hipMemcpyHostToDevice));
    std::vector<OpDesc> dev(descs);
    // bytes of one tiled CLV slot (pu_kernels.hip: C x tiles x K x 64 doubles); for K = 20
    // the scaler slot's (C x tiles x 64 doubles), which k_prune_mfma scales by 20 itself
    const long long slot_bytes =
        (long long)c->C * pu::ctx_pitch(c) * (c->K == 20 ? 1 : c->K) * pu::kTile * 8;
    for (OpDesc &d : dev)
        d.par_off = d.par_slot >= 0 ? (long long)(d.par_slot & ~pu::kReadBack) * slot_bytes : 0;
    int used = 0;
    for (size_t k = 0; k + 1 < op0.size(); ++k)
        for (int t = op0[k]; t < op0[k + 1]; ++t) {
            dev[t].use0 = used - tip0[k];
            used += dev[t].pat == pu::PAT_TT ? 2
                    : (dev[t].pat == pu::PAT_CT || dev[t].pat == pu::PAT_MT) ? 1 : 0;
        }
    HIPCHK(&c->err, hipMemcpy(c->d_ops, dev.data(), dev.size() * sizeof(OpDesc),
                              hipMemcpyHostToDevice));
    return PU_OK;
}

// Scaler memory and its skip-zero flags back to the consistent all-zero state (a new layout)
int reset_scalers(pu_ctx *c) {
    const size_t padS = (size_t)(pu::tile_pitch(c->S) + c->pitch_pad) * pu::kTile;
    HIPCHK(&c->err, hipMemsetAsync(c->d_scale, 0, c->clv_cap * padS * c->C * 8, c->stream));
    HIPCHK(&c->err, hipMemsetAsync(c->d_root_scale, 0, padS * c->C * 8, c->stream));
    HIPCHK(&c->err, hipMemsetAsync(c->d_sflag, 0,
                                   (c->clv_cap + 1) * (size_t)pu::tile_count(c->S) * c->C * 4,
                                   c->stream));
    return PU_OK;
}

// stateless workspace per device (pu_clv / pu_lnl_node)
struct Workspace {
    std::mutex mu;
    double *buf = nullptr;
    size_t cap = 0;
    hipStream_t stream = nullptr;
};
Workspace g_ws[64];

}  // namespace

std::mutex &pu::ws_mutex(int device) { return g_ws[device].mu; }


int pu::ws_get(int device, size_t doubles, double **out, hipStream_t *st) {
    Workspace &w = g_ws[device];
    if (!w.stream) HIPCHK(nullptr, hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking));
    if (w.cap < doubles) {
        dfree(w.buf);
        w.cap = 0;
        int rc = dalloc(nullptr, &w.buf, doubles);
        if (rc) return rc;
        w.cap = doubles;
    }
    *out = w.buf;
    *st = w.stream;
    return PU_OK;
}


int pu::check_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return set_err(nullptr, PU_E_HIP, "no HIP device available");
    }
    if (device < 0 || device >= n || device >= 64)
        return set_err(nullptr, PU_E_ARG, "device %d out of range (%d devices)", device, n);
    return PU_OK;
}


int grid_of(const pu_ctx *c) { return c->grid; }

// Occupancy-aware build choice for k_prune plans outside the KEEP occupancy rule (lnL-only,
// caller orders, explicit slots).  The default build needs ~106 SGPRs: with the 16 the hardware
// adds per wave that is 6 waves per SIMD (scripts/probes/occupancy_probe.hip); the 7-wave build
// trims SGPRs with a few spills to VGPR lanes, which costs latency per op.  It is chosen only
// when it saves a round of workgroups, and only for the tip-product lnL-only variant (the one
// other variant built for 7 waves is the KEEP occupancy plan's, pu_kernels.hip).
int pick_waves(const pu_ctx *c, size_t lds, int grid) {
    if (c->K > 4) return 0;
    const size_t gran = 512, lds_cap = 160 * 1024 - 1;
    const int by_lds = lds ? (int)(lds_cap / ((lds + gran - 1) / gran * gran)) : 8;
    auto rounds = [&](int per_cu) {
        const int slots = std::max(1, std::min(per_cu, by_lds)) * c->n_cu;
        return (grid + slots - 1) / slots;
    };
    return rounds(7) < rounds(6) ? 7 : 0;
}

// ---------------------------------------------------------------- KEEP occupancy (r04)
// A DNA KEEP traversal is a store stream: every op writes each workgroup's 4 x 64 lanes x
// (K + 1) doubles once.  How fast HBM absorbs it depends on how many workgroups share a CU,
// which the LDS request sets (k per CU for a request of at most lds_cap_for(k) bytes; the
// default build's 106 SGPRs allow 6 waves per SIMD, the 7- and 8-wave builds spill SGPRs).
//
// Measured (r04 sweeps, profiles/r04_occ_*.txt; k_prune ms, min of 2-3 interleaved rounds):
// * the store stream runs fastest at 4 workgroups per CU with the spill-free default build:
//   cfg4 (1000 taxa x 125k sites, 1954 workgroups) 2.58 / 2.84-3.11 ms on two boxes, against
//   3.34-4.05 at 3, 5 or 6 per CU, 3.76 with the 8-wave build and 3.13-3.38 for the r03 split
//   plan; 200 / 500 taxa at 100k-125k sites likewise;
// * what remains is batch arithmetic.  Every CU receives n = ceil(grid / CUs) workgroups and
//   runs them in ceil(n / k) batches.  At 4 per CU, n = 5 or 6 leaves a last batch of 1-2
//   workgroups per CU that takes nearly a full batch's time (latency, not bandwidth): 50 taxa
//   at 74k-82k sites 0.104 ms at 4 per CU, 0.088-0.091 with the 7-wave build at 7 per CU (one
//   batch); 100 taxa at 75k / 90k 0.208 / 0.205 against 0.178-0.193 / 0.200.  At n = 7 the
//   last 4-per-CU batch is 3/4 full and the two are level (cfg2: 0.1173 vs 0.1220); for
//   n <= 4 or n >= 7 every k in 4..8 is within the 5-10 % that the same plan varies between
//   two allocations in one process (cfg4: 2.84 vs 3.10 ms), except the spilling 7- / 8-wave
//   builds below 4 per CU (50 taxa at 40k-65k: 0.078-0.100 vs 0.058-0.071 ms).
// So: 4 per CU and the most stash slots that fit 40 KB, unless n is 5 or 6 -- then the 7-wave
// build at 7 per CU runs every workgroup in one batch.
struct KeepOcc {
    Plan plan;
    int k = 4, L = 2, R = 0, pad = 0, waves = 1;  // L LDS stash slots, R register slots
    int n_per_cu = 0;
};

// largest LDS request (bytes, a multiple of the 512-byte allocation granule) that still lets
// k workgroups share a CU's 160 KiB
inline size_t lds_cap_for(int k) { return (size_t)(163839 / k) / 512 * 512; }

// workgroups per CU of the chosen plan (see above); n: ceil(grid / CUs)
inline int keep_per_cu(int n) { return (n == 5 || n == 6) ? 7 : 4; }

template <class LdsOf>
int keep_occupancy(pu_ctx *c, int n_ops, const int32_t *ops, int root_a, int root_b, int grid,
                   LdsOf &lds_of, KeepOcc &out) {
    constexpr int kMaxSlots = 5;
    // LDS of 1..kMaxSlots stash slots (the tip-code chunking, and so the rest of the LDS, does
    // not depend on the slot count)
    Plan p1;
    if (int rc = make_plan(c, n_ops, ops, root_a, root_b, 1, true, true, p1)) return rc;
    size_t lds[kMaxSlots + 1] = {0};
    for (int L = 1; L <= kMaxSlots; ++L) lds[L] = lds_of(p1, L);
    int forced = 0;
    if (const char *env = getenv("PU_KEEP_OCC")) forced = atoi(env);
    if (forced && (forced < 3 || forced > 7))
        return set_err(&c->err, PU_E_ARG, "PU_KEEP_OCC must be in [3, 7]");
    const int n = (grid + c->n_cu - 1) / c->n_cu;
    int best_k = 0, best_L = 0;
    for (int k : {forced ? forced : keep_per_cu(n), 4}) {  // (4: if the first does not fit)
        const size_t cap = lds_cap_for(k);
        for (int l = kMaxSlots; l >= 1 && !best_L; --l)
            if (lds[l] <= cap) best_L = l;
        if (best_L) {
            best_k = k;
            break;
        }
    }
    if (!best_k) {  // not even one slot fits (huge code tables): the planner's default
        if (int rc = make_plan(c, n_ops, ops, root_a, root_b, 0, true, true, out.plan)) return rc;
        out.k = 0;
        out.L = out.R = 0;
        out.pad = 0;
        out.waves = -1;
        return PU_OK;
    }
    // stash overflow left: the default build also keeps two waiting parents in registers
    // (TV_RSLOTS); the spilling 7- / 8-wave builds do not
    Plan pL;
    if (int rc = make_plan(c, n_ops, ops, root_a, root_b, best_L, true, true, pL)) return rc;
    const int R = (best_k <= 6 && pL.n_mem > 0) ? 2 : 0;
    if (int rc = make_plan(c, n_ops, ops, root_a, root_b, best_L + R, true, true, out.plan))
        return rc;
    out.k = best_k;
    out.L = best_L;
    out.R = R;
    // the pad from the final plan's own LDS (its chunking matches p1's, so this is lds[best_L];
    // computed again so that a planner change cannot leave the pad sized for another plan)
    const size_t lds_final = lds_of(out.plan, best_L);
    if (lds_final > lds_cap_for(best_k))
        return set_err(&c->err, PU_E_STATE, "occupancy plan: %zu LDS bytes exceed %zu", lds_final,
                       lds_cap_for(best_k));
    out.pad = (int)(lds_cap_for(best_k) - lds_final);
    out.waves = best_k <= 6 ? 1 : 7;
    out.n_per_cu = n;
    return PU_OK;
}

// ====================================================================== C ABI
// one tiled CLV slot (+ scalers) back to the reference layout [S][C][K] in host memory
int untile_out(pu_ctx *c, const double *clv, const double *scale, double *out,
               double *out_scale) {
    const size_t nV = (size_t)c->S * c->C * c->K, nS = (size_t)c->S * c->C;
    double *tmp = nullptr;
    int rc = dalloc(&c->err, &tmp, nV + nS);
    if (rc) return rc;
    hipError_t e = (hipError_t)pu::launch_untile(c->stream, c->K, c->C, c->S, pu::ctx_pitch(c),
                                                 clv, scale, tmp,
                                                 tmp + nV);
    if (e == hipSuccess) e = hipMemcpyAsync(out, tmp, nV * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && out_scale)
        e = hipMemcpyAsync(out_scale, tmp + nV, nS * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dfree(tmp);
    if (e != hipSuccess)
        return set_err(&c->err, PU_E_HIP, "partials read-back failed: %s", hipGetErrorString(e));
    return PU_OK;
}

extern "C" {

const char *pu_version(void) { return "phylo_hip 0.1 (gfx950)"; }

const char *pu_last_error(const pu_ctx *ctx) {
    if (ctx && !ctx->err.empty()) return ctx->err.c_str();
    return g_err.c_str();
}

int pu_device_count(int *n) {
    if (!n) return set_err(nullptr, PU_E_ARG, "null pointer");
    *n = 0;
    if (hipGetDeviceCount(n) != hipSuccess) {
        (void)hipGetLastError();
        *n = 0;
    }
    return PU_OK;
}

int pu_clv(int device, int K, int C, int64_t S, const double *p1, const double *p2,
           const double *clv1, const double *clv2, const double *sa, const double *sb,
           double *cml, double *out) {
    if (K < 1 || K > 64 || C < 1 || C > 64 || S < 0)
        return set_err(nullptr, PU_E_ARG, "pu_clv: bad shape K=%d C=%d S=%lld", K, C,
                       (long long)S);
    if (!p1 || !p2 || (S > 0 && (!clv1 || !clv2 || !sa || !sb || !cml || !out)))
        return set_err(nullptr, PU_E_ARG, "pu_clv: null buffer");
    int rc = check_device(device);
    if (rc) return rc;
    if (S == 0) return PU_OK;
    DeviceGuard g(device);
    std::lock_guard<std::mutex> lk(ws_mutex(device));
    const size_t nP = (size_t)C * K * K, nV = (size_t)S * C * K, nS = (size_t)S * C;
    double *w;
    hipStream_t st;
    rc = ws_get(device, 2 * nP + 3 * nV + 3 * nS, &w, &st);
    if (rc) return rc;
    double *dp1 = w, *dp2 = dp1 + nP, *da = dp2 + nP, *db = da + nV, *dout = db + nV,
           *dsa = dout + nV, *dsb = dsa + nS, *dcml = dsb + nS;
    HIPCHK(nullptr, hipMemcpyAsync(dp1, p1, nP * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(dp2, p2, nP * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(da, clv1, nV * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(db, clv2, nV * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(dsa, sa, nS * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(dsb, sb, nS * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, (hipError_t)pu::launch_clv(st, K, C, S, dp1, dp2, da, db, dsa, dsb, dcml,
                                                dout));
    HIPCHK(nullptr, hipMemcpyAsync(out, dout, nV * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(nullptr, hipMemcpyAsync(cml, dcml, nS * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(nullptr, hipStreamSynchronize(st));
    return PU_OK;
}

int pu_lnl_node(int device, int K, int C, int64_t S, const double *pi, const double *partials,
                const double *scale, double *out) {
    if (K < 1 || K > 64 || C < 1 || S < 0)
        return set_err(nullptr, PU_E_ARG, "pu_lnl_node: bad shape");
    if (!pi || (S > 0 && (!partials || !scale || !out)))
        return set_err(nullptr, PU_E_ARG, "pu_lnl_node: null buffer");
    int rc = check_device(device);
    if (rc) return rc;
    if (S == 0) return PU_OK;
    DeviceGuard g(device);
    std::lock_guard<std::mutex> lk(ws_mutex(device));
    const size_t nV = (size_t)S * C * K, nS = (size_t)S * C;
    double *w;
    hipStream_t st;
    rc = ws_get(device, K + nV + 2 * nS, &w, &st);
    if (rc) return rc;
    double *dpi = w, *dv = dpi + K, *ds = dv + nV, *dout = ds + nS;
    HIPCHK(nullptr, hipMemcpyAsync(dpi, pi, K * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(dv, partials, nV * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, hipMemcpyAsync(ds, scale, nS * 8, hipMemcpyHostToDevice, st));
    HIPCHK(nullptr, (hipError_t)pu::launch_lnl_node(st, K, C, S, dpi, dv, ds, dout));
    HIPCHK(nullptr, hipMemcpyAsync(out, dout, nS * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(nullptr, hipStreamSynchronize(st));
    return PU_OK;
}

int pu_ctx_create(pu_ctx **out, int device, int n_nodes, int n_tips, int64_t S, int C, int K,
                  int flags) {
    if (!out) return set_err(nullptr, PU_E_ARG, "null out pointer");
    *out = nullptr;
    if (n_nodes < 2 || n_tips < 2 || n_tips > n_nodes || S < 1 || C < 1 || C > 64 || K < 2)
        return set_err(nullptr, PU_E_ARG, "pu_ctx_create: bad sizes n_nodes=%d n_tips=%d "
                       "S=%lld C=%d K=%d", n_nodes, n_tips, (long long)S, C, K);
    if (!pu::traverse_supported(K))
        return set_err(nullptr, PU_E_ARG, "pu_ctx_create: n_states=%d not supported by the "
                       "traversal kernels (2, 4, 20); use pu_clv for other alphabets", K);
    if (C > 256) return set_err(nullptr, PU_E_ARG, "too many categories");
    int rc = check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    pu_ctx *c = new pu_ctx();
    c->device = device;
    c->n_nodes = n_nodes;
    c->n_tips = n_tips;
    c->S = S;
    c->C = C;
    c->K = K;
    c->flags = flags;
    hipDeviceProp_t prop;
    c->n_cu = hipGetDeviceProperties(&prop, device) == hipSuccess ? prop.multiProcessorCount : 256;
    c->tip_slot.assign(n_nodes, -1);
    c->tip_kind.assign(n_tips, 0);
    c->code_stride = (S + 63) / 64 * 64;
    // room for PU_PITCH_EXTRA's unused tiles only when the A/B knob is set at creation
    c->pitch_pad = getenv("PU_PITCH_EXTRA") ? pu::kPitchPad : 0;
    auto fail = [&](int code) {
        pu_ctx_destroy(c);
        return code;
    };
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess)
        return fail(set_err(nullptr, PU_E_HIP, "hipStreamCreate failed"));
    c->stream = c->own_stream;
    if ((rc = dalloc(nullptr, &c->d_evecs, (size_t)K * K)) ||
        (rc = dalloc(nullptr, &c->d_evals, (size_t)K)) ||
        (rc = dalloc(nullptr, &c->d_ivecs, (size_t)K * K)) ||
        (rc = dalloc(nullptr, &c->d_pi, (size_t)K)) ||
        (rc = dalloc(nullptr, &c->d_rates, (size_t)C)) ||
        (rc = dalloc(nullptr, &c->d_logw, 2 * (size_t)C)) ||  // [log w][w]
        (rc = dalloc(nullptr, &c->d_root,
                     (size_t)(pu::tile_pitch(S) + c->pitch_pad) * pu::kTile * C * K)) ||
        (rc = dalloc(nullptr, &c->d_root_scale,
                     (size_t)(pu::tile_pitch(S) + c->pitch_pad) * pu::kTile * C)) ||
        (rc = dalloc(nullptr, &c->d_site_lnl, (size_t)S)) ||
        (rc = dalloc(nullptr, &c->d_pattern_w, (size_t)S)) ||
        (rc = dalloc(nullptr, &c->d_lnl, (size_t)1)))
        return fail(rc);
    if (hipHostMalloc((void **)&c->h_lnl, sizeof(double), 0) != hipSuccess)
        return fail(set_err(nullptr, PU_E_HIP, "hipHostMalloc failed"));
    std::vector<double> ones((size_t)S, 1.0);
    c->h_pattern_w = ones;
    if (hipMemcpy(c->d_pattern_w, ones.data(), S * 8, hipMemcpyHostToDevice) != hipSuccess)
        return fail(set_err(nullptr, PU_E_HIP, "upload of pattern weights failed"));
    *out = c;
    return PU_OK;
}

void pu_ctx_destroy(pu_ctx *c) {
    if (!c) return;
    DeviceGuard g(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->d_timing && c->n_timed && c->K == 20) {  // debug: PU_TIMING
        unsigned long long h[8] = {0};
        if (hipMemcpy(h, c->d_timing, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess) {
            const double n = (double)c->n_timed * (c->n_ops + 1);
            fprintf(stderr,
                    "[pu timing] s_memtime ticks per op (one wave, %d launches): children %.0f  "
                    "P wait %.0f  MFMA %.0f  epilogue %.0f  stash+stores %.0f\n",
                    c->n_timed, h[1] / n, h[2] / n, h[3] / n, h[4] / n, h[5] / n);
        }
    }
    edge_free(c);
    dfree(c->d_tips);
    if (c->tip_store) {  // shared tips: the last holder frees them
        c->d_codes = nullptr;
        c->d_table = nullptr;
        c->d_pattern_w = nullptr;
        c->tip_store.reset();
    }
    dfree(c->d_codes);
    dfree(c->d_table);
    dfree(c->d_evecs);
    dfree(c->d_evals);
    dfree(c->d_ivecs);
    dfree(c->d_pi);
    dfree(c->d_rates);
    dfree(c->d_logw);
    dfree(c->d_ops);
    dfree(c->d_brlens);
    dfree(c->d_P);
    dfree(c->d_Pa);
    dfree(c->d_timing);
    dfree(c->d_chunk_op0);
    dfree(c->d_chunk_tip0);
    dfree(c->d_tip_seq);
    dfree(c->d_tasks);
    dfree(c->d_ticket);
    dfree(c->d_PT);
    dfree(c->d_red_slots);
    dfree(c->d_cat_lnl);
    dfree(c->d_lse_ticket);
    dfree(c->d_clv);
    dfree(c->d_scale);
    dfree(c->d_sflag);
    dfree(c->d_root);
    dfree(c->d_root_scale);
    dfree(c->d_site_lnl);
    dfree(c->d_pattern_w);
    dfree(c->d_block);
    dfree(c->d_lnl);
    if (c->h_lnl) (void)hipHostFree(c->h_lnl);
    for (auto &e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

int pu_set_tip_partials(pu_ctx *c, int node, const double *partials) {
    if (!c || !partials) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (c->tip_store)
        return set_err(&c->err, PU_E_STATE, "the tips are shared (pu_share_tips) and frozen");
    DeviceGuard g(c->device);
    const int t = tip_slot_for(c, node);
    if (t < 0) return t;
    if (!c->d_tips) {
        int rc = dalloc(&c->err, &c->d_tips, (size_t)c->n_tips * c->S * c->K);
        if (rc) return rc;
        c->dense_dirty = true;  // previously coded tips need expanding
    }
    // an evaluation already enqueued on the context's stream may still read d_tips
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    HIPCHK(&c->err, hipMemcpy(c->d_tips + (size_t)t * c->S * c->K, partials,
                              (size_t)c->S * c->K * 8, hipMemcpyHostToDevice));
    c->tip_kind[t] = 1;
    return PU_OK;
}

int pu_set_code_table(pu_ctx *c, int n_codes, const double *table) {
    if (!c || !table || n_codes < 1 || n_codes > 256)
        return set_err(c ? &c->err : nullptr, PU_E_ARG, "bad code table (n_codes=%d)", n_codes);
    if (c->tip_store)
        return set_err(&c->err, PU_E_STATE, "the tips are shared (pu_share_tips) and frozen");
    DeviceGuard g(c->device);
    for (int t = 0; t < c->n_tips_used; ++t)
        if (c->tip_kind[t] == 2)
            return set_err(&c->err, PU_E_STATE, "code table set after coded tips");
    dfree(c->d_table);
    int rc = dalloc(&c->err, &c->d_table, (size_t)n_codes * c->K);
    if (rc) return rc;
    HIPCHK(&c->err, hipMemcpy(c->d_table, table, (size_t)n_codes * c->K * 8,
                              hipMemcpyHostToDevice));
    c->h_table.assign(table, table + (size_t)n_codes * c->K);
    c->n_codes = n_codes;
    return PU_OK;
}

int pu_set_tip_codes(pu_ctx *c, int node, const uint8_t *codes) {
    if (!c || !codes) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (c->n_codes == 0) return set_err(&c->err, PU_E_STATE, "pu_set_code_table first");
    if (c->tip_store)
        return set_err(&c->err, PU_E_STATE, "the tips are shared (pu_share_tips) and frozen");
    for (int64_t s = 0; s < c->S; ++s)
        if (codes[s] >= c->n_codes)
            return set_err(&c->err, PU_E_ARG, "code %d at site %lld >= n_codes %d", codes[s],
                           (long long)s, c->n_codes);
    DeviceGuard g(c->device);
    const int t = tip_slot_for(c, node);
    if (t < 0) return t;
    if (!c->d_codes) {
        int rc = dalloc(&c->err, &c->d_codes, (size_t)c->n_tips * c->code_stride);
        if (rc) return rc;
        HIPCHK(&c->err, hipMemset(c->d_codes, 0, (size_t)c->n_tips * c->code_stride));
        c->h_codes.assign((size_t)c->n_tips * c->S, 0);
    }
    memcpy(c->h_codes.data() + (size_t)t * c->S, codes, c->S);
    // an evaluation already enqueued on the context's stream may still read d_codes
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    HIPCHK(&c->err, hipMemcpy(c->d_codes + (size_t)t * c->code_stride, codes, c->S,
                              hipMemcpyHostToDevice));
    c->tip_kind[t] = 2;
    c->dense_dirty = true;
    return PU_OK;
}

int pu_set_tips(pu_ctx *c, int n_tips, const int32_t *nodes, int n_codes,
                const double *code_table, const uint8_t *codes, const double *partials,
                const double *pattern_weights) {
    if (!c || n_tips < 0 || (n_tips > 0 && !nodes) || (!codes == !partials))
        return set_err(c ? &c->err : nullptr, PU_E_ARG,
                       "pu_set_tips: give tip nodes and exactly one of codes / partials");
    int rc;
    if (codes) {
        if (!code_table) return set_err(&c->err, PU_E_ARG, "pu_set_tips: codes need a table");
        if ((rc = pu_set_code_table(c, n_codes, code_table))) return rc;
        for (int i = 0; i < n_tips; ++i)
            if ((rc = pu_set_tip_codes(c, nodes[i], codes + (size_t)i * c->S))) return rc;
    } else {
        const size_t per = (size_t)c->S * c->K;
        for (int i = 0; i < n_tips; ++i)
            if ((rc = pu_set_tip_partials(c, nodes[i], partials + (size_t)i * per))) return rc;
    }
    return pattern_weights ? pu_set_pattern_weights(c, pattern_weights) : PU_OK;
}

int pu_set_tip_nodes(pu_ctx *c, int n, const int32_t *nodes) {
    if (!c || !nodes) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (n != c->n_tips_used)
        return set_err(&c->err, PU_E_ARG, "pu_set_tip_nodes: %d nodes for %d tips set", n,
                       c->n_tips_used);
    std::vector<int> ts(c->n_nodes, -1);
    for (int i = 0; i < n; ++i) {
        const int v = nodes[i];
        if (v < 0 || v >= c->n_nodes) return set_err(&c->err, PU_E_ARG, "node %d out of range", v);
        if (ts[v] >= 0) return set_err(&c->err, PU_E_ARG, "node %d given twice", v);
        ts[v] = i;
    }
    c->tip_slot.swap(ts);  // the tip data stay in their slots
    c->have_sched = false;  // a new topology needs its schedule
    c->ran = false;
    return PU_OK;
}

int pu_share_tips(pu_ctx *c, pu_ctx *owner, int n, const int32_t *nodes) {
    if (!c || !owner || !nodes || c == owner)
        return set_err(c ? &c->err : nullptr, PU_E_ARG, "pu_share_tips: bad arguments");
    if (owner->device != c->device || owner->n_tips != c->n_tips || owner->S != c->S ||
        owner->K != c->K)
        return set_err(&c->err, PU_E_ARG, "pu_share_tips: device/n_tips/S/K %d/%d/%lld/%d vs "
                       "the owner's %d/%d/%lld/%d", c->device, c->n_tips, (long long)c->S, c->K,
                       owner->device, owner->n_tips, (long long)owner->S, owner->K);
    if (c->n_tips_used || c->d_codes || c->d_tips || c->tip_store)
        return set_err(&c->err, PU_E_STATE, "pu_share_tips: the context already has tips");
    if (n != owner->n_tips_used || n < 1 || !owner->d_codes)
        return set_err(&c->err, PU_E_ARG, "pu_share_tips: %d nodes for the owner's %d coded "
                       "tips", n, owner->n_tips_used);
    for (int t = 0; t < n; ++t)
        if (owner->tip_kind[t] != 2)
            return set_err(&c->err, PU_E_ARG, "pu_share_tips: owner tip slot %d is not coded", t);
    std::vector<int> ts(c->n_nodes, -1);
    for (int i = 0; i < n; ++i) {
        const int v = nodes[i];
        if (v < 0 || v >= c->n_nodes) return set_err(&c->err, PU_E_ARG, "node %d out of range", v);
        if (ts[v] >= 0) return set_err(&c->err, PU_E_ARG, "node %d given twice", v);
        ts[v] = i;
    }
    DeviceGuard g(c->device);
    if (!owner->tip_store) {  // the owner's buffers move into a store both contexts hold
        // an evaluation already enqueued on the owner's stream reads them where they are
        auto st = std::make_shared<pu::TipStore>();
        st->device = owner->device;
        st->first = owner;
        st->codes = owner->d_codes;
        st->table = owner->d_table;
        st->pattern_w = owner->d_pattern_w;
        owner->tip_store = st;
    }
    // an evaluation enqueued on this context may still read its own weights
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    dfree(c->d_pattern_w);
    c->tip_store = owner->tip_store;
    c->d_codes = owner->d_codes;
    c->d_table = owner->d_table;
    c->d_pattern_w = owner->d_pattern_w;
    c->h_pattern_w = owner->h_pattern_w;
    c->h_table = owner->h_table;
    c->n_codes = owner->n_codes;
    c->code_stride = owner->code_stride;
    c->n_tips_used = n;
    c->tip_kind.assign(owner->tip_kind.begin(), owner->tip_kind.end());
    c->tip_slot.swap(ts);
    c->dense_dirty = false;
    c->have_sched = false;
    c->ran = false;
    return PU_OK;
}

int pu_set_pattern_weights(pu_ctx *c, const double *w) {
    if (!c || !w) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (c->tip_store)
        return set_err(&c->err, PU_E_STATE, "the tips are shared (pu_share_tips) and frozen");
    DeviceGuard g(c->device);
    // an evaluation already enqueued on the context's stream may still read the weights
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    HIPCHK(&c->err, hipMemcpy(c->d_pattern_w, w, (size_t)c->S * 8, hipMemcpyHostToDevice));
    c->h_pattern_w.assign(w, w + c->S);
    return PU_OK;
}

// the model parts that do not come from an eigen-decomposition (pu_set_model_p)
static int set_model_common(pu_ctx *c, const double *freqs, const double *rates,
                            const double *weights) {
    std::vector<double> logw(2 * (size_t)c->C);  // [log w][w] (d_logw)
    for (int k = 0; k < c->C; ++k) {
        if (!(weights[k] >= 0) || !(rates[k] >= 0))
            return set_err(&c->err, PU_E_ARG, "negative or NaN rate/weight in category %d", k);
        logw[k] = log(weights[k]);
        logw[c->C + k] = weights[k];
    }
    HIPCHK(&c->err, hipMemcpy(c->d_pi, freqs, (size_t)c->K * 8, hipMemcpyHostToDevice));
    HIPCHK(&c->err, hipMemcpy(c->d_rates, rates, (size_t)c->C * 8, hipMemcpyHostToDevice));
    c->h_rates.assign(rates, rates + c->C);
    HIPCHK(&c->err, hipMemcpy(c->d_logw, logw.data(), 2 * (size_t)c->C * 8,
                              hipMemcpyHostToDevice));
    return PU_OK;
}

int pu_set_model(pu_ctx *c, const double *evecs, const double *evals, const double *ivecs,
                 const double *freqs, const double *rates, const double *weights) {
    if (!c || !evecs || !evals || !ivecs || !freqs || !rates || !weights)
        return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    DeviceGuard g(c->device);
    // an enqueued evaluation may still read the model (k_pmatrix, pi, weights)
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    const int K = c->K;
    if (int rc = set_model_common(c, freqs, rates, weights)) return rc;
    HIPCHK(&c->err, hipMemcpy(c->d_evecs, evecs, (size_t)K * K * 8, hipMemcpyHostToDevice));
    HIPCHK(&c->err, hipMemcpy(c->d_evals, evals, (size_t)K * 8, hipMemcpyHostToDevice));
    HIPCHK(&c->err, hipMemcpy(c->d_ivecs, ivecs, (size_t)K * K * 8, hipMemcpyHostToDevice));
    c->h_eig.assign(evecs, evecs + (size_t)K * K);
    c->h_eig.insert(c->h_eig.end(), evals, evals + K);
    c->h_eig.insert(c->h_eig.end(), ivecs, ivecs + (size_t)K * K);
    c->have_model = true;
    c->host_p = false;  // back to P = evecs diag(exp(evals r t)) ivecs on the device
    return PU_OK;
}

int pu_set_model_p(pu_ctx *c, const double *freqs, const double *rates, const double *weights) {
    if (!c || !freqs || !rates || !weights)
        return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    DeviceGuard g(c->device);
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    if (int rc = set_model_common(c, freqs, rates, weights)) return rc;
    c->have_model = true;
    c->host_p = true;
    c->p_fresh = false;
    return PU_OK;
}

int pu_set_pmatrices(pu_ctx *c, const double *P) {
    if (!c || !P) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (!c->have_sched) return set_err(&c->err, PU_E_STATE, "pu_set_schedule first");
    if (!c->host_p) return set_err(&c->err, PU_E_STATE, "pu_set_model_p first");
    DeviceGuard g(c->device);
    const size_t per = 2 * (size_t)c->C * c->K * c->K, half = per / 2;
    for (size_t i = 0; i < per * ((size_t)c->n_ops + 1); ++i)
        if (!std::isfinite(P[i]))
            return set_err(&c->err, PU_E_ARG, "non-finite transition probability at %zu", i);
    // caller op order and child order -> the device's (the inverse of pu_get_pmatrices)
    std::vector<double> dev(per * ((size_t)c->n_ops + 1));
    auto put = [&](int t, int o) {
        const int sw = c->swap[t];
        memcpy(dev.data() + per * t + half * sw, P + per * o, half * 8);
        memcpy(dev.data() + per * t + half * (1 - sw), P + per * o + half, half * 8);
    };
    for (int t = 0; t < c->n_ops; ++t) put(t, c->perm[t]);
    put(c->n_ops, c->n_ops);
    // an enqueued evaluation may still read the previous matrices
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    if (int rc = pu::ensure_host_p(c)) return rc;
    HIPCHK(&c->err, hipMemcpy(c->d_P, dev.data(), dev.size() * 8, hipMemcpyHostToDevice));
    c->p_fresh = true;
    return PU_OK;
}

int pu_set_pmatrix_provider(pu_ctx *c, pu_pmat_provider fn, void *user) {
    if (!c) return set_err(nullptr, PU_E_ARG, "null context");
    c->pm_fn = fn;
    c->pm_user = user;
    return PU_OK;
}

}  // extern "C"

int pu::provide(pu_ctx *c, int order, int n, const double *t, double *out) {
    if (!c->pm_fn)
        return set_err(&c->err, PU_E_STATE, "this context runs on host transition matrices: "
                       "pu_set_pmatrix_provider first");
    if (c->pm_fn(c->pm_user, order, n, t, out))
        return set_err(&c->err, PU_E_STATE, "the transition-matrix provider failed");
    const size_t m = (size_t)n * c->C * c->K * c->K;
    for (size_t i = 0; i < m; ++i)
        if (!std::isfinite(out[i]))
            return set_err(&c->err, PU_E_ARG, "provider: non-finite matrix entry %zu", i);
    return PU_OK;
}

int pu::ensure_host_p(pu_ctx *c) {
    if (c->d_P || !c->have_sched) return PU_OK;
    return dalloc(&c->err, &c->d_P, 2 * ((size_t)c->n_ops + 1) * c->C * c->K * c->K);
}

int pu::refresh_host_p(pu_ctx *c) {
    if (!c->host_p || c->p_fresh || !c->pm_fn) return PU_OK;
    if (int rc = ensure_host_p(c)) return rc;
    const int n = 2 * (c->n_ops + 1);
    std::vector<double> P((size_t)n * c->C * c->K * c->K);
    if (int rc = provide(c, 0, n, c->h_brlens.data(), P.data())) return rc;
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));  // queued work may still read d_P
    HIPCHK(&c->err, hipMemcpy(c->d_P, P.data(), P.size() * 8, hipMemcpyHostToDevice));
    c->p_fresh = true;
    return PU_OK;
}

extern "C" {

int pu_set_branch_lengths(pu_ctx *c, const double *brlens, double root_len) {
    if (!c || (!brlens && c->n_ops > 0))
        return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (!c->have_sched) return set_err(&c->err, PU_E_STATE, "pu_set_schedule first");
    DeviceGuard g(c->device);
    std::vector<double> bl(2 * ((size_t)c->n_ops + 1));
    for (int t = 0; t < c->n_ops; ++t) {
        const int sw = c->swap[t];
        bl[2 * t + sw] = brlens[2 * c->perm[t]];
        bl[2 * t + 1 - sw] = brlens[2 * c->perm[t] + 1];
    }
    const int sw = c->swap[c->n_ops];
    bl[2 * c->n_ops + sw] = 0.0;  // P(0) on root_a, tree_model.py:189
    bl[2 * c->n_ops + 1 - sw] = root_len;
    c->h_brlens = bl;
    // the unrooted topology with its lengths, for the edge operations (pu_edge.cpp)
    c->parent.assign(c->n_nodes, -1);
    c->up_len.assign(c->n_nodes, 0.0);
    for (int o = 0; o < c->n_ops; ++o) {
        const int p = c->ops_in[3 * o];
        for (int k = 0; k < 2; ++k) {
            c->parent[c->ops_in[3 * o + 1 + k]] = p;
            c->up_len[c->ops_in[3 * o + 1 + k]] = brlens[2 * o + k];
        }
    }
    c->parent[c->root_a] = c->root_b;
    c->parent[c->root_b] = c->root_a;
    c->up_len[c->root_a] = c->up_len[c->root_b] = root_len;
    HIPCHK(&c->err, hipMemcpyAsync(c->d_brlens, bl.data(), bl.size() * 8, hipMemcpyHostToDevice,
                                   c->stream));
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    c->lengths_dirty = false;
    c->p_fresh = false;  // host-supplied P (pu_set_pmatrices) belong to the old lengths
    return PU_OK;
}

int pu_set_schedule(pu_ctx *c, int n_ops, const int32_t *ops, const double *brlens,
                    int root_a, int root_b, double root_len) {
    if (!c || n_ops < 0 || (n_ops > 0 && (!ops || !brlens)))
        return set_err(c ? &c->err : nullptr, PU_E_ARG, "bad schedule arguments");
    DeviceGuard g(c->device);
    // nodes that no op produces must be declared tips
    std::vector<char> produced(c->n_nodes, 0);
    for (int o = 0; o < n_ops; ++o)
        if (ops[3 * o] >= 0 && ops[3 * o] < c->n_nodes) produced[ops[3 * o]] = 1;
    auto check_leaf = [&](int v) -> int {
        if (v < 0 || v >= c->n_nodes) return PU_OK;  // range errors reported by the planner
        if (!produced[v] && c->tip_slot[v] < 0)
            return set_err(&c->err, PU_E_SCHED, "node %d is read but is neither produced by "
                           "an op nor a declared tip", v);
        return PU_OK;
    };
    for (int o = 0; o < n_ops; ++o) {
        int rc = check_leaf(ops[3 * o + 1]);
        if (!rc) rc = check_leaf(ops[3 * o + 2]);
        if (rc) return rc;
    }
    if (int rc = check_leaf(root_a)) return rc;
    if (int rc = check_leaf(root_b)) return rc;
    const bool keep = !(c->flags & PU_LNL_ONLY);
    const bool reorder = !(c->flags & PU_NO_REORDER);
    Plan pl;
    int L = c->K == 20 ? 3 : 2;
    if (const char *env = getenv("PU_LDS_SLOTS")) L = atoi(env);
    if (L < 0 || L > 8) return set_err(&c->err, PU_E_ARG, "PU_LDS_SLOTS must be in [0, 8]");
    // protein KEEP traversals: chain tasks + a top task (make_plan).  cfg3 (2512 waves, 2.45
    // per SIMD): 0.380 -> 0.330 ms with a target of n_ops / 3 (r03 sweep of 2 / 3 / 4 / 8);
    // 12288 sites (exactly 3 waves per SIMD) unchanged.  PU_SPLIT=0 or 1: one task.
    // DNA plans: see the occupancy rule below
    int split = c->K == 20 ? 3 : 0;
    const char *split_env = getenv("PU_SPLIT");
    if (split_env) split = atoi(split_env);
    // (the protein kernel's wait-for-zero check mode has no chain tasks)
    if (c->K == 20 && getenv("PU_FORCE_GENERIC")) split = 0;
    int rc = make_plan(c, n_ops, ops, root_a, root_b, L, reorder, keep, pl, split);
    if (rc) return rc;
    // Occupancy.  When the default plan needs a second round of workgroups (cfg4's 125k-site
    // shard), a KEEP plan of >= 128 ops is split into chain tasks of about 100 ops (a split
    // plan's grid is dealt in many short rounds, so two stash slots and the default build no
    // longer cost a round): cfg4 4.16-4.30 -> 3.29-3.61 ms (r03 sweep: targets n/2..n/16, 0-3
    // slots, 1 / 7 / 8 waves); at 125k sites 200 / 400 taxa 0.849 -> 0.758 / 1.609 -> 1.493 ms,
    // 100 taxa even, 50 taxa (131k sites) 0.213 -> 0.282 ms, hence the 128-op floor.
    // Otherwise (short trees, lnL-only, caller order) a plan with one stash slot and the 8-wave
    // build may fit the grid in one round (r02: cfg4 4.58 -> 4.31 ms); cfg2 fits one round with
    // the default plan.
    int auto_waves = -1;
    int auto_pad = 0;
    int r_slots = 0;  // stash slots held in registers (TV_RSLOTS)
    const bool coded_tips = !any_dense(c);
    auto lds_of = [&](const Plan &p, int nl) {
        std::vector<int> s1, t1, o1;
        return pu::traverse_lds_bytes(c->K, c->C, c->n_codes,
                                      chunk_schedule(p.descs, s1, t1, o1), coded_tips, nl);
    };
    // DNA KEEP plans (r04): an occupancy plan -- k workgroups per CU, the most LDS stash slots
    // that fit k, the build that allows k -- chosen by keep_occupancy (below).  PU_KEEP_OCC=k
    // forces k (sweeps); the env overrides of the slots, split, waves or pad bypass it.
    const bool occ_plan = keep && c->K <= 4 && reorder && !getenv("PU_LDS_SLOTS") && !split_env &&
                          !getenv("PU_LDS_PAD");
    if (occ_plan) {
        const int grid = (int)((pu::tile_count(c->S) * c->C + 3) / 4);
        KeepOcc oc;
        if ((rc = keep_occupancy(c, n_ops, ops, root_a, root_b, grid, lds_of, oc))) return rc;
        pl = std::move(oc.plan);
        L = oc.L;
        auto_pad = oc.pad;
        auto_waves = oc.waves;
        r_slots = oc.R;
        if (getenv("PU_DEBUG_PLAN"))
            fprintf(stderr, "[pu plan] KEEP S=%lld ops=%d grid=%d: %d per CU, %d stash slots "
                    "+ %d register slots (%d read-backs), build %d, pad %d B (%d workgroups per "
                    "CU in all)\n", (long long)c->S, n_ops, grid, oc.k, oc.L, oc.R, pl.n_mem,
                    oc.waves, oc.pad, oc.n_per_cu);
    } else if (!getenv("PU_LDS_SLOTS") && c->K <= 4 && L > 1) {
        const int grid = (int)((pu::tile_count(c->S) * c->C + 3) / 4);
        auto rounds = [&](size_t lds, int per_cu) {
            const size_t gran = 512, cap = 160 * 1024 - 1;
            const int by_lds = (int)(cap / ((lds + gran - 1) / gran * gran));
            const int slots = std::max(1, std::min(per_cu, by_lds)) * c->n_cu;
            return (grid + slots - 1) / slots;
        };
        const size_t lds_def = lds_of(pl, L);
        if (std::min(rounds(lds_def, 6), rounds(lds_def, 7)) > 1) {
            Plan p1;
            if (reorder && !split_env && n_ops >= 128 &&
                make_plan(c, n_ops, ops, root_a, root_b, L, reorder, keep, p1,
                          std::max(2, n_ops / 100)) == PU_OK &&
                !p1.tasks.empty()) {
                pl = std::move(p1);
                auto_waves = 1;  // the default build
            }
        }
    }
    // Protein plans (r05 late): the kernel's 114-119 VGPRs allow 4 waves per SIMD, but 3 LDS
    // stash slots (36 KB) + the code table + a chunk of ~32 tip uses' codes take just over
    // 40 KB, so only 3 workgroups fit a CU.  Shorter staging chunks (more, cheaper barriers)
    // fit the fourth: cfg3 traversal 0.325-0.327 -> 0.316-0.318 ms at 8 uses per chunk on one
    // box (scripts/r05/exp39_cfg3_chunks.sh).  The largest chunk target >= 8 that fits 4 per CU.
    c->chunk_cap = 0;
    if (c->K == 20 && coded_tips && !getenv("PU_CHUNK_USES")) {
        auto lds_at = [&](int cap) {
            std::vector<int> s1, t1, o1;
            return pu::traverse_lds_bytes(20, c->C, c->n_codes,
                                          chunk_schedule(pl.descs, s1, t1, o1, task_breaks(pl), cap),
                                          true, L);
        };
        // 4 per CU, measured (scripts/r05/exp47_cfg3_occupancy.sh: resident waves per CU from
        // SQ_WAVE_CYCLES / SQ_BUSY_CU_CYCLES): 40.6 KB of dynamic LDS (8 uses) fits 4, 40.9 KB
        // (13 uses) does not -- so the kernel's static LDS and a 1 KB margin are counted
        auto fits4 = [](size_t lds) { return 4 * ((lds + 64 + 255) / 256 * 256) <= 163840 - 1024; };
        if (!fits4(lds_at(pu::kChunkUses)))
            for (int cap = pu::kChunkUses - 1; cap >= 8; --cap)
                if (fits4(lds_at(cap))) {
                    c->chunk_cap = cap;
                    break;
                }
    }
    // (re)allocate schedule-sized buffers
    dfree(c->d_ops);
    dfree(c->d_brlens);
    dfree(c->d_P);
    dfree(c->d_Pa);
    const size_t KK = (size_t)c->K * c->K;
    if ((rc = dalloc(&c->err, &c->d_ops, (size_t)n_ops + 1)) ||
        (rc = dalloc(&c->err, &c->d_brlens, 2 * ((size_t)n_ops + 1))) ||
        // plain P: every model but the protein eigen path, whose P launch writes only the
        // MFMA A operands (host matrices allocate it on demand: pu::ensure_host_p)
        ((!(c->K == 20 && pu::pmatrix_writes_pa(c->K)) || c->host_p) &&
         (rc = dalloc(&c->err, &c->d_P, 2 * ((size_t)n_ops + 1) * c->C * KK))))
        return rc;
    if (c->K == 20 && (rc = dalloc(&c->err, &c->d_Pa, 2 * ((size_t)n_ops + 1) * c->C * 640)))
        return rc;
    const int64_t n_tiles = pu::tile_count(c->S);
    // sites per (slot, category) layout row at the largest pitch the trial may pick
    const size_t padS = (size_t)(pu::tile_pitch(c->S) + c->pitch_pad) * pu::kTile;
    if ((size_t)pl.n_store > c->clv_cap || !c->d_sflag) {
        dfree(c->d_clv);
        dfree(c->d_scale);
        dfree(c->d_sflag);
        c->clv_cap = 0;
        const size_t cap = std::max(pl.n_store, 1);
        const size_t nflag = (cap + 1) * (size_t)n_tiles * c->C;
        if ((rc = dalloc(&c->err, &c->d_clv, cap * padS * c->C * c->K)) ||
            (rc = dalloc(&c->err, &c->d_scale, cap * padS * c->C)) ||
            (rc = dalloc(&c->err, &c->d_sflag, nflag)))
            return rc;
        // scaler memory and its flags start consistent: all zero
        HIPCHK(&c->err, hipMemset(c->d_scale, 0, cap * padS * c->C * 8));
        HIPCHK(&c->err, hipMemset(c->d_root_scale, 0, padS * c->C * 8));
        HIPCHK(&c->err, hipMemset(c->d_sflag, 0, nflag * 4));
        c->clv_cap = cap;
    }
    const int n_block = pu::traverse_block_sums(c->K, c->C, c->S);
    if (n_block > c->block_cap) {
        dfree(c->d_block);
        if ((rc = dalloc(&c->err, &c->d_block, (size_t)n_block))) return rc;
        c->block_cap = n_block;
    }
    if (pu::traverse_per_category(c->K, c->C) && !c->d_cat_lnl)
        if ((rc = dalloc(&c->err, &c->d_cat_lnl, padS * c->C))) return rc;
    if (pu::traverse_lse_in_kernel(c->K) && !c->d_lse_ticket) {  // [n_tiles] + the grid ticket
        if ((rc = dalloc(&c->err, &c->d_lse_ticket, (size_t)n_tiles + 1))) return rc;
        HIPCHK(&c->err, hipMemset(c->d_lse_ticket, 0, ((size_t)n_tiles + 1) * 4));
    }
    const int grid = (int)((n_tiles * c->C + 3) / 4);
    // skip-zero scalers need one writer per slot and run (kept partials); HBM read-backs
    // need the general kernel variant
    int variant = keep ? pu::TV_SKIP_ZERO_SCALE : 0;
    for (const OpDesc &d : pl.descs)  // (the K = 20 kernel reads back in every mode)
        if (c->K != 20 && (d.pat == pu::PAT_MC || d.pat == pu::PAT_MT || d.pat == pu::PAT_MM))
            variant |= pu::TV_GENERIC;
    if (getenv("PU_FORCE_GENERIC")) variant |= pu::TV_GENERIC;
    // a split DNA plan: the top task reads the chain roots back (K = 20: a.tasks selects it)
    if (c->K != 20 && !pl.tasks.empty()) variant |= pu::TV_GENERIC | pu::TV_CHAIN;
    // the protein kernel's waits count on every op storing its parent (KEEP)
    bool all_store = true;
    for (int t = 0; t < n_ops; ++t) all_store &= pl.descs[t].par_slot >= 0;
    if (all_store) variant |= pu::TV_KEEP;
    if (r_slots) variant |= pu::TV_RSLOTS;

    // layout pitch (r05 A/B knob): PU_PITCH_EXTRA unused tiles more per layout row; a pitch
    // other than the previous schedule's moves the scaler rows, so their flags start again
    {
        const int prev = c->pitch_extra;
        c->pitch_extra = 0;
        if (const char *fix = getenv("PU_PITCH_EXTRA"))
            c->pitch_extra = std::max(0, std::min(c->pitch_pad - 1, atoi(fix)));
        if (c->pitch_extra != prev && c->d_sflag && (rc = reset_scalers(c))) return rc;
    }
    if ((rc = upload_schedule(c, pl))) return rc;
    c->n_mem = pl.n_mem;
    c->n_tip_uses = pl.n_tip;
    c->n_store_ops = 0;
    for (int t = 0; t < n_ops; ++t) c->n_store_ops += pl.descs[t].par_slot >= 0;
    c->n_lds = L;
    // experiment knobs (scripts/sweep.py), latched with the schedule
    c->lds_pad = getenv("PU_LDS_PAD") ? atoi(getenv("PU_LDS_PAD")) : auto_pad;
    c->waves = auto_waves;  // -1: pick_waves at enqueue
    c->swap = pl.swap;
    c->grid = grid;
    c->n_tiles = (int)n_tiles;
    c->variant = variant;
    c->n_ops = n_ops;
    c->n_store = pl.n_store;
    c->perm = pl.order;
    c->store_slot = pl.store_slot;
    c->ops_in.assign(ops, ops + 3 * (size_t)n_ops);
    c->root_a = root_a;
    c->root_b = root_b;
    c->have_sched = true;
    c->ran = false;
    return pu_set_branch_lengths(c, brlens, root_len);
}

}  // extern "C"

// Everything a traversal launch needs, checked and built before any device work of the
// launch (pu_enqueue, pu_batch_enqueue): provider matrices refreshed, tips synced, the
// tip-product buffer sized, the P and traversal arguments
int pu::prepare_launch(pu_ctx *c, LaunchPlan &L) {
    int rc = check_ready(c);
    if (rc) return rc;
    c->lnl_batch = nullptr;  // this launch's lnL lands in the context's own output
    if ((rc = pu::flush_lengths(c))) return rc;  // lengths moved by pu_optimise_edge
    // host matrices: regenerated from the provider when one is set and the lengths moved;
    // otherwise refused before any device work or profiling event
    if ((rc = pu::refresh_host_p(c))) return rc;
    if (c->host_p && !c->p_fresh)
        return set_err(&c->err, PU_E_STATE, "host transition matrices are stale: "
                       "pu_set_pmatrices after pu_set_schedule / pu_set_branch_lengths");
    if ((rc = sync_tips(c))) return rc;
    const bool coded = !any_dense(c);
    int variant = c->variant;
    // lnL-only coded DNA: a tip child's product P * table[code] comes from PT, built in the P
    // launch (k_pmatrix_lane), instead of K^2 FMAs per tip child in the traversal
    const bool ptip = c->K <= 4 && coded && (c->flags & PU_LNL_ONLY) && !c->host_p &&
                      c->n_codes > 0 && !(variant & pu::TV_SKIP_ZERO_SCALE) &&
                      !getenv("PU_NO_PTIP");
    if (ptip) {
        const size_t need = 2 * ((size_t)c->n_ops + 1) * c->C * c->n_codes * c->K;
        if (need > c->pt_cap) {
            dfree(c->d_PT);
            c->pt_cap = 0;
            if ((rc = dalloc(&c->err, &c->d_PT, need))) return rc;
            c->pt_cap = need;
        }
        variant |= pu::TV_PTIP;
    }
    const size_t lds = pu::traverse_lds_bytes(c->K, c->C, c->n_codes, c->max_chunk_uses, coded,
                                              c->n_lds);
    if (lds > 160 * 1024)
        return set_err(&c->err, PU_E_ARG, "LDS request %zu exceeds 160 KiB", lds);
    pu::PmatArgs &pa = L.pa;
    pa = pu::PmatArgs();
    pa.K = c->K;
    pa.C = c->C;
    pa.n_sides = 2 * (c->n_ops + 1);
    pa.evecs = c->d_evecs;
    pa.evals = c->d_evals;
    pa.ivecs = c->d_ivecs;
    pa.brlens = c->d_brlens;
    pa.rates = c->d_rates;
    pa.P = c->d_P;
    pa.Pa = c->K == 20 ? c->d_Pa : nullptr;  // K = 20: the A operands in the same launch
    if (ptip) {
        pa.PT = c->d_PT;
        pa.table = c->d_table;
        pa.n_codes = c->n_codes;
    }
    pu::TraverseArgs &a = L.a;
    a = pu::TraverseArgs();
    a.ops = c->d_ops;
    a.chunk_op0 = c->d_chunk_op0;
    a.chunk_tip0 = c->d_chunk_tip0;
    a.tip_seq = c->d_tip_seq;
    a.n_ops = c->n_ops;
    a.n_chunks = c->n_chunks;
    a.max_chunk_uses = c->max_chunk_uses;
    a.C = c->C;
    a.T = pu::tiles_per_block(c->C);
    a.n_codes = coded ? c->n_codes : 0;
    a.n_tiles = c->n_tiles;
    a.tile_pitch = (int)pu::ctx_pitch(c);
    a.n_store = (int)c->clv_cap;
    a.S = c->S;
    a.code_stride = c->code_stride;
    a.P = c->d_P;
    a.Pa = c->d_Pa;
    a.pa_ready = (!c->host_p && c->d_Pa && pu::pmatrix_writes_pa(c->K)) ? 1 : 0;
    a.PT = ptip ? c->d_PT : nullptr;
    a.tasks = c->n_tasks > 0 ? c->d_tasks : nullptr;
    a.n_tasks = c->n_tasks;
    a.ticket = c->d_ticket;
    a.table = c->d_table;
    a.codes = c->d_codes;
    a.tips = c->d_tips;
    a.clv = c->d_clv;
    a.scale = c->d_scale;
    a.root_clv = c->d_root;
    a.root_scale = c->d_root_scale;
    a.pi = c->d_pi;
    a.logw = c->d_logw;
    a.pattern_w = c->d_pattern_w;
    a.site_lnl = c->d_site_lnl;
    a.block_sum = c->d_block;
    a.sflag = c->d_sflag;
    a.cat_lnl = pu::traverse_per_category(c->K, c->C) ? c->d_cat_lnl : nullptr;
    a.lse_ticket = pu::traverse_lse_in_kernel(c->K) ? c->d_lse_ticket : nullptr;
    // K = 20: the traversal's last tile also writes the lnL (no k_reduce launch)
    double *lnl_dst = c->d_lnl_ext ? c->d_lnl_ext : c->d_lnl;
    a.lnl_out = a.lse_ticket ? lnl_dst : nullptr;
    a.n_lds = c->n_lds;
    a.lds_pad = c->lds_pad;
    a.waves = c->waves >= 0 ? c->waves : pick_waves(c, lds, grid_of(c));
    a.timing = nullptr;
    {
        const size_t padS = (size_t)(pu::tile_pitch(c->S) + c->pitch_pad) * pu::kTile,
                     KK = (size_t)c->K * c->K;
        a.pa_bytes = c->d_Pa ? 2 * ((size_t)c->n_ops + 1) * c->C * 640 * 8 : 0;
        a.clv_bytes = c->clv_cap * padS * c->C * c->K * 8;
        a.scale_bytes = c->clv_cap * padS * c->C * 8;
        a.root_bytes = padS * c->C * c->K * 8;
        a.root_scale_bytes = padS * c->C * 8;
        a.lds_bytes = lds;
        (void)KK;
    }
    L.variant = variant;
    L.coded = coded;
    L.lds = lds;
    L.lnl_dst = lnl_dst;
    return PU_OK;
}

extern "C" {

int pu_enqueue(pu_ctx *c) {
    DeviceGuard g(c ? c->device : 0);  // also for the provider refresh's synchronous copies
    pu::LaunchPlan L;
    int rc = c ? pu::prepare_launch(c, L) : check_ready(c);
    if (rc) return rc;
    pu::PmatArgs &pa = L.pa;
    pu::TraverseArgs &a = L.a;
    const int variant = L.variant;
    const bool coded = L.coded;
    const size_t lds = L.lds;
    double *lnl_dst = L.lnl_dst;
    hipEvent_t *evs = nullptr;
    if (c->profile && c->n_prof < kMaxProf) {
        if (c->ev.size() < 4 * (size_t)(c->n_prof + 1)) {
            const size_t old = c->ev.size();
            c->ev.resize(4 * (size_t)(c->n_prof + 1), nullptr);
            for (size_t i = old; i < c->ev.size(); ++i)
                HIPCHK(&c->err, hipEventCreate(&c->ev[i]));
        }
        evs = &c->ev[4 * (size_t)c->n_prof];
        HIPCHK(&c->err, hipEventRecord(evs[0], c->stream));
    }
    if (!c->host_p) HIPCHK(&c->err, (hipError_t)pu::launch_pmatrix(c->stream, pa));
#ifdef PU_WG_STAMPS  // diagnostic build: per-workgroup timeline of k_prune (8 words each)
    const char *stamps_file = c->K != 20 ? getenv("PU_STAMPS_FILE") : nullptr;
    if (stamps_file) {
        const size_t n = 8 * (size_t)c->grid;
        if ((size_t)c->n_timed < n) {
            dfree(c->d_timing);
            c->d_timing = nullptr;
            if ((rc = dalloc(&c->err, &c->d_timing, n))) return rc;
            c->n_timed = (int)n;
        }
        HIPCHK(&c->err, hipMemsetAsync(c->d_timing, 0, n * 8, c->stream));
        a.timing = c->d_timing;
    }
#endif
    if (getenv("PU_TIMING") && c->K == 20) {  // debug: per-phase cycle sums of one wave
        if (!c->d_timing) {
            if ((rc = dalloc(&c->err, &c->d_timing, 8))) return rc;
            HIPCHK(&c->err, hipMemset(c->d_timing, 0, 64));
        }
        a.timing = c->d_timing;
        c->n_timed++;
    }
    if (getenv("PU_DEBUG_PTRS")) {  // debug: device ranges, to attribute a fault address
        auto rng = [](const char *n, const void *p, size_t b) {
            fprintf(stderr, "[pu ptrs] %-10s %p .. %p (%zu B)\n", n, p, (const char *)p + b, b);
        };
        const size_t padS = (size_t)(pu::tile_pitch(c->S) + c->pitch_pad) * pu::kTile;
        rng("ops", a.ops, ((size_t)c->n_ops + 1) * sizeof(pu::OpDesc));
        rng("chunk_op0", a.chunk_op0, ((size_t)c->n_chunks + 1) * 4);
        rng("chunk_tip0", a.chunk_tip0, ((size_t)c->n_chunks + 1) * 4);
        rng("tip_seq", a.tip_seq, 4);
        rng("P", a.P, 2 * ((size_t)c->n_ops + 1) * c->C * c->K * c->K * 8);
        rng("Pa", a.Pa, a.pa_bytes);
        rng("table", a.table, (size_t)c->n_codes * c->K * 8);
        rng("codes", a.codes, (size_t)c->n_tips * c->code_stride);
        rng("clv", a.clv, a.clv_bytes);
        rng("scale", a.scale, a.scale_bytes);
        rng("root_clv", a.root_clv, a.root_bytes);
        rng("root_scale", a.root_scale, a.root_scale_bytes);
        rng("site_lnl", a.site_lnl, (size_t)c->S * 8);
        rng("block_sum", a.block_sum, (size_t)c->block_cap * 8);
        rng("sflag", a.sflag, (c->clv_cap + 1) * (size_t)c->n_tiles * c->C * 4);
        rng("cat_lnl", a.cat_lnl, a.cat_lnl ? padS * c->C * 8 : 0);
        fprintf(stderr, "[pu ptrs] K %d C %d S %lld n_ops %d chunks %d max_uses %d grid %d "
                "variant %d n_lds %d lds %zu\n", c->K, c->C, (long long)c->S, c->n_ops,
                c->n_chunks, c->max_chunk_uses, c->grid, variant, c->n_lds, lds);
    }
    if (getenv("PU_DEBUG_PTRS"))
        fprintf(stderr, "[pu ptrs] pending HIP error before the launch: %s\n",
                hipGetErrorString(hipPeekAtLastError()));
    if (evs) HIPCHK(&c->err, hipEventRecord(evs[1], c->stream));
    // r06, opt-in (PU_RED_FUSED=1; DESIGN 4.8: the same throughput, ~3 us more traversal): the
    // lnL sum in the traversal's last workgroup (TraverseArgs::red_slots) for DNA trees
    // without chain tasks, outside graph captures (a replay would reuse the generation)
    if (c->K == 4 && !a.lnl_out && !a.cat_lnl && !(variant & pu::TV_CHAIN) &&
        getenv("PU_RED_FUSED") && atoi(getenv("PU_RED_FUSED")) == 1) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(c->stream, &cs) != hipSuccess) {
            (void)hipGetLastError();
            cs = hipStreamCaptureStatusActive;
        }
        const int nb = pu::traverse_block_sums(c->K, c->C, c->S);
        if (cs == hipStreamCaptureStatusNone && nb == c->grid) {
            if (c->red_cap < nb || c->red_gen >= 0x7fffffffu) {
                if (c->red_cap < nb) {
                    dfree(c->d_red_slots);
                    c->red_cap = 0;
                    if ((rc = dalloc(&c->err, &c->d_red_slots, 2 * (size_t)nb))) return rc;
                    c->red_cap = nb;
                }
                HIPCHK(&c->err, hipMemsetAsync(c->d_red_slots, 0, 16 * (size_t)c->red_cap,
                                               c->stream));
                c->red_gen = 0;
            }
            a.red_slots = c->d_red_slots;
            a.red_out = lnl_dst;
            a.red_gen = ++c->red_gen;
            a.red_n = nb;
        }
    }
    if (c->tickets_dirty) {  // a previous launch failed: its tickets may be off
        if (c->d_ticket)
            HIPCHK(&c->err, hipMemsetAsync(c->d_ticket, 0,
                                           (size_t)c->n_tiles * c->C * sizeof(int), c->stream));
        if (c->d_lse_ticket)
            HIPCHK(&c->err, hipMemsetAsync(c->d_lse_ticket, 0,
                                           ((size_t)c->n_tiles + 1) * sizeof(int), c->stream));
        c->tickets_dirty = false;
    }
    c->tickets_dirty = true;  // until the launches below are enqueued
    HIPCHK(&c->err, (hipError_t)pu::launch_traverse(c->stream, c->K, coded, variant, a,
                                                     c->grid));
    if (evs) HIPCHK(&c->err, hipEventRecord(evs[2], c->stream));  // the traversal alone
#ifdef PU_WG_STAMPS
    if (stamps_file) {  // header {grid, n_tiles, n_ops, S} then grid x 8 words
        std::vector<unsigned long long> h(8 * (size_t)c->grid + 4);
        h[0] = (unsigned long long)c->grid;
        h[1] = (unsigned long long)c->n_tiles;
        h[2] = (unsigned long long)c->n_ops;
        h[3] = (unsigned long long)c->S;
        HIPCHK(&c->err, hipStreamSynchronize(c->stream));
        HIPCHK(&c->err, hipMemcpy(h.data() + 4, c->d_timing, 8 * (size_t)c->grid * 8,
                                  hipMemcpyDeviceToHost));
        if (FILE *f = fopen(stamps_file, "ab")) {
            fwrite(h.data(), 8, h.size(), f);
            fclose(f);
        }
    }
#endif
    if (!a.lnl_out && !a.red_slots)
        HIPCHK(&c->err, (hipError_t)pu::launch_reduce(
                            c->stream, c->d_block, pu::traverse_block_sums(c->K, c->C, c->S),
                            lnl_dst));
    if ((rc = enqueue_ascbias(c, lnl_dst))) return rc;
    c->tickets_dirty = false;
    if (evs) {
        HIPCHK(&c->err, hipEventRecord(evs[3], c->stream));
        c->n_prof++;
    }
    if (!c->d_lnl_ext)
        HIPCHK(&c->err, hipMemcpyAsync(c->h_lnl, c->d_lnl, sizeof(double),
                                       hipMemcpyDeviceToHost, c->stream));
    c->ran = true;
    c->root_stale = false;
    return PU_OK;
}

int pu_synchronize(pu_ctx *c, double *lnl_out) {
    if (!c) return set_err(nullptr, PU_E_ARG, "null context");
    DeviceGuard g(c->device);
    if (hipError_t e = hipStreamSynchronize(c->stream); e != hipSuccess) {
        c->tickets_dirty = true;  // the failed launch may have left its tickets counted
        return set_err(&c->err, PU_E_HIP, "hipStreamSynchronize: %s", hipGetErrorString(e));
    }
    if (lnl_out) {
        if (c->lnl_batch)  // the last evaluation was a batch's, into its caller's buffer
            HIPCHK(&c->err, hipMemcpy(lnl_out, c->lnl_batch, sizeof(double),
                                      hipMemcpyDeviceToHost));
        else if (c->d_lnl_ext)
            HIPCHK(&c->err, hipMemcpy(lnl_out, c->d_lnl_ext, sizeof(double),
                                      hipMemcpyDeviceToHost));
        else
            *lnl_out = *c->h_lnl;
    }
    return PU_OK;
}

int pu_run(pu_ctx *c, double *lnl_out, double *sitewise_out) {
    int rc = pu_enqueue(c);
    if (rc) return rc;
    if ((rc = pu_synchronize(c, lnl_out))) return rc;
    return sitewise_out ? pu_get_site_lnl(c, sitewise_out) : PU_OK;
}

int pu_get_site_lnl(pu_ctx *c, double *out) {
    if (!c || !out) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (!c->ran) return set_err(&c->err, PU_E_STATE, "pu_run first");
    DeviceGuard g(c->device);
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    HIPCHK(&c->err, hipMemcpy(out, c->d_site_lnl, (size_t)c->S * 8, hipMemcpyDeviceToHost));
    return PU_OK;
}

int pu_get_partials(pu_ctx *c, int node, double *partials_out, double *scale_out) {
    if (!c || !partials_out) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (node < 0 || node >= c->n_nodes) return set_err(&c->err, PU_E_ARG, "bad node %d", node);
    DeviceGuard g(c->device);
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    const size_t nV = (size_t)c->S * c->C * c->K, nS = (size_t)c->S * c->C;
    const int t = c->tip_slot[node];
    if (t >= 0) {
        if (c->tip_kind[t] == 0) return set_err(&c->err, PU_E_STATE, "tip %d has no data", node);
        if (int rc = sync_tips(c)) return rc;
        double *tmp = nullptr;
        int rc = dalloc(&c->err, &tmp, nV);
        if (rc) return rc;
        const bool coded = c->tip_kind[t] == 2 && !any_dense(c);
        hipError_t e = (hipError_t)pu::launch_expand_tip(c->stream, c->K, c->C, c->S, c->code_stride, coded, t,
                                                          c->d_tips, c->d_codes, c->d_table, tmp);
        if (e == hipSuccess) e = hipMemcpyAsync(partials_out, tmp, nV * 8, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        dfree(tmp);
        if (e != hipSuccess)
            return set_err(&c->err, PU_E_HIP, "tip expansion failed: %s", hipGetErrorString(e));
        if (scale_out) memset(scale_out, 0, nS * 8);
        return PU_OK;
    }
    if (!c->have_sched || !c->ran) return set_err(&c->err, PU_E_STATE, "pu_run first");
    const int s = c->store_slot[node];
    if (s < 0 || (c->flags & PU_LNL_ONLY))
        return set_err(&c->err, PU_E_STATE, "partials of node %d are not kept (PU_LNL_ONLY "
                       "or node not in schedule)", node);
    const size_t padS = (size_t)pu::ctx_pitch(c) * pu::kTile;  // layout rows
    return untile_out(c, c->d_clv + (size_t)s * padS * c->C * c->K,
                      c->d_scale + (size_t)s * padS * c->C, partials_out, scale_out);
}

int pu_get_root(pu_ctx *c, double *rp, double *rs) {
    if (!c || !rp || !rs) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (!c->ran) return set_err(&c->err, PU_E_STATE, "pu_run first");
    if (c->root_stale)
        return set_err(&c->err, PU_E_STATE, "the last run was a pu_batch launch, which does not "
                       "write the root partials: pu_enqueue / pu_run first");
    DeviceGuard g(c->device);
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    return untile_out(c, c->d_root, c->d_root_scale, rp, rs);
}

int pu_get_pmatrices(pu_ctx *c, double *out) {
    if (!c || !out) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (!c->ran) return set_err(&c->err, PU_E_STATE, "pu_run first");
    DeviceGuard g(c->device);
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    const size_t per = 2 * (size_t)c->C * c->K * c->K;
    std::vector<double> dev(per * (c->n_ops + 1));
    if (c->K == 20 && !c->host_p && pu::pmatrix_writes_pa(c->K)) {
        // k_pmatrix_aa writes only the A operands [side][cat][q][lane][2]; every P entry is
        // in them (rows 0..15 in .x of lane 16 (j % 4) + i, rows 16..19 in .y of lane
        // 16 (j % 4) + i - 16, k-step q = j / 4)
        constexpr int K = 20, NA = 5 * 128;
        const size_t nm = 2 * ((size_t)c->n_ops + 1) * c->C;
        std::vector<double> pa(nm * NA);
        HIPCHK(&c->err, hipMemcpy(pa.data(), c->d_Pa, pa.size() * 8, hipMemcpyDeviceToHost));
        for (size_t m = 0; m < nm; ++m)
            for (int i = 0; i < K; ++i)
                for (int j = 0; j < K; ++j) {
                    const int q = j >> 2, k = j & 3;
                    const int lane = 16 * k + (i < 16 ? i : i - 16);
                    dev[m * K * K + i * K + j] = pa[m * NA + q * 128 + 2 * lane + (i < 16 ? 0 : 1)];
                }
    } else {
        HIPCHK(&c->err, hipMemcpy(dev.data(), c->d_P, dev.size() * 8, hipMemcpyDeviceToHost));
    }
    // back to the caller's op order and child order
    const size_t half = per / 2;
    auto put = [&](int t, int o) {
        const int sw = c->swap[t];
        memcpy(out + per * o, dev.data() + per * t + half * sw, half * 8);
        memcpy(out + per * o + half, dev.data() + per * t + half * (1 - sw), half * 8);
    };
    for (int t = 0; t < c->n_ops; ++t) put(t, c->perm[t]);
    put(c->n_ops, c->n_ops);
    return PU_OK;
}

int pu_plan_stats(int n_nodes, int n_ops, const int32_t *ops, int root_a, int root_b, int R,
                  int L, int flags, int32_t *stats) {
    if (n_nodes < 2 || n_ops < 0 || !stats || (n_ops > 0 && !ops) || R < 0 || L < 0)
        return set_err(nullptr, PU_E_ARG, "pu_plan_stats: bad arguments");
    pu_ctx c;  // host-only shell: no device state is touched
    c.n_nodes = n_nodes;
    c.tip_slot.assign(n_nodes, -1);
    std::vector<char> produced(n_nodes, 0);
    for (int o = 0; o < n_ops; ++o)
        if (ops[3 * o] >= 0 && ops[3 * o] < n_nodes) produced[ops[3 * o]] = 1;
    int t = 0;
    for (int v = 0; v < n_nodes; ++v)
        if (!produced[v]) c.tip_slot[v] = t++;
    Plan pl;
    int rc = make_plan(&c, n_ops, ops, root_a, root_b, L, !(flags & PU_NO_REORDER),
                       !(flags & PU_LNL_ONLY), pl, R);
    if (rc) {
        g_err = c.err;
        return rc;
    }
    stats[0] = pl.n_mem;
    stats[1] = (int)pl.tasks.size();
    stats[2] = pl.n_lds;
    stats[3] = pl.n_tip;
    stats[4] = pl.n_store;
    stats[5] = pl.max_live;
    stats[6] = pl.n_cur;
    stats[7] = pl.tasks.empty() ? 0 : n_ops - pl.top_lo;
    return PU_OK;
}

void *pu_ctx_stream(pu_ctx *c) { return c ? (void *)c->stream : nullptr; }

int pu_write_ceiling(int device, int64_t bytes, int reps, double *ms_out) {
    if (bytes < 4 || reps < 1 || !ms_out)
        return set_err(nullptr, PU_E_ARG, "pu_write_ceiling: bad arguments");
    if (int rc = check_device(device)) return rc;
    DeviceGuard g(device);
    const size_t n32 = (size_t)bytes / 4;
    void *buf = nullptr;
    hipStream_t st = nullptr;
    std::vector<hipEvent_t> ev(2 * (size_t)reps, nullptr);
    auto done = [&](int rc) {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        if (st) (void)hipStreamDestroy(st);
        if (buf) (void)hipFree(buf);
        return rc;
    };
    if (hipMalloc(&buf, n32 * 4) != hipSuccess) {
        buf = nullptr;
        (void)hipGetLastError();
        return done(set_err(nullptr, PU_E_NOMEM, "pu_write_ceiling: %lld bytes", (long long)bytes));
    }
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess)
        return done(set_err(nullptr, PU_E_HIP, "pu_write_ceiling: hipStreamCreate"));
    for (auto &e : ev)
        if (hipEventCreate(&e) != hipSuccess)
            return done(set_err(nullptr, PU_E_HIP, "pu_write_ceiling: hipEventCreate"));
    for (int i = 0; i < 3; ++i)
        if (hipMemsetD32Async((hipDeviceptr_t)buf, 0x3ff00000u + i, n32, st) != hipSuccess)
            return done(set_err(nullptr, PU_E_HIP, "pu_write_ceiling: hipMemsetD32Async"));
    for (int i = 0; i < reps; ++i) {
        (void)hipEventRecord(ev[2 * i], st);
        if (hipMemsetD32Async((hipDeviceptr_t)buf, 0x3ff00000u + i, n32, st) != hipSuccess)
            return done(set_err(nullptr, PU_E_HIP, "pu_write_ceiling: hipMemsetD32Async"));
        (void)hipEventRecord(ev[2 * i + 1], st);
    }
    if (hipStreamSynchronize(st) != hipSuccess)
        return done(set_err(nullptr, PU_E_HIP, "pu_write_ceiling: synchronize"));
    std::vector<float> t(reps);
    for (int i = 0; i < reps; ++i)
        if (hipEventElapsedTime(&t[i], ev[2 * i], ev[2 * i + 1]) != hipSuccess)
            return done(set_err(nullptr, PU_E_HIP, "pu_write_ceiling: hipEventElapsedTime"));
    std::nth_element(t.begin(), t.begin() + reps / 2, t.end());
    *ms_out = t[reps / 2];
    return done(PU_OK);
}

int64_t pu_ctx_device_bytes(const pu_ctx *c) {
    if (!c) return 0;
    const int64_t S = c->S, C = c->C, K = c->K;
    const int64_t padS = (pu::tile_pitch(S) + c->pitch_pad) * pu::kTile;
    int64_t b = (int64_t)c->clv_cap * padS * C * (K + 1) * 8;
    b += padS * C * (K + 1) * 8 + 2 * S * 8;
    if (c->d_tips) b += (int64_t)c->n_tips * S * K * 8;
    // shared tips (pu_share_tips) count once, in the context that uploaded them
    if (c->d_codes && (!c->tip_store || c->tip_store->first == c)) b += (int64_t)c->n_tips * S;
    b += 2 * ((int64_t)c->n_ops + 1) * C * K * K * 8;
    return b;
}

int pu_ctx_profile(pu_ctx *c, int enable) {
    if (!c) return set_err(nullptr, PU_E_ARG, "null context");
    c->profile = enable != 0;
    c->n_prof = 0;
    c->n_edge_prof = 0;
    return PU_OK;
}

int pu_ctx_kernel_ms(pu_ctx *c, double *trav, double *total, int *n) {
    if (!c) return set_err(nullptr, PU_E_ARG, "null context");
    DeviceGuard g(c->device);
    double acc_t = 0.0, acc_a = 0.0;
    for (int k = 0; k < c->n_prof; ++k) {
        hipEvent_t *e = &c->ev[4 * (size_t)k];
        HIPCHK(&c->err, hipEventSynchronize(e[3]));
        float t_tr = 0.f, t_all = 0.f;
        HIPCHK(&c->err, hipEventElapsedTime(&t_tr, e[1], e[2]));
        HIPCHK(&c->err, hipEventElapsedTime(&t_all, e[0], e[3]));
        acc_t += t_tr;
        acc_a += t_all;
    }
    const int k = c->n_prof;
    if (trav) *trav = k ? acc_t / k : 0.0;
    if (total) *total = k ? acc_a / k : 0.0;
    if (n) *n = k;
    return PU_OK;
}

int pu_ctx_kernel_times(pu_ctx *c, double *trav, double *total, int cap, int *n) {
    if (!c || cap < 0 || (cap > 0 && (!trav || !total)))
        return set_err(c ? &c->err : nullptr, PU_E_ARG, "bad arguments");
    DeviceGuard g(c->device);
    const int k = std::min(cap, c->n_prof);
    for (int i = 0; i < k; ++i) {
        hipEvent_t *e = &c->ev[4 * (size_t)i];
        HIPCHK(&c->err, hipEventSynchronize(e[3]));
        float t_tr = 0.f, t_all = 0.f;
        HIPCHK(&c->err, hipEventElapsedTime(&t_tr, e[1], e[2]));
        HIPCHK(&c->err, hipEventElapsedTime(&t_all, e[0], e[3]));
        trav[i] = t_tr;
        total[i] = t_all;
    }
    if (n) *n = k;
    return PU_OK;
}

int pu_ctx_plan_info(const pu_ctx *c, int32_t *out) {
    if (!c || !out) return set_err(nullptr, PU_E_ARG, "null argument");
    if (!c->have_sched) return set_err(nullptr, PU_E_STATE, "pu_set_schedule first");
    out[0] = c->grid;
    out[1] = c->waves;
    out[2] = c->variant;
    out[3] = c->n_lds;
    out[4] = c->n_chunks;
    out[5] = c->lds_pad;
    out[6] = c->n_tiles;
    out[7] = (int32_t)((c->n_tiles * (int64_t)c->C + 3) / 4);
    out[8] = c->pitch_extra;
    out[9] = (int32_t)pu::ctx_pitch(c);
    return PU_OK;
}

int pu_ctx_traffic(pu_ctx *c, int64_t *out) {
    if (!c || !out) return set_err(c ? &c->err : nullptr, PU_E_ARG, "null argument");
    if (!c->have_sched || !c->ran) return set_err(&c->err, PU_E_STATE, "pu_run first");
    DeviceGuard g(c->device);
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    const int64_t padS = (int64_t)c->n_tiles * pu::kTile, C = c->C, K = c->K;  // bytes moved
    const int64_t nwt = (int64_t)c->n_tiles * C;
    // parents written (every storing op + the root, which a pu_batch run does not write),
    // 8 B per double
    const int64_t root = c->root_stale ? 0 : 1;
    out[0] = (int64_t)(c->n_store_ops + root) * padS * C * K * 8;
    // scalers: with TV_SKIP_ZERO_SCALE an all-zero wave tile over zero memory is not stored, so
    // in steady state exactly the tiles whose flag is set are written (pu_kernels.hip k_prune)
    if ((c->variant & pu::TV_SKIP_ZERO_SCALE) && c->K != 20) {
        std::vector<uint32_t> f((size_t)(c->clv_cap + 1) * nwt);
        HIPCHK(&c->err, hipMemcpy(f.data(), c->d_sflag, f.size() * 4, hipMemcpyDeviceToHost));
        int64_t nz = 0;
        for (size_t s = 0; s < (size_t)c->n_store; ++s)
            for (int64_t w = 0; w < nwt; ++w) nz += f[s * nwt + w] != 0;
        for (int64_t w = 0; w < nwt && root; ++w) nz += f[(size_t)c->clv_cap * nwt + w] != 0;
        out[1] = nz * pu::kTile * 8;
    } else {
        out[1] = (int64_t)(c->n_store_ops + root) * padS * C * 8;
    }
    // tip data read: one byte per site and tip use (codes), or the dense K-vector
    out[2] = (int64_t)c->n_tip_uses * padS * (any_dense(c) ? K * 8 : 1);
    // parents read back from HBM (stash overflow), CLV + scaler
    out[3] = (int64_t)c->n_mem * padS * C * (K + 1) * 8;
    // sitewise lnL written, pattern weights read
    out[4] = 2 * c->S * 8;
    return PU_OK;
}

int pu_ctx_set_stream(pu_ctx *c, void *st) {
    if (!c) return set_err(nullptr, PU_E_ARG, "null context");
    DeviceGuard g(c->device);
    HIPCHK(&c->err, hipStreamSynchronize(c->stream));
    // NULL is the HIP null stream (torch's default stream has handle 0: its collectives must
    // stay ordered after the traversal); PU_OWN_STREAM selects the context's own stream
    c->stream = st == PU_OWN_STREAM ? c->own_stream : (hipStream_t)st;
    return PU_OK;
}

int pu_set_lnl_device_output(pu_ctx *c, double *dptr) {
    if (!c) return set_err(nullptr, PU_E_ARG, "null context");
    c->d_lnl_ext = dptr;
    return PU_OK;
}

}  // extern "C"

void *pu::ctx_stream(pu_ctx *c) { return c ? (void *)c->stream : nullptr; }
