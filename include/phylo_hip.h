/*
 * phylo_hip.h -- C ABI of libphylo_hip.so, the MI355X (gfx950) Felsenstein
 * pruning engine behind phylo_utils' likelihood-engine seam.
 *
 * The reference selects its engine by module import
 * (phylo_utils/tree_model.py:1 `from phylo_utils.likelihood.numba_likelihood_engine
 * import clv, lnl_node`).  Every entry point below replaces one reference
 * interface; the citation is given on each declaration (paths relative to the
 * reference repository root).
 *
 * Conventions
 *   - plain pointers and sizes; no C++ types, no exceptions cross this ABI;
 *   - every int-returning call returns PU_OK (0) or a negative PU_E* code and
 *     records a message readable with pu_last_error();
 *   - host buffers are caller-owned and copied in/out; device buffers are
 *     owned by the context;
 *   - a context is bound to one device and one HIP stream and is not
 *     thread-safe (one host thread per context);
 *   - layouts are the reference's C-contiguous fp64 layouts:
 *       partials [site][category][state], scalers [site][category],
 *       P matrices [category][parent state][child state].
 */
#ifndef PHYLO_HIP_H
#define PHYLO_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PU_OK 0
#define PU_E_ARG (-1)     /* bad argument / shape (numba raises on shape mismatch)     */
#define PU_E_HIP (-2)     /* HIP runtime error                                          */
#define PU_E_STATE (-3)   /* call order violated (e.g. run before set_schedule)         */
#define PU_E_SCHED (-4)   /* schedule is not a valid post-order over the declared tips  */
#define PU_E_NOMEM (-5)   /* device allocation failed                                   */
#define PU_E_COMM (-6)    /* RCCL error                                                 */

/* context flags */
#define PU_KEEP_PARTIALS 0x0 /* default: every internal CLV kept in HBM (tree_model.py:117-124) */
#define PU_LNL_ONLY 0x1      /* internal CLVs live only as long as needed (buffer reuse)        */
#define PU_NO_REORDER 0x2    /* evaluate ops in the caller's order (default: register-aware)    */

typedef struct pu_ctx pu_ctx;

/* ---- library / errors ------------------------------------------------------------- */
const char *pu_version(void);
/* Last error of ctx, or the process-wide last error when ctx is NULL. */
const char *pu_last_error(const pu_ctx *ctx);
int pu_device_count(int *n);

/* ---- stateless engine seam: exactly the numba engine's gufuncs --------------------- */
/* numba `clv`, phylo_utils/likelihood/numba_likelihood_engine.py:10-46.
 * p1,p2 [C][K][K]; clv1,clv2,out [S][C][K]; scaler_a,scaler_b,cml_scaler [S][C].
 * cml_scaler is written in place (numba_likelihood_engine.py:40,44). */
int pu_clv(int device, int n_states, int n_cat, int64_t n_sites, const double *p1,
           const double *p2, const double *clv1, const double *clv2, const double *scaler_a,
           const double *scaler_b, double *cml_scaler, double *out);
/* numba `lnl_node`, numba_likelihood_engine.py:82-87: out[s][c] = log(sum_i pi_i *
 * partials[s][c][i]) + scale[s][c], or -inf when the sum is <= 0. */
int pu_lnl_node(int device, int n_states, int n_cat, int64_t n_sites, const double *pi,
                const double *partials, const double *scale, double *out);

/* ---- discrete gamma: phylo_utils.discrete_gamma.discrete_gamma ---------------------- */
/* src/discrete_gamma.pyx:30-47 -> src/c_discrete_gamma.c:285-321 (alpha == beta).
 * Host routine (AS91 / AS32 / AS70 / Pike-Hill), no device involved. */
int pu_discrete_gamma(double alpha, int n_cat, int median_rates, double *rates_out);

/* ---- TreeModel-equivalent context ---------------------------------------------------- */
/* TreeModel.initialise allocation, tree_model.py:101-124.  n_nodes = 2N-2 node
 * indices as numbered by Traversal (traversal.py:16-21); n_patterns = S. */
int pu_ctx_create(pu_ctx **out, int device, int n_nodes, int n_tips, int64_t n_patterns,
                  int n_cat, int n_states, int flags);
void pu_ctx_destroy(pu_ctx *ctx);

/* Tip partials for node `node` ([S][K]); tree_model.py:142-148 copies these into
 * every category -- the engine stores them once and broadcasts. */
int pu_set_tip_partials(pu_ctx *ctx, int node, const double *partials);
/* Compact tips (the same information as charmap partial vectors,
 * alignment/charmaps.py:8-86, alignment.py:26-37): one code table
 * [n_codes][K] per context (n_codes <= 256), then codes[S] per tip node.
 * A context whose tips are all coded streams 1 byte per tip site instead of
 * K doubles; mixing with pu_set_tip_partials is allowed (coded tips are then
 * expanded on the host). */
int pu_set_code_table(pu_ctx *ctx, int n_codes, const double *code_table);
int pu_set_tip_codes(pu_ctx *ctx, int node, const uint8_t *codes);
/* Pattern counts from alignment_to_numpy (alignment/alignment.py:47-51); default 1. */
int pu_set_pattern_weights(pu_ctx *ctx, const double *weights);
/* All tips at once (SURVEY 8(b) B2 `pu_set_tips`; tree_model.py:142-148): tip i is node
 * nodes[i]; exactly one of codes [n_tips][S] (with code_table [n_codes][K]) or partials
 * [n_tips][S][K]; pattern_weights [S] or NULL (all 1). */
int pu_set_tips(pu_ctx *ctx, int n_tips, const int32_t *nodes, int n_codes,
                const double *code_table, const uint8_t *codes, const double *partials,
                const double *pattern_weights);

/* A new topology over the same taxa (many trees on one alignment): tip
 * slot i -- the i-th tip node given to pu_set_tips / pu_set_tip_* -- becomes node
 * nodes[i] of the new numbering (Traversal, traversal.py:16-21).  No tip data move; the
 * next pu_set_schedule describes the new tree (tree_model.py:87-89 set_tree). */
int pu_set_tip_nodes(pu_ctx *ctx, int n_tips, const int32_t *nodes);

/* One resident alignment for many contexts (r06, SURVEY 8(e) G2: "the same (replicated)
 * alignment" per GPU; the reference holds one alignment and swaps trees,
 * tree_model.py:42-50, 87-89).  ctx -- fresh: no tips set yet -- reads owner's coded tips,
 * code table and pattern weights in place instead of holding its own copies; owner's tip
 * slot i is node nodes[i] of ctx's numbering (as pu_set_tip_nodes).  Both contexts must be
 * on one device with equal n_tips, S and K, and every owner tip must be coded.  From then on
 * the shared tips, table and weights are frozen in every context that holds them
 * (pu_set_tip_*, pu_set_code_table, pu_set_pattern_weights return PU_E_STATE); the storage
 * lives until the last context holding it is destroyed, in any order. */
int pu_share_tips(pu_ctx *ctx, pu_ctx *owner, int n_tips, const int32_t *nodes);

/* Model.p inputs (substitution_models/abstract.py:49-59, 99-105): evecs [K][K],
 * evals [K], ivecs [K][K] row-major; freqs [K] (lnl_node pi); rate-model rates and
 * weights [C] (rate_models.py:15-47). */
int pu_set_model(pu_ctx *ctx, const double *evecs, const double *evals, const double *ivecs,
                 const double *freqs, const double *rates, const double *weights);

/* Models without a real eigen-decomposition -- the non-reversible DNANonReversibleModel
 * family (Strsym, Unrest: P(t) = expm(Q r t), substitution_models/abstract.py:163-180):
 * pu_set_model_p sets freqs (lnl_node pi; q_to_freqs for these models), rates and weights,
 * and the context then skips its own P computation.  After every pu_set_schedule /
 * pu_set_branch_lengths the caller supplies the matrices with pu_set_pmatrices:
 * P [n_ops + 1][2][C][K][K] in the caller's op and child order (the row after the last op:
 * root_a's P(0), root_b's P(root_len); the layout pu_get_pmatrices returns); until then
 * pu_enqueue / pu_run fail with PU_E_STATE.  Edge operations (pu_edge_*, pu_update_partials,
 * pu_optimise_*) need pu_set_model and fail with PU_E_STATE on such a context.
 * pu_set_model switches back to device-computed P. */
int pu_set_model_p(pu_ctx *ctx, const double *freqs, const double *rates, const double *weights);
int pu_set_pmatrices(pu_ctx *ctx, const double *P);
/* Matrix provider of a context on host transition matrices (pu_set_model_p), for the
 * operations whose lengths are chosen on the device side of the ABI -- the edge lnL /
 * derivatives, partial updates and the Newton optimisers (pu_edge_*, pu_update_partials,
 * pu_optimise_*), and the traversal after they move a length.  fn(user, order, n, t, out)
 * fills out[n][C][K][K] with d^order/dt^order P(t[i] r_c), order 0, 1 or 2, the chain-rule
 * factor r_c included (for the non-reversible models r Q expm(Q r t) and r^2 Q^2 expm(Q r t);
 * the reference's DNANonReversibleModel.dp_dt / d2p_dt2, abstract.py:180-192, return
 * Q expm(Q r t) and Q^2 expm(Q r t)).  Returns 0, non-zero on failure.  NULL removes it. */
typedef int (*pu_pmat_provider)(void *user, int order, int n, const double *t, double *out);
int pu_set_pmatrix_provider(pu_ctx *ctx, pu_pmat_provider fn, void *user);

/* Traversal.postorder_traversal (traversal.py:28,36; utils.py:127-134): ops[n_ops][3]
 * = (parent, child1, child2); brlens[n_ops][2] = lengths of (parent,child1) and
 * (parent,child2) (Traversal.brlens); root edge (root_a, root_b, root_len) as in
 * compute_partials_at_edge (tree_model.py:178-198): P(0) on root_a, P(len) on root_b. */
int pu_set_schedule(pu_ctx *ctx, int n_ops, const int32_t *ops, const double *brlens,
                    int root_a, int root_b, double root_len);
/* New branch lengths for the current topology (same layout as pu_set_schedule). */
int pu_set_branch_lengths(pu_ctx *ctx, const double *brlens, double root_len);

/* compute_partials + compute_likelihood_at_edge + sum (tree_model.py:160-217,
 * bin/phy.py:146).  Synchronous: lnl_out = sum_s weight[s] * site_lnl[s]; sitewise_out
 * [S] (nullable) = the per-pattern lnL (tree_model.py:216, before the inverse-index
 * expansion). */
int pu_run(pu_ctx *ctx, double *lnl_out, double *sitewise_out);
/* Asynchronous form for timing loops: enqueue on the context stream only. */
int pu_enqueue(pu_ctx *ctx);
int pu_synchronize(pu_ctx *ctx, double *lnl_out);
/* Per-pattern log-likelihood (compute_likelihood_at_edge before the inverse-index
 * expansion, tree_model.py:216). */
int pu_get_site_lnl(pu_ctx *ctx, double *out);
/* Read back TreeModel.partials[node] / scale[node] (tips are expanded per category)
 * and root_partials / root_scale.  Requires PU_KEEP_PARTIALS for internal nodes; the root
 * after the context's own last run (not a pu_batch_enqueue, PU_E_STATE). */
int pu_get_partials(pu_ctx *ctx, int node, double *partials_out, double *scale_out);
int pu_get_root(pu_ctx *ctx, double *root_partials_out, double *root_scale_out);
/* Transition matrices the last run used: [n_ops+1][2][C][K][K] (last row = root). */
int pu_get_pmatrices(pu_ctx *ctx, double *out);

/* Lewis ascertainment-bias correction (TreeModel.set_ascertainment_bias_correction,
 * tree_model.py:92-98; dummy sites :151-156; correction :209-214).  The caller appends K
 * dummy invariant patterns [first_dummy, S) -- at dummy pattern first_dummy + k every tip
 * is the one-hot vector of state k -- with pattern weight 0.  After every evaluation
 * (pu_run / pu_enqueue / pu_edge_lnl): corr = log(1 - exp(x)), site_lnl[s] -= corr for
 * s < first_dummy, lnl -= corr * sum of their weights.  mode 1 (the reference): x =
 * logsumexp over the K x C lnl_node values of the dummy sites, unweighted over categories
 * (so NaN for Gamma rates with C > 1, as the reference); mode 2 (weighted Lewis): x =
 * logsumexp_k of the dummy sites' mixture lnL.  mode 0: off. */
int pu_set_ascertainment(pu_ctx *ctx, int mode, int64_t first_dummy);
/* The correction (log(1 - P(invariant))) the last evaluation applied. */
int pu_get_ascertainment_correction(pu_ctx *ctx, double *corr_out);

/* ---- edge operations on the resident CLVs (need PU_KEEP_PARTIALS) ------ */
/* Category limits (one workgroup's LDS holds the per-(category, site) values): edge lnL
 * C <= 194 (K = 4) / 21 (K = 20); derivatives and the optimisers C <= 72 (K = 2), 60 (K = 4),
 * 10 (K = 20).  Beyond them the call fails with PU_E_ARG. */
/* compute_partials_at_edge + compute_likelihood_at_edge (tree_model.py:178-217) with the
 * root on ANY edge (a, b) of the current topology, on the nodes' CURRENT partials (the
 * reference's "only valid if the CLVs at a and b are valid", tree_model.py:181-182): P(0) on
 * a, P(length of (a,b)) on b.  Writes the root partials (pu_get_root) and sitewise lnL;
 * PU_E_ARG "There is no edge connecting nodes a and b" as tree_model.py:184-187. */
int pu_edge_lnl(pu_ctx *ctx, int node_a, int node_b, double *lnl_out, double *sitewise_out);
/* out3 = {lnL, dlnL/dt, d2lnL/dt2} at edge length t = length (< 0: the current length) for
 * the pattern-weighted sum over sites of log sum_c w_c f_c, f_c as in lnl_branch_derivs
 * (numba_likelihood_engine.py:49-57) with dP/dt = evecs diag(l r e^{l t r}) ivecs -- the
 * exact derivative of P(t r); Model.dp_dt (abstract.py:61-77) omits the factor r. */
int pu_edge_derivs(pu_ctx *ctx, int node_a, int node_b, double length, double *out3);
/* In-place partials updates on any nodes, in order: partials[par] = clv(P(len1), P(len2),
 * partials[ch1], partials[ch2]) for ops[n][3] = (par, ch1, ch2), brlens[n][2] -- the
 * re-orientation and restore rows of the optimising traversal (utils.py:137-188). */
int pu_update_partials(pu_ctx *ctx, int n_ops, const int32_t *ops, const double *brlens);
/* Newton-Raphson (monotone safeguard) on the length of edge (a, b), all evaluations on the
 * device with the current partials of a and b; lengths are kept in [1e-8, 100].  The new
 * length is stored (pu_get_branch_lengths) and returned. */
int pu_optimise_edge(pu_ctx *ctx, int node_a, int node_b, double tol, int max_iter,
                     double *length_out, double *lnl_out);
/* One pass of the optimising traversal (Traversal.optimising_traversal, traversal.py:29,34-35;
 * utils.py:137-188): rows[n_rows][5]; a row (p, s, g, n, p) re-orients p towards n from s and
 * g, then optimises edge (n, p); (n, c1, c2, -1, -1) restores n; (-1, -1, -1, a, b) optimises
 * edge (a, b).  Ends with a full traversal at the new lengths: lnl_out; evals_out = Newton
 * iterations taken. */
int pu_optimise_sweep(pu_ctx *ctx, int n_rows, const int32_t *rows, double tol, int max_iter,
                      double *lnl_out, int *evals_out);
/* The reference's own 1-D minimisers on the length of edge (a, b) (r06): method 1 = brent
 * (src/optimisation.pyx:86-177), 2 = dbrent (:179-297), over the objective f(t) = -lnL(t) (and
 * f'(t) = -dlnL/dt for dbrent) with the current partials of a and b: brent(lo, t0, hi, f, tol,
 * out) -- the bracket spanned by lo and hi, the search from t0 -- with the reference's steps,
 * tolerances, iteration limits and quirks (phylo_utils_amd/optimisation.py documents them).
 * out3 = the reference's out: {x, f(x), iterations}.  DNA contexts of up to 4 categories on
 * the device eigen-system run the whole minimisation in one persistent launch (the
 * k_edge_newton machinery); others one k_edge launch per evaluation, with the same state
 * machine.  The length x is stored (pu_get_branch_lengths). */
int pu_minimise_edge(pu_ctx *ctx, int node_a, int node_b, int method, double lo, double t0,
                     double hi, double tol, double *out3);
/* Current lengths in pu_set_schedule's layout: brlens_out[n_ops][2], root length. */
int pu_get_branch_lengths(pu_ctx *ctx, double *brlens_out, double *root_len_out);

/* ---- stateless branch likelihoods: the numba engine's lnl_branch / lnl_branch_derivs ---- */
/* numba_likelihood_engine.py:60-79 / :49-57 over E items (broadcast flattened by the caller):
 * item e uses probs[pidx ? pidx[e] : e % n_p] ([n_p][K][K], or [n_p][3][K][K] = P, dP, d2P
 * for the derivs); partials_a, partials_b [E][K]; scale_a, scale_b [E]; pi [K].
 * lnl_branch: out[E] = log(f) + sa + sb, f = sum((P . a) * b * pi);
 * lnl_branch_derivs: out[E][3] = {log f + sa + sb, f'/f, (f'' f - f'^2) / f^2}. */
int pu_lnl_branch(int device, int n_states, int64_t n_items, int n_p, const int32_t *pidx,
                  const double *probs, const double *pi, const double *partials_a,
                  const double *partials_b, const double *scale_a, const double *scale_b,
                  double *out);
int pu_lnl_branch_derivs(int device, int n_states, int64_t n_items, int n_p,
                         const int32_t *pidx, const double *probs, const double *pi,
                         const double *partials_a, const double *partials_b,
                         const double *scale_a, const double *scale_b, double *out);

/* ---- site-pattern compression --------------------------------------- */
/* Replaces np.unique(alignment, return_inverse=True, return_counts=True, axis=1) in
 * alignment_to_numpy (phylo_utils/alignment/alignment.py:40-57), on tip codes.
 * codes: [n_taxa][n_sites] uint8, row-major, each < n_codes (<= 256), numbered in the
 * lexicographic order of their partial vectors (then the byte order of code columns is the
 * order np.unique gives the float columns).  Outputs: *n_unique = U; unique_out [n_taxa][U]
 * (compact rows; the buffer holds n_taxa * n_sites bytes), counts_out [U], inverse_out
 * [n_sites] -- np.unique's three results, patterns in lexicographic order.  n_sites < 2^32,
 * n_taxa <= 65000.
 * Host buffers (copied in and out). */
int pu_compress_patterns(int device, const uint8_t *codes, int n_taxa, int64_t n_sites,
                         int n_codes, uint8_t *unique_out, int64_t *counts_out,
                         int64_t *inverse_out, int64_t *n_unique_out);
/* The same on device buffers, on the caller's HIP stream (hipStream_t as void*).  Row t of
 * the unique columns is written at d_unique + t * ld_unique (ld_unique >= n_sites; 0: U,
 * compact; an even ld_unique and base take 2-byte stores).  Returns when the result is
 * complete (U is read back between phases). */
int pu_compress_patterns_device(int device, void *stream, const uint8_t *d_codes, int n_taxa,
                                int64_t n_sites, int n_codes, uint8_t *d_unique,
                                int64_t ld_unique, int64_t *d_counts, int64_t *d_inverse,
                                int64_t *n_unique_out);

/* ---- multi-device / stream interop (site sharding) ------------------- */
/* Launch on the caller's HIP stream (hipStream_t as void*), e.g.
 * torch.cuda.current_stream().cuda_stream, so the RCCL all-reduce of the lnL is
 * stream-ordered after the traversal with no host synchronisation.  NULL is the HIP null
 * stream (torch's default stream: handle 0); PU_OWN_STREAM returns to the context's own
 * non-blocking stream, which is NOT ordered with the null stream. */
#define PU_OWN_STREAM ((void *)(intptr_t)-1)
int pu_ctx_set_stream(pu_ctx *ctx, void *hip_stream);
/* Also write each run's lnL (one double) to this DEVICE pointer (NULL = off); when set,
 * pu_enqueue skips its device->host copy and pu_synchronize reads it from here. */
int pu_set_lnl_device_output(pu_ctx *ctx, double *device_ptr);

/* ---- several trees per launch ------------------------------------
 * Replaces the reference's loop over trees -- set_tree, compute_partials, likelihood per tree
 * (tree_model.py:87-89, 160-176) -- for trees on one alignment (bootstrap replicates,
 * candidate trees: BASELINE cfg5).  A batch evaluates the lnL of n contexts with one P launch,
 * one traversal launch and one reduction for all of them, on the batch's stream; each
 * context keeps its own schedule, branch lengths and buffers, and each tree's lnL and sitewise
 * lnL are bitwise those of pu_enqueue on that context.  Accepted at pu_batch_enqueue (else
 * PU_E_ARG, and pu_enqueue per context is the way): contexts on one device, created with
 * PU_LNL_ONLY, K = 2 or 4, coded tips, the model's eigen-system (no host matrices), no
 * ascertainment correction, equal K, C and S.  The contexts must outlive the batch; work a
 * context queued on its own stream is ordered before the batch's launches, and the batch's
 * results are complete after pu_batch_synchronize (or on the batch's stream). */
typedef struct pu_batch pu_batch;
int pu_batch_create(pu_batch **out, int n, pu_ctx *const *ctxs);
void pu_batch_destroy(pu_batch *b);
const char *pu_batch_last_error(const pu_batch *b);
/* stream of the batch's launches: NULL the HIP null stream, PU_OWN_STREAM its own (default) */
int pu_batch_set_stream(pu_batch *b, void *stream);
/* tree i's lnL into lnl_dev[i] (device memory, n doubles); lnl_dev NULL: into each context's
 * own output (its pu_set_lnl_device_output, or pu_synchronize(ctx, &lnl) after
 * pu_batch_synchronize).  With lnl_dev, pu_synchronize(ctx_i, &lnl) until ctx_i's next own
 * evaluation reads lnl_dev[i] (which must then still be allocated).  Work later queued on a
 * context's own stream is ordered after the batch's launches (an event the stream waits on).
 * Refused (PU_E_ARG): a category count other than 1, 2 or 4.  The root partials are not
 * written (r06: nothing of a batched lnL-only tree reads them): pu_get_root on a context
 * refuses (PU_E_STATE) until its next own pu_enqueue / pu_run. */
int pu_batch_enqueue(pu_batch *b, double *lnl_dev);
int pu_batch_synchronize(pu_batch *b);
/* profiling (bench.py): on = 1 records hipEvents around each enqueue's traversal launch (and
 * its P and reduction launches) from here on; pu_batch_kernel_times returns up to cap
 * per-enqueue times in ms (trav: the traversal launch, total: P + traversal + reduction) */
int pu_batch_profile(pu_batch *b, int on);
int pu_batch_kernel_times(pu_batch *b, double *trav, double *total, int cap, int *n);

/* ---- one process, several devices (SURVEY 8(b) B2 pu_group_create, 8(e) G1) ----------- */
/* One context per device over contiguous pattern shards of an n_patterns alignment (shard
 * sizes differ by at most one) and an RCCL communicator over the devices
 * (ncclCommInitAll).  devices = NULL: 0 .. n_dev-1.  On failure *out is still set for
 * pu_group_last_error and must be destroyed. */
typedef struct pu_group pu_group;
int pu_group_create(pu_group **out, int n_dev, const int *devices, int n_nodes, int n_tips,
                    int64_t n_patterns, int n_cat, int n_states, int flags);
void pu_group_destroy(pu_group *g);
const char *pu_group_last_error(const pu_group *g);
int pu_group_size(const pu_group *g);
/* pattern range [first, first + count) of device i, and its context */
int pu_group_shard(const pu_group *g, int i, int64_t *first, int64_t *count);
pu_ctx *pu_group_ctx(pu_group *g, int i);
/* the pu_set_tips / pu_set_model / pu_set_schedule / pu_set_branch_lengths of every shard;
 * tips, codes and weights are given for all n_patterns and sliced per device */
int pu_group_set_tips(pu_group *g, int n_tips, const int32_t *nodes, int n_codes,
                      const double *code_table, const uint8_t *codes, const double *partials,
                      const double *pattern_weights);
int pu_group_set_model(pu_group *g, const double *evecs, const double *evals,
                       const double *ivecs, const double *freqs, const double *rates,
                       const double *weights);
int pu_group_set_schedule(pu_group *g, int n_ops, const int32_t *ops, const double *brlens,
                          int root_a, int root_b, double root_len);
int pu_group_set_branch_lengths(pu_group *g, const double *brlens, double root_len);
/* pu_set_model_p / pu_set_pmatrices of every shard (the same matrices on every device) */
int pu_group_set_model_p(pu_group *g, const double *freqs, const double *rates,
                         const double *weights);
int pu_group_set_pmatrices(pu_group *g, const double *P);
/* every shard's traversal, then ncclAllReduce(sum) of the per-device lnL on the shards'
 * streams (8 bytes, the only collective); sitewise_out [n_patterns] (nullable) gathers
 * the shards' per-pattern lnL */
int pu_group_run(pu_group *g, double *lnl_out, double *sitewise_out);

/* ---- planner introspection (host only, no device) -------------------------------------- */
/* Run the schedule planner of pu_set_schedule for a tree whose leaves are the nodes no op
 * produces, with L LDS stash slots and R = the split target (PU_SPLIT; 0: one task).
 * stats_out[8] = {n_mem, n_chains, n_lds, n_tip, n_store, max_live, n_cur, n_top}: children
 * read back from HBM, chain tasks of a split plan (0: not split), children from the LDS
 * stash / tips, HBM slots allocated, peak number of values waiting for a later consumer,
 * children taken straight from the previous op's result, ops of the top task. */
int pu_plan_stats(int n_nodes, int n_ops, const int32_t *ops, int root_a, int root_b, int R,
                  int L, int flags, int32_t *stats_out);

/* ---- measurement hooks (bench.py) ----------------------------------------------------- */
/* HIP stream the context launches on (hipStream_t as void*). */
void *pu_ctx_stream(pu_ctx *ctx);
/* Bytes resident on the device for this context. */
int64_t pu_ctx_device_bytes(const pu_ctx *ctx);
/* Device-side Newton (pu_optimise_edge / pu_optimise_sweep, r06): the persistent launches
 * made and the evaluations they ran since the context's edge buffers were set up. */
int pu_ctx_newton_stats(pu_ctx *ctx, int *launches, int *evaluations);
/* The device's write-stream ceiling for a traversal's store stream (r06, bench.py's
 * roofline.ceiling_GBps): hipMemsetAsync of `bytes` into a fresh buffer, `reps` times after 3
 * warm-ups, on a stream of its own; ms_out = the median time (ms).  The fastest write stream
 * measured on this hardware (6.4-6.6 TB/s, against 5.0-5.7 for k_prune-shaped
 * probes), so box-to-box spread shows in it as in the kernel. */
int pu_write_ceiling(int device, int64_t bytes, int reps, double *ms_out);
/* Event timing on the launch stream: with pu_ctx_profile(ctx, 1) every pu_enqueue
 * records events around its kernels (up to 4096 runs); pu_ctx_kernel_ms waits for them
 * and returns the mean time of the traversal launch alone and the mean P + traversal +
 * reduction time (ms) over the recorded runs.  pu_ctx_profile(ctx, 0|1) also clears the
 * record. */
int pu_ctx_profile(pu_ctx *ctx, int enable);
int pu_ctx_kernel_ms(pu_ctx *ctx, double *traverse_ms_avg, double *total_ms_avg, int *n);
/* The per-run times behind pu_ctx_kernel_ms, in launch order: up to `cap` runs into
 * traverse_ms[] (the traversal launch alone) and total_ms[] (P + traversal + reduction);
 * *n = the number written.  bench.py takes medians of these. */
int pu_ctx_kernel_times(pu_ctx *ctx, double *traverse_ms, double *total_ms, int cap, int *n);
/* The traversal's compulsory HBM bytes per launch for the current plan, after a run:
 * out[0] parents written (CLVs of every storing op and the root), out[1] scalers written
 * (in steady state: only the non-zero wave tiles under TV_SKIP_ZERO_SCALE), out[2] tip data
 * read, out[3] parents read back from HBM (stash overflow, CLV + scaler), out[4] sitewise
 * lnL written + pattern weights read.  bench.py checks its PMC traffic against the sum. */
int pu_ctx_traffic(pu_ctx *ctx, int64_t out[5]);
/* The traversal plan of the current schedule (r05): out[10] = {launch grid, k_prune build
 * (1 default, 7 the 7-wave build, -1 chosen at enqueue), kernel variant bits (pu_internal.h
 * TV_*), LDS stash slots, staging chunks, LDS pad bytes, 64-site tiles, blocks, unused tiles
 * per layout row (PU_PITCH_EXTRA), tiles per layout row}. */
int pu_ctx_plan_info(const pu_ctx *ctx, int32_t out[10]);
/* With pu_ctx_profile(ctx, 1), also the mean kernel time of the edge reductions
 * (pu_edge_lnl / pu_edge_derivs / the Newton evaluations of pu_optimise_*), in ms. */
int pu_ctx_edge_kernel_ms(pu_ctx *ctx, double *kernel_ms_avg, int *n);
/* The same, plus the mean time of the k_edge launch alone (before its reduction launch). */
int pu_ctx_edge_kernel_ms2(pu_ctx *ctx, double *kernel_ms_avg, double *edge_ms_avg, int *n);

#ifdef __cplusplus
}
#endif
#endif /* PHYLO_HIP_H */
