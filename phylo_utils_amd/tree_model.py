"""TreeModel on the GPU -- mirror of ``phylo_utils/tree_model.py`` (TreeModel :12-217).

Same methods and call order as the reference (``set_alignment``,
``set_substitution_model``, ``set_rate_model``, ``set_tree``, ``initialise``,
``compute_partials``, ``compute_partials_at_edge``, ``compute_likelihood_at_edge``),
but everything between "tips uploaded" and "sitewise lnL" happens in HBM in one
``pu_run`` (P matrices, the whole post-order, the root combine, ``lnl_node``,
the logsumexp over categories and the pattern-weighted sum).  ``partials``,
``scale``, ``root_partials`` and ``root_scale`` are fetched lazily from the device
with the reference's shapes ([node][site][category][state] etc.).
"""
from __future__ import annotations

import ctypes
import os
import logging

import numpy as np

from . import _native as N
from . import optimisation
from .alignment import alignment_to_codes, invariant_sites, partials_to_codes
from .tree import Traversal, prepare_tree

logger = logging.getLogger(__name__)


class _LazyPartials(object):
    """[ntaxa][S][K] view of coded tips, materialised per row on demand."""

    def __init__(self, codes, table):
        self.codes, self.table = codes, table
        self.shape = codes.shape + (table.shape[1],)

    def __getitem__(self, i):
        return self.table[self.codes[i]]

    def __array__(self, dtype=None, copy=None):
        a = self.table[self.codes]
        return a if dtype is None else a.astype(dtype)

    def __mul__(self, other):
        return np.asarray(self) * other


class TreeModel(object):
    alignment = None
    ascbias = False

    def __init__(self, device=0, keep_partials=True, compact_tips=True, reorder=True):
        self.device = device
        self.keep_partials = keep_partials
        self.compact_tips = compact_tips
        self.reorder = reorder
        self._ctx = None
        self._slot_names = None
        self._dirty = True
        self._lnl = None
        self._site_valid = False
        self._tips_owner = None

    # ------------------------------------------------------------------ inputs
    def set_alignment(self, alignment, alphabet, compress=True):
        """tree_model.py:42-50 (Biopython-free: [(name, seq)], dict or .name/.seq records).
        Tips are kept as codes (alignment_to_codes); the pattern compression runs on this
        model's device with np.unique's exact result (pu_compress_patterns).  The
        `alignment` attribute reads as the reference's [ntaxa][S][K] partials."""
        codes, table, sw, ii, names = alignment_to_codes(alignment, alphabet, compress,
                                                          self.device)
        if self.compact_tips:
            self._codes = (codes, table)
            self.alignment = _LazyPartials(codes, table)
        else:  # dense fp64 tips (pu_set_tip_partials)
            self._codes = None
            self.alignment = np.ascontiguousarray(table[codes])
        self.inverse_index = ii
        self.siteweights = sw
        self.names = names
        self._tips_owner = None
        self._free()

    def set_alignment_partials(self, partials, names, siteweights=None, inverse_index=None):
        """Tip partials given directly ([ntaxa][S][K]), e.g. for synthetic data."""
        self._codes = None
        self.alignment = np.ascontiguousarray(partials, dtype=np.float64)
        S = self.alignment.shape[1]
        self.siteweights = np.ones(S) if siteweights is None else np.asarray(siteweights)
        self.inverse_index = np.arange(S) if inverse_index is None else np.asarray(inverse_index)
        self.names = dict(names) if isinstance(names, dict) else {n: i for i, n in enumerate(names)}
        self._tips_owner = None
        self._free()

    def set_alignment_codes(self, codes, table, names, siteweights=None):
        """Compact tips directly: codes uint8 [ntaxa][S] into table [n_codes][K] (the engine's
        native tip format; avoids materialising [ntaxa][S][K] partials for large inputs)."""
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        table = np.ascontiguousarray(table, dtype=np.float64)
        self._codes = (codes, table)
        self.alignment = _LazyPartials(codes, table)
        S = codes.shape[1]
        self.siteweights = np.ones(S) if siteweights is None else np.asarray(siteweights)
        self.inverse_index = np.arange(S)
        self.names = {n: i for i, n in enumerate(names)}
        self._tips_owner = None
        self._free()

    def share_alignment(self, owner):
        """Read `owner`'s resident alignment instead of uploading a copy (r06, SURVEY 8(e) G2:
        one alignment per GPU for many trees; the reference swaps trees on one alignment,
        tree_model.py:42-50, 87-89).  `owner` is a TreeModel on the same device whose
        alignment is coded (compact tips); this model's context borrows owner's tip codes,
        code table and pattern weights (pu_share_tips), which then stay frozen in both.  The
        storage lives as long as any model holding it."""
        if not isinstance(owner, TreeModel) or owner is self:
            raise ValueError("share_alignment needs another TreeModel")
        if owner.device != self.device:
            raise ValueError("share_alignment: models on devices %d and %d"
                             % (owner.device, self.device))
        owner._ensure()  # the owner's context holds the tips
        self._codes = getattr(owner, "_codes", None)
        self.alignment = owner.alignment
        self.siteweights = owner.siteweights
        self.inverse_index = owner.inverse_index
        self.names = owner.names
        self.compact_tips = owner.compact_tips
        self._free()
        self._tips_owner = owner

    def get_empirical_freqs(self, pseudocount=None, include_ambiguous=False):
        """tree_model.py:52-73."""
        if self.alignment is None:
            logger.error("No alignment has been set")
            return 0
        counts = (self.alignment * self.siteweights[np.newaxis, :, np.newaxis]).sum((0, 1))
        if pseudocount is not None:
            try:
                counts = counts + np.array(pseudocount)
            except (TypeError, ValueError):
                logger.warning("Pseudocount %s ignored", pseudocount)
        return counts / counts.sum()

    def set_substitution_model(self, model):
        self.substitution_model = model
        self._dirty = True
        if self._ctx is not None:
            self._upload_model()

    def set_rate_model(self, rate_model):
        if self._ctx is not None and getattr(self, "rate_model", None) is not None \
                and rate_model.ncat != self.rate_model.ncat:
            self._free()
        self.rate_model = rate_model
        self._dirty = True
        if self._ctx is not None:
            self._upload_model()

    def set_tree(self, tree):
        """tree_model.py:87-89; `tree` is a newick string or a phylo_utils_amd.tree.Tree.
        A device context built for the same taxa is kept: the next initialise() only
        re-binds the tips to the new node numbering (pu_set_tip_nodes) and plans the new
        schedule -- no tip data are uploaded again (many trees on one alignment)."""
        self.tree = prepare_tree(tree)
        self.traversal = Traversal(self.tree)
        self._dirty = True

    def set_ascertainment_bias_correction(self, weighted=False):
        """Lewis ascertainment-bias correction (tree_model.py:92-98): K dummy invariant
        sites are appended (:151-156) and lnL_s -= log(1 - P(invariant)) (:209-214).

        weighted=False reproduces the reference exactly: P(invariant) sums the dummy
        sites' lnl_node values over categories WITHOUT the category weights (:213), which
        exceeds 1 -- and gives NaN -- for Gamma rates with C > 1.
        weighted=True uses the weighted mixture sum_c w_c (the Lewis correction)."""
        if np.any(invariant_sites(np.asarray(self.alignment))):
            logger.warning("Using Lewis ascertainment bias correction on an alignment with "
                           "invariant sites!")
        self.ascbias = True
        self._asc_mode = 2 if weighted else 1
        self._free()  # the context is rebuilt with the K dummy patterns

    # ------------------------------------------------------------------ device context
    def _free(self):
        if self._ctx is not None:
            N.lib().pu_ctx_destroy(self._ctx)
            self._ctx = None
        self._slot_names = None  # taxon of each tip slot of the context
        self._dirty = True

    def __del__(self):
        try:
            self._free()
        except Exception:
            pass

    def _upload_model(self):
        fr = N.f64(self.substitution_model.freqs)
        rates = N.f64(self.rate_model.rates)
        w = N.f64(self.rate_model.weights)
        if len(rates) != self.rate_model.ncat:
            raise ValueError("rate model has %d rates for ncat=%d" % (len(rates),
                                                                       self.rate_model.ncat))
        if self._host_p():
            # non-reversible: no eigen-decomposition; P = expm(Q r t) comes from the host
            # before every traversal (_upload_pmatrices)
            N.check(N.lib().pu_set_model_p(self._ctx, N.ptr(fr), N.ptr(rates), N.ptr(w)),
                    self._ctx, "pu_set_model_p")
            # the edge operations and optimisers choose lengths inside the library: they ask
            # the host for P, dP/dt, d2P/dt2 through this provider
            self._pm_provider = N.PMAT_PROVIDER(self._provide_pmatrices)
            N.check(N.lib().pu_set_pmatrix_provider(self._ctx, self._pm_provider, None),
                    self._ctx, "pu_set_pmatrix_provider")
        else:
            ev, el, iv = self.substitution_model.engine_eigen()
            N.check(N.lib().pu_set_model(self._ctx, N.ptr(ev), N.ptr(el), N.ptr(iv), N.ptr(fr),
                                         N.ptr(rates), N.ptr(w)), self._ctx, "pu_set_model")
        self._dirty = True

    def _provide_pmatrices(self, _user, order, n, t_ptr, out_ptr):
        """pu_pmat_provider: out[i] = d^order/dt^order P(t[i] r) of the current models
        (Model.p_derivative; order 0 is Model.p, as _upload_pmatrices).  Returns 0, or 1 after
        an exception (the library then reports the failure)."""
        try:
            rates = np.asarray(self.rate_model.rates, dtype=np.float64)
            K = len(self.substitution_model.freqs)
            t = np.ctypeslib.as_array(t_ptr, shape=(n,))
            out = np.ctypeslib.as_array(out_ptr, shape=(n, len(rates), K, K))
            for i in range(n):
                out[i] = self.substitution_model.p_derivative(float(t[i]), rates, order)
            return 0
        except Exception:  # noqa: BLE001 -- must not unwind through the C frames
            return 1

    def _host_p(self):
        return not getattr(self.substitution_model, "reversible", True)

    def _upload_pmatrices(self):
        """The transition matrices of the current lengths, computed exactly as the reference
        does per op (Model.p: tree_model.py:166-169 and :189-190 for the root edge; for the
        non-reversible models expm(Q r t), abstract.py:172-177), in the caller's op order
        and child order (pu_set_pmatrices)."""
        tr = self.traversal
        rates = self.rate_model.rates
        p = self.substitution_model.p
        bl = tr.op_lengths()
        P = [np.stack([p(l1, rates), p(l2, rates)]) for l1, l2 in bl]
        P.append(np.stack([p(0, rates), p(tr.root_length(), rates)]))
        P = N.f64(np.stack(P))
        N.check(N.lib().pu_set_pmatrices(self._ctx, N.ptr(P)), self._ctx, "pu_set_pmatrices")

    def initialise(self):
        """Allocate HBM buffers, upload tips/model/schedule, run compute_partials
        (tree_model.py:101-158)."""
        if self.alignment is None or not hasattr(self, "traversal"):
            raise ValueError("set_alignment and set_tree before initialise")
        n_leaves, S, K = self.alignment.shape
        C = self.rate_model.ncat
        tr = self.traversal
        Sx = S + K if self.ascbias else S  # + K dummy invariant sites (tree_model.py:113-114)
        if set(tr.names) != set(self.names):
            missing = sorted(set(tr.names) ^ set(self.names))[:5]
            raise ValueError("tree and alignment taxa differ, e.g. %s" % missing)
        ops = np.ascontiguousarray(tr.postorder_traversal, dtype=np.int32)
        bl = N.f64(tr.op_lengths())
        a, b = tr.root_edge
        if self._ctx is not None and self._slot_names is not None and \
                self._ctx_shape == (tr.n_nodes, n_leaves, Sx, C, K):
            # same taxa and sizes, new topology: re-bind the resident tips, plan the tree
            nodes = np.array([tr.names[n] for n in self._slot_names], dtype=np.int32)
            N.check(N.lib().pu_set_tip_nodes(self._ctx, len(nodes), N.ptr(nodes)), self._ctx,
                    "pu_set_tip_nodes")
            N.check(N.lib().pu_set_schedule(self._ctx, len(ops), N.ptr(ops), N.ptr(bl), a, b,
                                            tr.root_length()), self._ctx, "pu_set_schedule")
            self.compute_partials()
            return
        owner = self._tips_owner
        if owner is not None:
            owner._ensure()  # (re)built with its tips if it was freed meanwhile
            osh = owner._ctx_shape if owner._ctx is not None else None
            # tips, table and weights depend on the taxa, patterns and states, not on C
            if osh is None or (osh[1], osh[2], osh[4]) != (n_leaves, Sx, K) or \
                    owner.ascbias != self.ascbias:
                raise ValueError("share_alignment: the owner's context (%s) does not hold this "
                                 "model's alignment" % (osh,))
        self._free()
        flags = (N.PU_KEEP_PARTIALS if self.keep_partials else N.PU_LNL_ONLY) | \
            (0 if self.reorder else N.PU_NO_REORDER)
        ctx = ctypes.c_void_p()
        N.check(N.lib().pu_ctx_create(ctypes.byref(ctx), self.device, tr.n_nodes, n_leaves, Sx,
                                      C, K, flags), None, "pu_ctx_create")
        self._ctx = ctx
        if owner is not None:
            nodes = np.array([tr.names[n] for n in owner._slot_names], dtype=np.int32)
            N.check(N.lib().pu_share_tips(ctx, owner._ctx, len(nodes), N.ptr(nodes)), ctx,
                    "pu_share_tips")
            self._slot_names = list(owner._slot_names)
            self._ctx_shape = (tr.n_nodes, n_leaves, Sx, C, K)
            if self.ascbias:
                N.check(N.lib().pu_set_ascertainment(ctx, self._asc_mode, S), ctx,
                        "pu_set_ascertainment")
            self._upload_model()
            N.check(N.lib().pu_set_schedule(ctx, len(ops), N.ptr(ops), N.ptr(bl), a, b,
                                            tr.root_length()), ctx, "pu_set_schedule")
            self.compute_partials()
            return
        enc = getattr(self, "_codes", None) if isinstance(self.alignment, _LazyPartials) \
            else None
        if enc is None and self.compact_tips:
            enc = partials_to_codes(np.asarray(self.alignment))
        eye = np.eye(K)
        if enc is not None and self.ascbias:
            # dummy site k: every tip is the one-hot vector of state k (tree_model.py:151-156)
            codes, table = enc
            ids = []
            for k in range(K):
                hit = np.nonzero((table == eye[k]).all(axis=1))[0]
                if len(hit):
                    ids.append(int(hit[0]))
                else:
                    table = np.vstack([table, eye[k]])
                    ids.append(len(table) - 1)
            enc = None if len(table) > 256 else (
                np.ascontiguousarray(np.hstack([codes, np.tile(np.array(ids, dtype=np.uint8),
                                                               (len(codes), 1))])),
                np.ascontiguousarray(table))
        if enc is not None:
            codes, table = enc
            N.check(N.lib().pu_set_code_table(ctx, len(table), N.ptr(table)), ctx,
                    "pu_set_code_table")
        for name, node in tr.names.items():
            row = self.names[name]
            if enc is not None:
                cd = np.ascontiguousarray(enc[0][row])
                N.check(N.lib().pu_set_tip_codes(ctx, node, N.ptr(cd)), ctx, "pu_set_tip_codes")
            else:
                tp = np.asarray(self.alignment[row])
                if self.ascbias:
                    tp = np.vstack([tp, eye])
                tp = np.ascontiguousarray(tp, dtype=np.float64)
                N.check(N.lib().pu_set_tip_partials(ctx, node, N.ptr(tp)), ctx,
                        "pu_set_tip_partials")
        self._slot_names = list(tr.names)  # tip slot i holds this taxon
        self._ctx_shape = (tr.n_nodes, n_leaves, Sx, C, K)
        w = N.f64(np.concatenate([self.siteweights, np.zeros(Sx - S)]))
        N.check(N.lib().pu_set_pattern_weights(ctx, N.ptr(w)), ctx, "pu_set_pattern_weights")
        if self.ascbias:
            N.check(N.lib().pu_set_ascertainment(ctx, self._asc_mode, S), ctx,
                    "pu_set_ascertainment")
        self._upload_model()
        N.check(N.lib().pu_set_schedule(ctx, len(ops), N.ptr(ops), N.ptr(bl), a, b,
                                        tr.root_length()), ctx, "pu_set_schedule")
        self.compute_partials()

    def update_branch_lengths(self):
        """Re-read branch lengths from self.traversal.brlens (same topology)."""
        bl = N.f64(self.traversal.op_lengths())
        N.check(N.lib().pu_set_branch_lengths(self._ctx, N.ptr(bl),
                                              self.traversal.root_length()), self._ctx,
                "pu_set_branch_lengths")
        self._dirty = True

    def compute_partials(self):
        """One post-order traversal (tree_model.py:160-176) -- fused with the root combine
        and lnL reduction in a single device pass."""
        if self._ctx is None:
            raise ValueError("initialise first")
        if self._host_p():
            self._upload_pmatrices()
        lnl = ctypes.c_double()
        N.check(N.lib().pu_run(self._ctx, ctypes.byref(lnl), None), self._ctx, "pu_run")
        self._lnl = lnl.value
        self._dirty = False
        self._site_valid = True

    def _ensure(self):
        if self._ctx is None:
            self.initialise()
        elif self._dirty:
            self.compute_partials()

    def _check_edge(self, node_a, node_b):
        try:
            self.traversal.brlens[node_a, node_b]
        except KeyError:
            raise ValueError("There is no edge connecting nodes {} and {}".format(node_a, node_b))

    def _is_root_edge(self, node_a, node_b):
        return (node_a, node_b) == tuple(self.traversal.root_edge)

    def _edge_lnl(self, node_a, node_b):
        """Root on edge (a, b) over the nodes' current partials (pu_edge_lnl)."""
        self._check_edge(node_a, node_b)
        self._ensure()
        if not self.keep_partials:
            raise ValueError("compute_likelihood_at_edge off the root edge needs "
                             "keep_partials=True (PU_LNL_ONLY reuses CLV storage)")
        site = np.empty(self._n_patterns())
        lnl = ctypes.c_double()
        N.check(N.lib().pu_edge_lnl(self._ctx, int(node_a), int(node_b), ctypes.byref(lnl),
                                    N.ptr(site)), self._ctx, "pu_edge_lnl")
        self._site_valid = False  # the device sitewise/root buffers now hold this edge
        return lnl.value, site

    def compute_partials_at_edge(self, node_a, node_b):
        """Root combine on edge (a, b) (tree_model.py:178-198) -> (root_partials, root_scale).
        As in the reference, any edge is accepted and the nodes' current partials are used
        ("only valid if the CLVs at a and b are valid", :181-182)."""
        if self._is_root_edge(node_a, node_b):
            self._check_edge(node_a, node_b)
            self._ensure()
            if not self._site_valid:
                self.compute_partials()
        else:
            self._edge_lnl(node_a, node_b)
        return self._root()

    def compute_likelihood_at_edge(self, node_a, node_b):
        """Sitewise log-likelihood, expanded to alignment columns (tree_model.py:200-217)."""
        if self._is_root_edge(node_a, node_b):
            self._check_edge(node_a, node_b)
            self._ensure()
            return self.sitewise_patterns()[self.inverse_index]
        return self._edge_lnl(node_a, node_b)[1][self.inverse_index]

    # ------------------------------------------------------------------ edges
    def edge_derivatives(self, node_a, node_b, length=None):
        """(lnL, dlnL/dt, d2lnL/dt2) at length t of edge (a, b) (current length when None):
        the rate mixture of lnl_branch_derivs (numba_likelihood_engine.py:49-57) summed
        over patterns, on the nodes' current partials."""
        self._check_edge(node_a, node_b)
        self._ensure()
        out = np.zeros(3)
        N.check(N.lib().pu_edge_derivs(self._ctx, int(node_a), int(node_b),
                                       -1.0 if length is None else float(length), N.ptr(out)),
                self._ctx, "pu_edge_derivs")
        return float(out[0]), float(out[1]), float(out[2])

    def update_partials(self, ops, brlens):
        """In place, in order: partials[p] = clv(P(l1), P(l2), partials[c1], partials[c2]) for
        ops [n][3] (p, c1, c2) -- e.g. the re-orientation rows of optimising_traversal."""
        self._ensure()
        ops = np.ascontiguousarray(ops, dtype=np.int32).reshape(-1, 3)
        bl = N.f64(brlens).reshape(-1, 2)
        if len(bl) != len(ops):
            raise ValueError("one (len1, len2) pair per op")
        N.check(N.lib().pu_update_partials(self._ctx, len(ops), N.ptr(ops), N.ptr(bl)),
                self._ctx, "pu_update_partials")
        self._site_valid = False

    def _pull_lengths(self):
        """Device branch lengths -> self.traversal.brlens (the reference's BranchLengths)."""
        tr = self.traversal
        bl = np.empty((len(tr.postorder_traversal), 2))
        rl = ctypes.c_double()
        N.check(N.lib().pu_get_branch_lengths(self._ctx, N.ptr(bl), ctypes.byref(rl)),
                self._ctx, "pu_get_branch_lengths")
        for (p, a, b), (la, lb) in zip(tr.postorder_traversal, bl):
            tr.brlens[tuple(sorted((int(p), int(a))))] = float(la)
            tr.brlens[tuple(sorted((int(p), int(b))))] = float(lb)
        tr.brlens[tuple(sorted(tr.root_edge))] = rl.value

    def _minimise_edge(self, node_a, node_b, t0, method, tol, bracket):
        """The reference's 1-D minimisers (brent / dbrent of src/optimisation.pyx:86-297) on
        -lnL(t) of edge (a, b) over `bracket`, from t0: pu_minimise_edge, the whole
        minimisation in one persistent launch where the device takes it (r06), otherwise the
        same state machine with one k_edge launch per evaluation.  PU_PY_MINIMISE=1: the
        Python restatement (phylo_utils_amd.optimisation) over pu_edge_derivs instead (the
        tests' check of the library's state machine).  Returns (t, lnL at t)."""
        lo, hi = float(bracket[0]), float(bracket[1])
        if not 0.0 < lo < hi:
            raise ValueError("bracket must satisfy 0 < lo < hi, got %r" % (bracket,))
        if not os.environ.get("PU_PY_MINIMISE"):
            out = np.zeros(3)
            t0c = min(max(float(t0), lo), hi)
            N.check(N.lib().pu_minimise_edge(self._ctx, int(node_a), int(node_b),
                                             1 if method == "brent" else 2, lo, t0c, hi,
                                             float(tol), N.ptr(out)),
                    self._ctx, "pu_minimise_edge")
            self.last_edge_evaluations = int(out[2])
            return float(out[0]), -float(out[1])
        last = [None, None]
        out3 = np.zeros(3)

        def ev(t):
            if last[0] != t:
                N.check(N.lib().pu_edge_derivs(self._ctx, int(node_a), int(node_b), float(t),
                                               N.ptr(out3)), self._ctx, "pu_edge_derivs")
                last[0], last[1] = t, (float(out3[0]), float(out3[1]))
            return last[1]

        out = np.zeros(3)
        t0 = min(max(float(t0), lo), hi)
        if method == "brent":
            optimisation.brent(lo, t0, hi, lambda t: -ev(t)[0], tol, out)
        else:
            optimisation.dbrent(lo, t0, hi, lambda t: -ev(t)[0], lambda t: -ev(t)[1], tol, out)
        self.last_edge_evaluations = int(out[2])
        return float(out[0]), -float(out[1])

    def optimise_edge(self, node_a, node_b, tol=1e-8, max_iter=50, method="newton",
                      bracket=(1e-8, 10.0)):
        """Optimise the length of edge (a, b) with the partials of a and b held fixed (valid
        for the root edge, or after re-orientation); returns (length, lnL).
        method "newton": Newton-Raphson in the library (pu_optimise_edge); "brent" /
        "dbrent": the reference's minimisers (src/optimisation.pyx) over `bracket`."""
        self._check_edge(node_a, node_b)
        self._ensure()
        if method in ("brent", "dbrent"):
            key = tuple(sorted((int(node_a), int(node_b))))
            t, lnl = self._minimise_edge(node_a, node_b, self.traversal.brlens[key], method,
                                         tol, bracket)
            self.traversal.brlens[key] = t
            self.update_branch_lengths()
            return t, lnl
        if method != "newton":
            raise ValueError("method must be 'newton', 'brent' or 'dbrent'")
        t, lnl = ctypes.c_double(), ctypes.c_double()
        N.check(N.lib().pu_optimise_edge(self._ctx, int(node_a), int(node_b), float(tol),
                                         int(max_iter), ctypes.byref(t), ctypes.byref(lnl)),
                self._ctx, "pu_optimise_edge")
        self._pull_lengths()
        self._dirty = True
        return t.value, lnl.value

    def _sweep_minimise(self, rows, method, tol, bracket):
        """One optimising-traversal pass with brent / dbrent per edge, driven from the host:
        re-orientation rows are in-place device updates (pu_update_partials) at the lengths
        found so far, every evaluation a k_edge launch; then one traversal at the new
        lengths.  (Newton runs the whole pass inside the library: pu_optimise_sweep.)"""
        tr = self.traversal
        L = lambda u, v: tr.brlens[tuple(sorted((int(u), int(v))))]
        n_eval = 0
        for row in rows:
            if row[0] >= 0:
                op = np.ascontiguousarray(row[:3], dtype=np.int32)
                bl = N.f64([L(row[0], row[1]), L(row[0], row[2])])
                N.check(N.lib().pu_update_partials(self._ctx, 1, N.ptr(op), N.ptr(bl)),
                        self._ctx, "pu_update_partials")
            if row[3] >= 0:
                key = tuple(sorted((int(row[3]), int(row[4]))))
                t, _ = self._minimise_edge(row[3], row[4], tr.brlens[key], method, tol,
                                           bracket)
                tr.brlens[key] = t
                n_eval += self.last_edge_evaluations
        self.update_branch_lengths()
        self.compute_partials()
        return n_eval

    def optimise_branch_lengths(self, tol=1e-8, max_iter=50, sweeps=1, lnl_tol=None,
                                method="newton", bracket=(1e-8, 10.0)):
        """Branch-length optimisation over the optimising traversal
        (Traversal.optimising_traversal, utils.py:137-188): per pass, every edge in turn is
        optimised on GPU-resident re-oriented partials -- Newton-Raphson (default), or the
        reference's brent / dbrent (src/optimisation.pyx) over `bracket`.  Repeats up to
        `sweeps` passes, stopping early when a pass gains less than `lnl_tol`.  Returns the
        lnL."""
        self._ensure()
        if not self.keep_partials:
            raise ValueError("branch-length optimisation needs keep_partials=True")
        if method not in ("newton", "brent", "dbrent"):
            raise ValueError("method must be 'newton', 'brent' or 'dbrent'")
        rows = np.ascontiguousarray(self.traversal.optimising_traversal, dtype=np.int32)
        prev = self._lnl
        for _ in range(int(sweeps)):
            if method != "newton":
                self.last_newton_iterations = self._sweep_minimise(rows, method, tol, bracket)
                if lnl_tol is not None and self._lnl - prev < lnl_tol:
                    break
                prev = self._lnl
                continue
            lnl, n_it = ctypes.c_double(), ctypes.c_int()
            N.check(N.lib().pu_optimise_sweep(self._ctx, len(rows), N.ptr(rows), float(tol),
                                              int(max_iter), ctypes.byref(lnl),
                                              ctypes.byref(n_it)), self._ctx,
                    "pu_optimise_sweep")
            self._lnl = lnl.value
            self._site_valid = True
            self.last_newton_iterations = n_it.value
            if lnl_tol is not None and self._lnl - prev < lnl_tol:
                break
            prev = self._lnl
        self._pull_lengths()
        return self._lnl

    # ------------------------------------------------------------------ outputs
    def likelihood(self):
        """Total lnL = sum of sitewise lnL over alignment columns (bin/phy.py:146)."""
        self._ensure()
        return self._lnl

    def _n_patterns(self):
        n = self.alignment.shape[1]
        return n + self.alignment.shape[2] if self.ascbias else n

    def sitewise_patterns(self):
        """Per-pattern lnL (tree_model.py:216, before the inverse-index expansion; with
        the ascertainment correction the K dummy patterns come last)."""
        self._ensure()
        if not self._site_valid:
            self.compute_partials()
        out = np.empty(self._n_patterns())
        N.check(N.lib().pu_get_site_lnl(self._ctx, N.ptr(out)), self._ctx, "pu_get_site_lnl")
        return out

    def node_partials(self, node):
        self._ensure()
        S, K = self._n_patterns(), self.alignment.shape[2]
        C = self.rate_model.ncat
        p = np.empty((S, C, K))
        s = np.empty((S, C))
        N.check(N.lib().pu_get_partials(self._ctx, int(node), N.ptr(p), N.ptr(s)), self._ctx,
                "pu_get_partials")
        return p, s

    @property
    def partials(self):
        """[2N-2][S][C][K], tips broadcast over categories (tree_model.py:117-148)."""
        return np.stack([self.node_partials(v)[0] for v in range(self.traversal.n_nodes)])

    @property
    def scale(self):
        return np.stack([self.node_partials(v)[1] for v in range(self.traversal.n_nodes)])

    def _root(self):
        self._ensure()
        S, K = self._n_patterns(), self.alignment.shape[2]
        C = self.rate_model.ncat
        rp = np.empty((S, C, K))
        rs = np.empty((S, C))
        N.check(N.lib().pu_get_root(self._ctx, N.ptr(rp), N.ptr(rs)), self._ctx, "pu_get_root")
        return rp, rs

    @property
    def root_partials(self):
        return self._root()[0]

    @property
    def root_scale(self):
        return self._root()[1]
