"""Several trees per launch (pu_batch): every tree's lnL and sitewise lnL
bitwise those of its own context's launch (the reference's per-tree loop, tree_model.py:87-89,
160-176), against the oracle, after new branch lengths, into a device output, and the
contexts a batch refuses."""
import ctypes

import numpy as np
import pytest

from phylo_utils_amd import TreeModel
from phylo_utils_amd import _native as N
from phylo_utils_amd import substitution_models as SM
from phylo_utils_amd.batch import TreeBatch
from phylo_utils_amd.rate_models import GammaRateModel
from phylo_utils_amd.synthetic import CFG2_FREQS, CFG2_GTR_RATES, random_tree, simulate_states

pytestmark = pytest.mark.gpu

LNL_RTOL = 1e-12


def _alignment(n_taxa, n_sites, model, rm, seed):
    tree = random_tree(np.random.default_rng(seed), n_taxa)
    st = simulate_states(np.random.default_rng(seed + 1), tree, model, rm.rates, n_sites)
    names = sorted(st, key=lambda s: int(s[1:]))
    return names, np.stack([st[n] for n in names]).astype(np.uint8)


def _models(n_trees, n_taxa, n_sites, keep=False, seed=5, model=None, sites_of=None,
            share=False, ncat=4):
    rm = GammaRateModel(ncat, 0.5)
    model = model or SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    names, codes = _alignment(n_taxa, n_sites, model, rm, seed)
    out = []
    for i in range(n_trees):
        tree = random_tree(np.random.default_rng(100 + i), n_taxa)
        tm = TreeModel(keep_partials=keep)
        c = codes if sites_of is None else codes[:, :sites_of(i)]
        if share and out:
            tm.share_alignment(out[0])
        else:
            tm.set_alignment_codes(c, np.eye(4), names)
        tm.set_substitution_model(model)
        tm.set_rate_model(rm)
        tm.set_tree(tree)
        tm.initialise()
        out.append(tm)
    return out


def _site(tm):
    out = np.empty(tm._n_patterns())
    N.check(N.lib().pu_get_site_lnl(tm._ctx, N.ptr(out)), tm._ctx, "pu_get_site_lnl")
    return out


@pytest.mark.parametrize("n_trees,n_taxa,n_sites", [(1, 8, 300), (5, 30, 5000), (12, 100, 9000)])
def test_batch_bitwise_equal_to_single_launches(n_trees, n_taxa, n_sites):
    tms = _models(n_trees, n_taxa, n_sites)
    single = [tm.likelihood() for tm in tms]
    site1 = [_site(tm) for tm in tms]
    b = TreeBatch(tms)
    for rep in range(3):  # the uploaded arguments are reused
        got = b.likelihoods()
        assert list(got) == single, (rep, got, single)
        for i, tm in enumerate(tms):
            np.testing.assert_array_equal(b.sitewise(i), site1[i])
    b.close()


def _oracle_lnl(orc, tm):
    tr = tm.traversal
    tips = {tr.names[n]: tm.alignment[i] for n, i in tm.names.items()}
    ev, el, iv = tm.substitution_model.engine_eigen()
    lnl, _ = orc.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                          tr.root_length(), ev, el, iv, tm.substitution_model.freqs, tm.rate_model.rates,
                          tm.rate_model.weights, n_nodes=tr.n_nodes, nthreads=8)
    return lnl


@pytest.mark.parametrize("env", [{"PU_BATCH_GROUP": "0"}, {"PU_BATCH_GROUP": "4"},
                                 {"PU_BATCH_GROUP": "8", "PU_BATCH_WAVES": "7"},
                                 {"PU_BATCH_GROUP": "16", "PU_BATCH_WAVES": "1"}])
def test_batch_grid_orders_bitwise(monkeypatch, env):
    """Every grid order of the batched traversal (tree-major, groups of g trees with a tile
    index's workgroups adjacent, the last group smaller) and both builds give each tree its
    own launch's lnL and sitewise lnL bit for bit (11 trees: groups of 4 end with 3)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    tms = _models(11, 40, 6000, seed=9)
    single = [tm.likelihood() for tm in tms]
    site1 = [_site(tm) for tm in tms]
    b = TreeBatch(tms)
    got = b.likelihoods()
    assert list(got) == single
    for i in range(len(tms)):
        np.testing.assert_array_equal(b.sitewise(i), site1[i])
    b.close()


def test_batch_against_oracle_and_new_lengths(oracle_mod):
    tms = _models(4, 20, 3000)
    b = TreeBatch(tms)
    got = b.likelihoods()
    for i, tm in enumerate(tms):
        ref = _oracle_lnl(oracle_mod, tm)
        assert abs(got[i] - ref) <= LNL_RTOL * abs(ref), (i, got[i], ref)
    # new branch lengths on two trees: the batch follows, bitwise the single launch
    for j in (1, 3):
        tr = tms[j].traversal
        for e in list(tr.brlens):
            tr.brlens[e] = tr.brlens[e] * (0.8 + 0.1 * j)
        tms[j].update_branch_lengths()
    got2 = b.likelihoods()
    single2 = [tm.likelihood() for tm in tms]
    assert list(got2) == single2
    assert got2[0] == got[0] and got2[2] == got[2]
    assert got2[1] != got[1] and got2[3] != got[3]
    b.close()


def test_batch_follows_new_topologies_and_rebuilt_contexts():
    """set_tree on a model keeps its context and re-plans it (the batch re-uploads that tree's
    arguments); a model whose context is rebuilt (another rate model) is picked up too."""
    tms = _models(4, 24, 3000, seed=13)
    b = TreeBatch(tms)
    b.likelihoods()
    tms[2].set_tree(random_tree(np.random.default_rng(777), 24))
    tms[2].initialise()
    got = b.likelihoods()
    assert list(got) == [tm.likelihood() for tm in tms]
    # 4 -> 2 categories: every context is destroyed and created again (the allocator may
    # hand out the same address; the batch reads its contexts afresh at every enqueue)
    for i in range(4):
        tms[i].set_rate_model(GammaRateModel(2, 0.7))
        tms[i].initialise()
    got = b.likelihoods()
    assert list(got) == [tm.likelihood() for tm in tms]
    b.close()


def test_batch_device_output_and_stream():
    import torch
    tms = _models(6, 24, 4000)
    single = np.array([tm.likelihood() for tm in tms])
    out = torch.zeros(len(tms), dtype=torch.float64, device="cuda")
    st = torch.cuda.Stream()
    for tm in tms:  # the contexts on the batch's stream too: no joins
        N.check(N.lib().pu_ctx_set_stream(tm._ctx, ctypes.c_void_p(st.cuda_stream)), tm._ctx)
    b = TreeBatch(tms)
    b.set_stream(st.cuda_stream)
    for _ in range(2):
        b.enqueue(out.data_ptr())
    st.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), single)
    b.close()


def test_batch_refuses_what_it_cannot_run():
    keep = _models(2, 10, 500, keep=True)
    b = TreeBatch(keep)
    with pytest.raises(N.PhyloHipError, match="lnL-only"):
        b.enqueue()
    b.close()
    ragged = _models(2, 10, 500, sites_of=lambda i: 500 - 100 * i)
    b = TreeBatch(ragged)
    with pytest.raises(N.PhyloHipError, match="differ"):
        b.enqueue()
    b.close()


def test_shared_alignment_batch_bitwise_and_vs_oracle(oracle_mod):
    """One resident alignment for every tree (pu_share_tips, r06): the batch over models that
    borrow tree 0's tips gives exactly the lnL and sitewise lnL of models holding their own
    copies, agrees with the oracle, and the borrowed codes cost no device memory."""
    own = _models(6, 30, 5000, seed=21)
    shared = _models(6, 30, 5000, seed=21, share=True)
    ref = [tm.likelihood() for tm in own]
    assert [tm.likelihood() for tm in shared] == ref
    b = TreeBatch(shared)
    got = b.likelihoods()
    assert list(got) == ref
    for i, tm in enumerate(own):
        np.testing.assert_array_equal(b.sitewise(i), _site(tm))
    for i in (0, 3):
        r = _oracle_lnl(oracle_mod, shared[i])
        assert abs(got[i] - r) <= LNL_RTOL * abs(r), (i, got[i], r)
    lib = N.lib()
    b_own = [lib.pu_ctx_device_bytes(tm._ctx) for tm in own]
    b_sh = [lib.pu_ctx_device_bytes(tm._ctx) for tm in shared]
    codes = 30 * 5000
    assert b_sh[0] == b_own[0]
    assert all(o - s_ == codes for o, s_ in zip(b_own[1:], b_sh[1:])), (b_own, b_sh)
    b.close()


def test_shared_tips_are_frozen_and_outlive_their_owner():
    tms = _models(3, 16, 2000, seed=23, share=True)
    ref = [tm.likelihood() for tm in tms]
    lib = N.lib()
    w = np.ones(2000)
    for tm in tms:  # owner and borrowers alike
        assert lib.pu_set_pattern_weights(tm._ctx, N.ptr(w)) == N.PU_E_STATE
        assert b"frozen" in lib.pu_last_error(tm._ctx)
    # the owner's context goes first: the borrowers keep reading the same tips
    tms[0]._free()
    assert [tm.likelihood() for tm in tms[1:]] == ref[1:]
    b = TreeBatch(tms[1:])
    assert list(b.likelihoods()) == ref[1:]
    b.close()
    # a new topology re-binds the borrowed tips (pu_set_tip_nodes), as for owned ones
    own = _models(1, 16, 2000, seed=23)[0]
    for tm in (tms[2], own):
        tm.set_tree(random_tree(np.random.default_rng(4242), 16))
        tm.initialise()
    assert tms[2].likelihood() == own.likelihood()


def test_share_tips_refuses_mismatches():
    a = _models(1, 12, 1000, seed=3)[0]
    other = _models(1, 12, 900, seed=3)[0]
    lib = N.lib()
    nodes = np.arange(12, dtype=np.int32)
    assert lib.pu_share_tips(other._ctx, a._ctx, 12, N.ptr(nodes)) != 0  # has its own tips
    tree = random_tree(np.random.default_rng(9), 12)
    tm = TreeModel()  # keeps its partials (a = lnL-only owner): sharing is about the tips only
    tm.share_alignment(a)
    tm.set_substitution_model(a.substitution_model)
    tm.set_rate_model(a.rate_model)
    tm.set_tree(tree)
    a.set_tree(tree)
    a.initialise()
    assert tm.likelihood() == a.likelihood()
    with pytest.raises(ValueError):
        tm.share_alignment(tm)
    # a borrower of another site count is refused before any context is made
    tm2 = TreeModel()
    tm2.share_alignment(other)
    other.set_alignment_codes(np.zeros((12, 500), np.uint8), np.eye(4),
                              ["t%d" % i for i in range(12)])
    tm2.set_substitution_model(a.substitution_model)
    tm2.set_rate_model(a.rate_model)
    tm2.set_tree(tree)
    with pytest.raises(ValueError, match="taxa differ|does not hold"):
        tm2.initialise()


def test_batch_refuses_categories_not_dividing_4():
    """C = 3 leaves the category combine to k_site_lse, which the batch does not launch: it is
    refused, while each context alone still evaluates it."""
    tms = _models(2, 12, 800, ncat=3)
    b = TreeBatch(tms)
    with pytest.raises(N.PhyloHipError, match="C = 1, 2 or 4"):
        b.enqueue()
    b.close()


def test_batch_device_output_reaches_pu_synchronize_and_context_streams_follow():
    """lnl_dev given: pu_synchronize(ctx) reads the batch's entry for the tree (not a stale
    own output); contexts on their own streams wait for the batch before later work."""
    import torch
    tms = _models(4, 20, 3000, seed=31)
    single = [tm.likelihood() for tm in tms]
    out = torch.zeros(len(tms), dtype=torch.float64, device="cuda")
    b = TreeBatch(tms)
    # stale own outputs: a different length set evaluated per context first
    tr = tms[1].traversal
    for e in list(tr.brlens):
        tr.brlens[e] *= 1.3
    tms[1].update_branch_lengths()
    changed = tms[1].likelihood()
    for e in list(tr.brlens):
        tr.brlens[e] /= 1.3
    tms[1].update_branch_lengths()
    b.enqueue(out.data_ptr())
    # queued on tree 1's own stream right after the batch: ordered behind it
    site_after = b.sitewise(1)
    b.synchronize()
    v = ctypes.c_double()
    for i, tm in enumerate(tms):
        N.check(N.lib().pu_synchronize(tm._ctx, ctypes.byref(v)), tm._ctx)
        assert v.value == single[i] == float(out[i].item())
    assert single[1] != changed
    np.testing.assert_array_equal(site_after, _site(tms[1]))
    b.close()


def test_batch_does_not_write_root_partials():
    """r06: a batch skips the root partials' stores (nothing of a batched lnL-only tree reads
    them; cfg5: 1.0 of 4.84 GB per launch).  pu_get_root refuses after a batch run and gives the
    context's own run's root again after its next pu_run; the lnL is unchanged."""
    tms = _models(3, 16, 2000, seed=21)
    tm = tms[1]
    tm.compute_partials()
    rp0, rs0 = tm.root_partials.copy(), tm.root_scale.copy()
    l0 = tm.likelihood()
    b = TreeBatch(tms)
    got = b.likelihoods()
    assert got[1] == l0
    with pytest.raises(N.PhyloHipError, match="root partials"):
        tm.root_partials
    tm.compute_partials()
    np.testing.assert_array_equal(tm.root_partials, rp0)
    np.testing.assert_array_equal(tm.root_scale, rs0)
    assert tm.likelihood() == l0
    b.close()
