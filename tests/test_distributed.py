"""Multi-process sharding logic on the CPU: world_size 2, gloo backend.
The per-rank engine is the CPU oracle, injected through `engine_factory`; the
sharding, the lnL all-reduce and the sitewise / per-tree all-gathers are the
product code that runs with RCCL on the GPUs."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class OracleEngine(object):
    def __init__(self, tree, codes, table, names, siteweights, model, rate_model):
        import sys
        sys.path.insert(0, ROOT)
        from oracle import oracle as orc
        from phylo_utils_amd.tree import Traversal, prepare_tree
        tr = Traversal(prepare_tree(tree))
        tips = {tr.names[n]: table[codes[i]] for i, n in enumerate(names)}
        ev, el, iv = model.engine_eigen()
        self.lnl, self.site = orc.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(),
                                           tr.root_edge, tr.root_length(), ev, el, iv,
                                           model.freqs, rate_model.rates, rate_model.weights,
                                           site_weights=siteweights, n_nodes=tr.n_nodes)

    def likelihood(self):
        return self.lnl

    def sitewise_patterns(self):
        return self.site


def _problem():
    from phylo_utils_amd import substitution_models as SM
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import make_problem, random_tree
    model = SM.HKY85(2.0, [0.1, 0.2, 0.3, 0.4])
    rm = GammaRateModel(4, 0.5)
    tree, names, states = make_problem(12, 301, model, rm.rates, seed=3)
    trees = [random_tree(np.random.default_rng(s), 12) for s in range(5)]  # same taxa t0..t11
    w = np.arange(1, 302, dtype=np.float64) % 3 + 1
    return model, rm, tree, trees, names, states.astype(np.uint8), np.eye(4), w


def _worker(rank, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from phylo_utils_amd.parallel import SiteShardedLikelihood, TreeShardedLikelihoods
        model, rm, tree, trees, names, codes, table, w = _problem()
        sh = SiteShardedLikelihood(tree, codes, table, names, model, rm, siteweights=w,
                                   engine_factory=OracleEngine)
        lnl = sh.likelihood()
        site = sh.sitewise_patterns()
        ts = TreeShardedLikelihoods(trees, codes, table, names, model, rm, siteweights=w,
                                    engine_factory=OracleEngine)
        tl = ts.likelihoods()
        np.savez(os.path.join(out_dir, "r%d.npz" % rank), lnl=lnl, site=site, trees=tl,
                 lo=sh.lo, hi=sh.hi)
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    from phylo_utils_amd.parallel import shard_range
    for n in (1, 7, 8, 100, 125_000):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


def test_site_and_tree_sharding_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    model, rm, tree, trees, names, codes, table, w = _problem()
    full = OracleEngine(tree, codes, table, names, w, model, rm)
    res = [np.load(tmp_path / ("r%d.npz" % r)) for r in range(WORLD)]
    for r in res:
        assert abs(float(r["lnl"]) - full.lnl) <= 1e-12 * abs(full.lnl)
        np.testing.assert_allclose(r["site"], full.site, rtol=0, atol=0)
        ref_trees = [OracleEngine(t, codes, table, names, w, model, rm).lnl for t in trees]
        np.testing.assert_allclose(r["trees"], ref_trees, rtol=1e-14)
    assert int(res[0]["hi"]) == int(res[1]["lo"])


def _ring_worker(rank, port, out_dir):
    """bench.py's LnlRing with gloo on the CPU: every step's value is summed over ranks,
    slots alternate, and a slot is reused only after its previous sum completed."""
    import sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from bench import LnlRing
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        ring = LnlRing(lambda: torch.zeros(1, dtype=torch.float64), WORLD,
                       lambda t: dist.all_reduce(t, async_op=True))
        seen = []

        def fill(slot):
            # the slot's previous all-reduce has completed: it holds that step's sum
            prev = float(ring.slots[slot][0])
            seen.append(prev)
            ring.slots[slot][0] = (rank + 1) * 1000.0 + ring.n

        for _ in range(7):
            ring.step(fill)
        ring.drain()
        np.savez(os.path.join(out_dir, "ring%d.npz" % rank), seen=np.array(seen),
                 last=float(ring.last()[0]), n=ring.n)
    finally:
        dist.destroy_process_group()


def _warm_worker(rank, port, out_dir):
    """bench.warm_for with ranks of different speeds: every rank runs the same number of
    batches, so the per-step collectives stay paired (a per-rank clock would not)."""
    import sys
    import time
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from bench import warm_for
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        sums = []

        def batch():
            time.sleep(0.01 * (1 + 3 * rank))  # rank 1 is 4x slower
            t = torch.ones(1, dtype=torch.float64)
            dist.all_reduce(t)
            sums.append(float(t[0]))

        n = warm_for(0.3, batch, WORLD)
        t = torch.tensor([12345.0 + rank])  # the next collective pairs with its peer's
        dist.all_reduce(t)
        np.savez(os.path.join(out_dir, "warm%d.npz" % rank), n=n, sums=np.array(sums),
                 after=float(t[0]))
    finally:
        dist.destroy_process_group()


def test_bench_warmup_agreed_across_ranks_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_warm_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    d = [np.load(tmp_path / ("warm%d.npz" % r)) for r in range(WORLD)]
    assert int(d[0]["n"]) == int(d[1]["n"]) >= 1
    for x in d:
        np.testing.assert_array_equal(x["sums"], 2.0)
        assert float(x["after"]) == 12345.0 * 2 + 1


def test_bench_lnl_ring_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_ring_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    for r in range(WORLD):
        d = np.load(tmp_path / ("ring%d.npz" % r))
        # step k (1-based) writes (rank + 1) * 1000 + k; the sum over 2 ranks is 3000 + 2k
        assert float(d["last"]) == 3000.0 + 2 * 7
        # steps 3..7 found the sum of step k - 2 in their slot
        np.testing.assert_array_equal(d["seen"][2:], [3000.0 + 2 * k for k in range(1, 6)])


class OracleTreeEngine(object):
    """CPU engine with TreeModel's edge interface (edge_derivatives, update_partials,
    update_branch_lengths, compute_partials, likelihood) over the oracle, for the sharded
    branch-length optimisation."""

    def __init__(self, tree, codes, table, names, siteweights, model, rate_model):
        import sys
        sys.path.insert(0, ROOT)
        from oracle import oracle as orc
        from phylo_utils_amd.tree import Traversal, prepare_tree
        self.orc = orc
        self.traversal = Traversal(prepare_tree(tree))
        self.tips = {self.traversal.names[n]: table[codes[i]] for i, n in enumerate(names)}
        self.model, self.rm = model, rate_model
        self.sw = np.asarray(siteweights, dtype=np.float64)
        self.eig = model.engine_eigen()
        self.compute_partials()

    def compute_partials(self):
        tr = self.traversal
        ev, el, iv = self.eig
        st = self.orc.tree_lnl(self.tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                               tr.root_length(), ev, el, iv, self.model.freqs, self.rm.rates,
                               self.rm.weights, site_weights=self.sw, n_nodes=tr.n_nodes,
                               return_all=True)
        self.lnl, self.partials, self.scale = st["lnl"], st["partials"], st["scale"]

    def update_branch_lengths(self):
        pass  # compute_partials reads traversal.brlens

    def likelihood(self):
        return self.lnl

    def edge_derivatives(self, a, b, t):
        ev, el, iv = self.eig
        return self.orc.edge_derivs(self.partials[a], self.scale[a], self.partials[b],
                                    self.scale[b], ev, el, iv, t, self.rm.rates, self.rm.weights,
                                    self.model.freqs, self.sw)

    def update_partials(self, ops, brlens):
        ev, el, iv = self.eig
        for (p, x, y), (l1, l2) in zip(np.asarray(ops), np.asarray(brlens)):
            P1 = self.orc.pmatrix(ev, el, iv, l1, self.rm.rates)
            P2 = self.orc.pmatrix(ev, el, iv, l2, self.rm.rates)
            cml = np.zeros(self.scale[p].shape)
            self.partials[p] = self.orc.clv_c(P1, P2, self.partials[x], self.partials[y],
                                              self.scale[x], self.scale[y], cml)
            self.scale[p] = cml


def _opt_worker(rank, port, out_dir, method):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from phylo_utils_amd.parallel import SiteShardedLikelihood
        model, rm, tree, trees, names, codes, table, w = _problem()
        sh = SiteShardedLikelihood(tree, codes, table, names, model, rm, siteweights=w,
                                   engine_factory=OracleTreeEngine)
        lnl = sh.optimise_branch_lengths(tol=1e-10, method=method)
        lens = sorted(sh.engine.traversal.brlens.items())
        np.savez(os.path.join(out_dir, "opt%d.npz" % rank), lnl=lnl,
                 keys=np.array([k for k, _ in lens]), vals=np.array([v for _, v in lens]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("method", ["newton", "dbrent"])
def test_site_sharded_branch_optimisation_gloo_world2(tmp_path, method):
    """G1 x N1: the optimising-traversal sweep over 2 site shards, every evaluation of the
    whole-alignment (lnL, d1, d2) summed by an all-reduce, against the same sweep on the
    whole alignment (oracle.optimise_sweep for Newton; oracle partials + dbrent for dbrent):
    lengths 1e-6 relative, lnL 1e-9; both ranks end with identical lengths."""
    import torch.multiprocessing as mp
    from phylo_utils_amd import optimisation as opt
    from phylo_utils_amd.tree import Traversal, prepare_tree
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc
    mp.spawn(_opt_worker, args=(_free_port(), str(tmp_path), method), nprocs=WORLD, join=True)
    model, rm, tree, trees, names, codes, table, w = _problem()
    tr = Traversal(prepare_tree(tree))
    tips = {tr.names[n]: table[codes[i]] for i, n in enumerate(names)}
    ev, el, iv = model.engine_eigen()
    edge_opt = None
    if method == "dbrent":
        def edge_opt(evaluate, t0):
            out = np.zeros(3)
            opt.dbrent(1e-8, min(max(t0, 1e-8), 10.0), 10.0, lambda t: -evaluate(t)[0],
                       lambda t: -evaluate(t)[1], 1e-10, out)
            return out[0]
    lens, lnl = orc.optimise_sweep(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                   tr.root_length(), ev, el, iv, model.freqs, rm.rates,
                                   rm.weights, tr.optimising_traversal, tr.n_nodes,
                                   site_weights=w, tol=1e-10, edge_opt=edge_opt)
    res = [np.load(tmp_path / ("opt%d.npz" % r)) for r in range(WORLD)]
    np.testing.assert_array_equal(res[0]["vals"], res[1]["vals"])
    for r in res:
        assert abs(float(r["lnl"]) - lnl) <= 1e-9 * abs(lnl)
        for k, v in zip(r["keys"], r["vals"]):
            want = lens[tuple(int(x) for x in k)]
            assert abs(v - want) <= 1e-6 * max(want, 1e-3), (k, v, want)


class _FakeModel(object):
    """The two attributes bench.oracle_traversal reads from a TreeModel."""
    def __init__(self, tree, names):
        from phylo_utils_amd.tree import Traversal, prepare_tree
        self.traversal = Traversal(prepare_tree(tree))
        self.names = {n: i for i, n in enumerate(names)}


def _rank_check_worker(rank, port, out_dir):
    """bench.py's multi-rank self-check (r06) with gloo on the CPU: each rank runs the oracle
    on its own site shard in blocks, and rank_check reports the ranks the collective spans
    and the job's lnL against the summed oracle lnLs."""
    import sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    from phylo_utils_amd.parallel import shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        model, rm, tree, trees, names, codes, table, w = _problem()
        lo, hi = shard_range(codes.shape[1], rank, WORLD)
        fake = _FakeModel(tree, names)
        lnl, site, _ = bench.oracle_traversal(fake, model, rm, codes[:, lo:hi], 2, block=64)
        # the "GPU" value of this rehearsal: the whole alignment's lnL, as the ring holds it
        full = OracleEngine(tree, codes, table, names, np.ones(codes.shape[1]), model, rm)
        chk = bench.rank_check(dist, torch.device("cpu"), WORLD, full.lnl, lnl, 0.0,
                               "shard [%d, %d)" % (lo, hi))
        chk2 = bench.rank_check(dist, torch.device("cpu"), WORLD, float(site.sum()), lnl, 0.0,
                                "shard", gpu_local=True)
        np.savez(os.path.join(out_dir, "chk%d.npz" % rank), site=site, lo=lo, hi=hi,
                 world=chk["rccl_world"], rel=chk["lnl_rel_err_vs_cpu"],
                 cpu=chk["lnl_job_cpu"], rel2=chk2["lnl_rel_err_vs_cpu"],
                 gpu2=chk2["lnl_job_gpu"], backend=chk["backend"])
    finally:
        dist.destroy_process_group()


def test_bench_rank_check_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_rank_check_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    model, rm, tree, trees, names, codes, table, w = _problem()
    full = OracleEngine(tree, codes, table, names, np.ones(codes.shape[1]), model, rm)
    d = [np.load(tmp_path / ("chk%d.npz" % r)) for r in range(WORLD)]
    for x in d:
        assert int(x["world"]) == WORLD and str(x["backend"]) == "gloo"
        assert float(x["rel"]) <= 1e-13 and float(x["rel2"]) <= 1e-13
        assert abs(float(x["cpu"]) - full.lnl) <= 1e-13 * abs(full.lnl)
        assert abs(float(x["gpu2"]) - full.lnl) <= 1e-13 * abs(full.lnl)
    # the blocked oracle's sitewise values are the whole traversal's, shard by shard
    site = np.concatenate([x["site"] for x in d])
    np.testing.assert_allclose(site, full.site, rtol=1e-14, atol=0)


def test_oracle_traversal_reused_buffers_across_trees():
    """bench.oracle_traversal keeps its host buffers between calls of one shape (cfg5's trees):
    a tip node of one tree may be an internal node of the previous one, so its scaler is
    re-zeroed with the tip fill (a stale one gave rel-err ~1 on the first GPU run)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    model, rm, tree, trees, names, codes, table, w = _problem()
    ones = np.ones(codes.shape[1])
    for t in trees:
        lnl, site, secs = bench.oracle_traversal(_FakeModel(t, names), model, rm, codes, 2,
                                                 block=128)
        ref = OracleEngine(t, codes, table, names, ones, model, rm)
        assert abs(lnl - ref.lnl) <= 1e-13 * abs(ref.lnl)
        np.testing.assert_allclose(site, ref.site, rtol=1e-14, atol=0)
        assert secs > 0
