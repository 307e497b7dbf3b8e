"""`bench.py --gpus 2` end to end on the GPU box: no launcher environment, so bench starts
both ranks itself (bench.spawn_ranks); PU_BENCH_BACKEND=gloo puts both ranks on the one GPU
(RCCL refuses two ranks per device).  The site-sharded lnL it reports (the per-step
all-reduce, SURVEY 8(e) G1 / bin/phy.py:146's sum) must equal the one-rank lnL of the
concatenated sites, from the CPU oracle."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_gpus2_spawns_ranks_and_sums_site_shards(oracle_mod):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env["PU_BENCH_BACKEND"] = "gloo"
    S = 3000
    r = subprocess.run([sys.executable, "-u", "bench.py", "--gpus", "2", "--sites", str(S),
                        "--steps", "5", "--warmup", "2", "--warm-seconds", "0",
                        "--no-cpu-baseline"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["total_sites"] == 2 * S
    assert 0 < out["roofline"]["frac"] <= 1
    # r06: the line verifies itself -- the ranks the collective spans, and the job's lnL
    # against every rank's oracle lnL summed by the same collective
    assert out["rccl_world"] == 2 and out["rank_check"]["backend"] == "gloo"
    assert out["lnl_rel_err_vs_cpu"] <= 1e-9 and out["sitewise_max_rel_err_vs_cpu"] <= 1e-9

    from phylo_utils_amd import substitution_models as SM
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import CFG2_FREQS, CFG2_GTR_RATES, random_tree, simulate_states
    from phylo_utils_amd.tree import Traversal, prepare_tree
    model = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
    rm = GammaRateModel(4, 0.5)
    tree = random_tree(np.random.default_rng(1234), 50)        # bench.py's generator
    parts = [simulate_states(np.random.default_rng(1000 + k), tree, model, rm.rates, S)
             for k in range(2)]
    tr = Traversal(prepare_tree(tree))
    eye = np.eye(4)
    tips = {node: eye[np.concatenate([p[name] for p in parts])]
            for name, node in tr.names.items()}
    ev, el, iv = model.engine_eigen()
    lnl, _ = oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                 tr.root_length(), ev, el, iv, model.freqs, rm.rates, rm.weights,
                                 n_nodes=tr.n_nodes)
    assert abs(out["lnl"] - lnl) <= 1e-9 * abs(lnl), (out["lnl"], lnl)


def _bench(args, gloo=True, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    if gloo:
        env["PU_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, "-u", "bench.py"] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("config,taxa,total", [("cfg2", 50, 5000), ("cfg4", 1000, 3000)])
def test_bench_strong_scaling_total_sites_fixed(config, taxa, total):
    """--total-sites: one alignment split over the ranks (strong scaling, BASELINE cfg4 as
    stated: `bench.py --gpus 8 --config cfg4 --total-sites 1000000`, rehearsed here on the
    1000-taxon cfg4 tree with 2 gloo ranks).  Two gloo ranks on the one GPU report the same
    total lnL as one rank over all sites (bin/phy.py:146's sum), `total_sites` is the same, and
    `scaling` says strong."""
    common = ["--config", config, "--total-sites", str(total), "--steps", "3", "--warmup", "1",
              "--warm-seconds", "0", "--no-cpu-baseline"]
    one = _bench(["--gpus", "1"] + common)
    two = _bench(["--gpus", "2"] + common)
    for out, n in ((one, 1), (two, 2)):
        assert out["n_gpus"] == n and out["scaling"] == "strong"
        assert out["config"]["total_sites"] == total
        assert out["config"]["updates_per_step"] == (taxa - 1) * total * 4
    assert abs(two["lnl"] - one["lnl"]) <= 1e-10 * abs(one["lnl"]), (two["lnl"], one["lnl"])
    assert two["rccl_world"] == 2 and two["lnl_rel_err_vs_cpu"] <= 1e-9
    assert abs(two["rank_check"]["lnl_job_cpu"] - one["lnl"]) <= 1e-9 * abs(one["lnl"])


def test_bench_trees_two_ranks_check_every_tree():
    """cfg5's tree-sharded line at world 2 (gloo on the one GPU, 6 trees per rank at 5000
    sites): the ranks' trees checked against the oracle, the collective's size reported; one
    rank reports a cpu_baseline and the accuracy instead."""
    common = ["--config", "cfg5", "--trees", "6", "--sites", "5000", "--steps", "3",
              "--warmup", "1", "--warm-seconds", "0", "--cpu-seconds", "5"]
    two = _bench(["--gpus", "2"] + common)
    assert two["n_gpus"] == 2 and two["config"]["total_trees"] == 12
    assert two["rccl_world"] == 2 and two["lnl_rel_err_vs_cpu"] <= 1e-9
    one = _bench(["--gpus", "1"] + common)
    assert one["cpu_baseline"]["kind"] == "port" and one["accuracy_trees"] >= 1
    assert one["lnl_rel_err_vs_cpu"] <= 1e-9
