"""bench.py's own logic on the CPU: the rank launcher behind `bench.py --gpus N`, its refusal
of a mismatched launcher environment, and the roofline arithmetic (bytes actually moved,
frac <= 1; the SURVEY 8(d) algorithmic figure only as a labelled ratio).  The multi-rank run
of the real benchmark is tests/test_gpu_bench.py."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _run(code, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_spawn_ranks_gloo_world2():
    r = _run("import sys, bench; sys.exit(bench.spawn_ranks(2, ['tests/_rank_probe.py']))")
    assert r.returncode == 0, r.stderr
    assert "world=2 sum=3" in r.stdout


def test_spawn_ranks_reports_a_failing_rank():
    r = _run("import sys, bench; sys.exit(bench.spawn_ranks(2, ['tests/_rank_probe.py']))",
             {"PROBE_EXIT_RANK": "1"})
    assert r.returncode == 3, (r.returncode, r.stderr)


def test_bench_refuses_world_size_mismatch():
    env = {k: v for k, v in os.environ.items()}
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def _cfg2_counts():
    # cfg2 KEEP plan: 48 storing ops + root, 1563 tiles of 64 sites, C = 4, K = 4
    padS, C, K = 1563 * 64, 4, 4
    return np.array([49 * padS * C * K * 8, 0, 50 * padS, 0, 2 * 100_000 * 8], dtype=np.int64)


def test_roofline_from_measured_bytes_is_a_fraction():
    ev = {"trav_med": 0.13711, "n": 200}
    alg = 19_600_000 * 120 + 100_000 * 4 * 8 + 100_000 * 8
    r = bench.roofline_object(_cfg2_counts(), ev, 655468512.0, "r01_traffic_cfg2.json", alg,
                              19_600_000, 4)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s"
    assert 0 < r["frac"] <= 1
    assert abs(r["achieved"] - 655468512.0 / 0.13711e-3 / 1e9) < 0.1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-4
    assert "PMC" in r["bytes_basis"]
    # the algorithmic figure exceeds the peak here: it is reported, but never as `frac`
    assert r["alg_ratio"]["alg_bytes_per_s_over_peak"] > 1
    assert r["compulsory_bytes_per_launch"] == int(_cfg2_counts().sum())
    json.dumps(r)


def test_roofline_falls_back_to_compulsory_bytes():
    ev = {"trav_med": 0.2, "n": 50}
    r = bench.roofline_object(_cfg2_counts(), ev, None, None, 1, 1, 4)
    assert r["traffic"] is None and "compulsory" in r["bytes_basis"]
    assert r["achieved"] == round(int(_cfg2_counts().sum()) / 0.2e-3 / 1e9, 1)


def test_roofline_protein_is_mfma_bound():
    ev = {"trav_med": 0.383, "n": 50}
    upd = 199 * 10_000 * 4
    r = bench.roofline_object(np.zeros(5, dtype=np.int64) + 10 ** 8, ev, 1.4e9, "x", 1, upd, 20)
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s"
    assert abs(r["achieved"] - upd * 1600 / 0.383e-3 / 1e12) < 0.01
    assert 0 < r["frac"] <= 1 and 0 < r["hbm_frac"] <= 1


def test_pmc_tags_key_strong_scaling_shards_by_size():
    """profiles/ files are keyed by config and per-rank sites: the N = 8 shard of the strong
    1M-site cfg4 run (125k sites) is the cfg4 shard itself, N = 1 is cfg4_s1000000."""
    assert bench.pmc_tag("cfg4", 125_000) == "cfg4"
    assert bench.pmc_tag("cfg4", 1_000_000) == "cfg4_s1000000"
    lo, hi = bench.strong_slice(1_000_000, 8, 0)
    assert bench.pmc_tag("cfg4", hi - lo) == "cfg4"
    lo, hi = bench.strong_slice(1_000_000, 2, 1)
    assert bench.pmc_tag("cfg4", hi - lo) == "cfg4_s500000"
    assert bench.pmc_tag("cfg5", 50_000, lnl_only=True) == "cfg5_lnl"
    assert bench.pmc_tag("cfg2", 100_000, override=True) is None


def test_rocprof_check_agrees_with_the_event_fraction():
    ev = {"trav_med": 0.1114, "n": 200}
    r = bench.roofline_object(_cfg2_counts(), ev, 655468512.0, "r03_traffic_cfg2.json", 1,
                              19_600_000, 4)
    c = bench.rocprof_check(r, (111360.0, 8061, "r03_cfg2_kernel_stats.csv"), 655468512.0,
                            19_600_000, 4)
    assert abs(c["frac"] - r["frac"]) < 0.002 and c["avg_ms"] == 0.11136
    # the committed cfg2 stats give the number the verdict recomputed (0.736)
    ks = bench.latest_kernel_stats("cfg2")
    if ks:
        assert 0.1 < ks[0] * 1e-6 < 0.2 and ks[1] > 100


def test_host_cpu_info_fields():
    h = bench.host_cpu_info()
    for k in ("model", "sockets", "cores_per_socket", "physical_cores", "affinity_cpus"):
        assert k in h
    assert h["affinity_cpus"] >= 1


def test_strong_scaling_slices_cover_one_alignment():
    """--total-sites: the ranks' slices partition [0, T) and, generated rank by rank, give the
    same alignment as one rank (total_sites unchanged for every N)."""
    from phylo_utils_amd import substitution_models as SM
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import random_tree
    model = SM.GTR([1.2, 3.5, 0.8, 1.1, 4.2, 1.0], [0.3, 0.2, 0.25, 0.25])
    rm = GammaRateModel(4, 0.5)
    tree = random_tree(np.random.default_rng(1234), 12)
    total, block = 1000, 300
    names1, whole = bench.strong_alignment(tree, model, rm.rates, total, 0, total, block)
    assert whole.shape == (12, total)
    for world in (2, 3, 8):
        sl = [bench.strong_slice(total, world, r) for r in range(world)]
        assert sl[0][0] == 0 and sl[-1][1] == total
        assert all(sl[r][1] == sl[r + 1][0] for r in range(world - 1))
        parts = []
        for lo, hi in sl:
            nm, c = bench.strong_alignment(tree, model, rm.rates, total, lo, hi, block)
            assert nm == names1
            parts.append(c)
        np.testing.assert_array_equal(np.concatenate(parts, axis=1), whole)


def test_strong_scaling_shards_sum_to_the_whole_lnl(oracle_mod):
    """The strong form's per-rank lnLs (each rank's slice of the one alignment) add up to the
    one-rank lnL (the RCCL sum of bin/phy.py:146's total): oracle on the CPU."""
    from phylo_utils_amd import substitution_models as SM
    from phylo_utils_amd.rate_models import GammaRateModel
    from phylo_utils_amd.synthetic import random_tree
    from phylo_utils_amd.tree import Traversal, prepare_tree
    model = SM.GTR([1.2, 3.5, 0.8, 1.1, 4.2, 1.0], [0.3, 0.2, 0.25, 0.25])
    rm = GammaRateModel(4, 0.5)
    tree = random_tree(np.random.default_rng(1234), 10)
    total = 700
    names, whole = bench.strong_alignment(tree, model, rm.rates, total, 0, total, 250)
    tr = Traversal(prepare_tree(tree))
    ev, el, iv = model.engine_eigen()

    def lnl(codes):
        tips = {tr.names[n]: np.eye(4)[codes[i]] for i, n in enumerate(names)}
        return oracle_mod.tree_lnl(tips, tr.postorder_traversal, tr.op_lengths(), tr.root_edge,
                                   tr.root_length(), ev, el, iv, model.freqs, rm.rates,
                                   rm.weights, n_nodes=tr.n_nodes)[0]
    ref = lnl(whole)
    for world in (2, 4):
        got = sum(lnl(bench.strong_alignment(tree, model, rm.rates, total,
                                             *bench.strong_slice(total, world, r), 250)[1])
                  for r in range(world))
        assert abs(got - ref) <= 1e-11 * abs(ref), (world, got, ref)


def test_roofline_lnl_only_is_issue_bound():
    ev = {"trav_med": 0.0905, "n": 50}
    upd = 99 * 50_000 * 4
    pmc = {"SQ_INSTS_VALU": 99 * 3128 * 70.0, "SQ_INSTS_SALU": 99 * 3128 * 65.0, "file": "x"}
    r = bench.roofline_object(np.zeros(5, dtype=np.int64) + 10 ** 6, ev, None, None, 1, upd, 4,
                              lnl_only=True, pmc=pmc)
    assert r["bound"] == "valu" and r["unit"] == "TFLOP/s"
    assert abs(r["achieved"] - upd * 71 / 0.0905e-3 / 1e12) < 0.01
    assert 0 < r["frac"] <= 1 and r["hbm_frac"] < 0.2
    assert r["issue"]["per_update"]["SQ_INSTS_SALU"] == round(99 * 3128 * 65.0 / upd, 4)
    json.dumps(r)


def test_sweep_neighbour_check_flags_a_dip():
    """scripts/sweep.py's guard: a size whose per-update rate is more
    than 5 % below the better of its neighbours is flagged; a smooth curve passes."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import sweep
    rows = [{"variant": "default", "taxa": 50, "sites": s, "mups": v}
            for s, v in [(50000, 170.0), (62500, 175.0), (75000, 157.0), (87500, 180.0)]]
    flags = sweep.neighbour_check(rows)
    assert [f["sites"] for f in flags] == [75000]
    assert abs(flags[0]["below"] - (1 - 157.0 / 180.0)) < 1e-3
    rows = [dict(r, mups=170.0 + i) for i, r in enumerate(rows)]
    assert sweep.neighbour_check(rows) == [{"variant": "default", "taxa": 50, "ok": True,
                                            "points": 4}]
