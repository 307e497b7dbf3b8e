"""The C ABI library (no device compute on the CPU container): it loads, exports
every symbol include/phylo_hip.h declares, and fails loudly without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, has_gpu

from phylo_utils_amd import _native as N

HEADER = os.path.join(ROOT, "include", "phylo_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pu_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = N.lib()
    syms = declared_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    assert set(declared_symbols()) == set(N.SIGNATURES)


def test_library_is_gfx950_code_object():
    data = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_errors():
    assert b"gfx950" in N.lib().pu_version()
    out = ctypes.c_void_p()
    rc = N.lib().pu_ctx_create(ctypes.byref(out), 0, 4, 3, 0, 4, 4, 0)  # S = 0
    assert rc == -1 and out.value is None
    assert "bad sizes" in N.last_error()
    rc = N.lib().pu_ctx_create(ctypes.byref(out), 0, 10, 6, 100, 4, 7, 0)  # K = 7
    assert rc == -1 and "not supported" in N.last_error()


@pytest.mark.skipif(has_gpu(), reason="checks the no-device error path")
def test_no_device_fails_loudly():
    from phylo_utils_amd.likelihood import hip_likelihood_engine as E
    p = np.stack([np.eye(4)])
    a = np.ones((2, 1, 4))
    s = np.zeros((2, 1))
    with pytest.raises(N.PhyloHipError):
        E.clv(p, p, a, a, s, s, np.zeros((2, 1)))
    out = ctypes.c_void_p()
    assert N.lib().pu_ctx_create(ctypes.byref(out), 0, 4, 3, 10, 4, 4, 0) != 0


def test_engine_shape_validation():
    from phylo_utils_amd.likelihood import hip_likelihood_engine as E
    p = np.stack([np.eye(4)] * 2)
    with pytest.raises(ValueError):
        E.clv(p, p, np.ones((3, 2, 5)), np.ones((3, 2, 5)), np.zeros((3, 2)), np.zeros((3, 2)),
              np.zeros((3, 2)))
    with pytest.raises(TypeError):
        E.clv(p.astype(np.float32), p, np.ones((3, 2, 4)), np.ones((3, 2, 4)),
              np.zeros((3, 2)), np.zeros((3, 2)), np.zeros((3, 2)))


def _random_ops(rng, n_tips):
    """Random rooted binary tree as a caller schedule: (ops [n-2][3], root edge, n_nodes)."""
    nodes = list(range(n_tips))
    nxt = n_tips
    ops = []
    while len(nodes) > 2:
        i, j = sorted(rng.choice(len(nodes), 2, replace=False))
        a, b = nodes[i], nodes[j]
        nodes = [x for k, x in enumerate(nodes) if k not in (i, j)] + [nxt]
        ops.append((nxt, a, b))
        nxt += 1
    return np.array(ops, dtype=np.int32), (nodes[0], nodes[1]), nxt


@pytest.mark.parametrize("n_tips", [3, 4, 17, 50, 300])
def test_planner_child_sources(n_tips):
    """Host-only planner (pu_plan_stats, no device): every child is a tip, the previous
    op's parent, an LDS-stash parent or an HBM read-back; a DFS order with a stash as deep
    as the peak number of waiting parents needs no HBM read-back, and no stash means every
    waiting parent is read back."""
    rng = np.random.default_rng(n_tips)
    ops, root, n_nodes = _random_ops(rng, n_tips)
    n_children = 2 * (len(ops) + 1)
    base = N.plan_stats(n_nodes, ops, root, 0, 0)
    depth = base["max_live"]
    for L in (0, 1, 2, max(depth, 1)):
        st = N.plan_stats(n_nodes, ops, root, 0, L)
        assert st["mem"] + st["lds"] + st["tip"] + st["cur"] == n_children
        assert st["tip"] == n_tips
        assert st["max_live"] == depth
        if L == 0:
            assert st["lds"] == 0
        if L >= depth:
            assert st["mem"] == 0
    # LNL_ONLY stores only parents read back from HBM
    st = N.plan_stats(n_nodes, ops, root, 0, 0, N.PU_LNL_ONLY)
    assert st["store"] <= max(depth, 1)
    st = N.plan_stats(n_nodes, ops, root, 0, 8, N.PU_LNL_ONLY)
    assert st["store"] == (0 if depth <= 8 else st["store"])


@pytest.mark.parametrize("n_tips", [4, 17, 50, 200, 1000])
@pytest.mark.parametrize("split", [2, 3, 4])
def test_planner_split_into_chain_tasks(n_tips, split):
    """A split plan (PU_SPLIT, protein KEEP traversals): disjoint subtrees become chain tasks
    and the ops above them the top task.  Every child still has exactly one source, every chain
    root is read back from HBM by the top task, the top stays within n_ops / 16, split <= 1
    is never split, and an lnL-only plan splits the same way."""
    rng = np.random.default_rng(1000 + n_tips)
    ops, root, n_nodes = _random_ops(rng, n_tips)
    n_ops = len(ops)
    n_children = 2 * (n_ops + 1)
    st = N.plan_stats(n_nodes, ops, root, split, 3)
    assert st["mem"] + st["lds"] + st["tip"] + st["cur"] == n_children
    assert st["tip"] == n_tips
    if n_ops > 2 and n_tips >= 17:
        assert st["chains"] >= 2
    if st["chains"]:
        assert st["top"] <= max(1, n_ops // 16)
        assert st["mem"] >= st["chains"]
        assert st["chains"] <= 32
    assert N.plan_stats(n_nodes, ops, root, 1, 3)["chains"] == 0
    # lnL-only: the same tasks; each task colours its HBM slots apart (chains run at once)
    lo = N.plan_stats(n_nodes, ops, root, split, 3, N.PU_LNL_ONLY)
    assert lo["chains"] == st["chains"] and lo["top"] == st["top"]
    assert lo["mem"] == st["mem"]
    if lo["chains"]:
        assert lo["store"] >= lo["chains"]  # at least every chain root has a slot


def test_planner_rejects_bad_schedules():
    ops = np.array([[3, 0, 1]], dtype=np.int32)
    with pytest.raises(N.PhyloHipError):
        N.plan_stats(5, np.array([[3, 0, 0]], dtype=np.int32), (3, 2), 0, 2)  # repeated child
    with pytest.raises(N.PhyloHipError):
        N.plan_stats(5, np.array([[3, 0, 1], [3, 2, 4]], dtype=np.int32), (3, 2), 0, 2)
    st = N.plan_stats(4, ops, (3, 2), 0, 2)
    assert st["tip"] == 3 and st["cur"] == 1


@pytest.mark.skipif(has_gpu(), reason="checks the no-device error path")
def test_group_without_device_fails_loudly():
    g = ctypes.c_void_p()
    rc = N.lib().pu_group_create(ctypes.byref(g), 1, None, 6, 4, 100, 4, 4, 0)
    assert rc != 0
    assert N.lib().pu_group_last_error(g)
    N.lib().pu_group_destroy(g)
    # bad arguments are rejected before any device is touched
    assert N.lib().pu_group_create(ctypes.byref(g), 0, None, 6, 4, 100, 4, 4, 0) != 0


def test_shipped_library_has_no_result_altering_switches():
    """the timing-experiment switches that made results invalid
    (PU_STORE_MODE bits 4-5: every op on side 0's P, no parent stores) and the experiment
    kernels (PU_EXP_ALL4X4, PU_AA_PREFETCH) are gone from the default library: it never reads
    PU_STORE_MODE, and it loads and reports its symbols with the variable set."""
    data = open(N.LIB_PATH, "rb").read()
    assert b"PU_STORE_MODE" not in data
    import subprocess
    import sys
    env = dict(os.environ, PU_STORE_MODE="48", PU_HIP_RUNTIME="system")
    r = subprocess.run([sys.executable, "-c", "from phylo_utils_amd import _native as N; "
                        "print(N.lib().pu_version().decode())"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "phylo_hip" in r.stdout, r.stderr
    src = open(os.path.join(ROOT, "phylo_utils_amd", "csrc", "pu_kernels.hip")).read()
    for flag in ("PU_EXP_ALL4X4", "PU_AA_PREFETCH", "store_mode"):
        assert flag not in src, flag
