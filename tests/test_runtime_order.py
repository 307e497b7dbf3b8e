"""One HIP runtime per process whichever of torch and libphylo_hip loads first
(_native._preload_hip_runtime).  The GPU case runs in fresh subprocesses:
the library initialises HIP before torch is imported, then torch must still see the device
and both must work on the same stream."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

LIB_FIRST = r"""
import ctypes, numpy as np
from phylo_utils_amd import _native as N
assert N.device_count() >= 1                      # libphylo_hip initialises HIP first
import torch
assert torch.cuda.is_available(), "torch sees no GPU after libphylo_hip"
x = torch.arange(8, dtype=torch.float64, device="cuda").sum().item()
assert x == 28.0
from phylo_utils_amd.likelihood import hip_likelihood_engine as E
pi = np.full(4, 0.25); part = np.random.default_rng(0).random((5, 2, 4)); sc = np.zeros((5, 2))
np.testing.assert_allclose(E.lnl_node(pi, part, sc), np.log(part @ pi), rtol=1e-14)
print("ok", N.lib()._name)
"""


def test_preload_finds_torch_runtime():
    from phylo_utils_amd import _native as N
    d = N._preload_hip_runtime()
    assert d is None or os.path.exists(os.path.join(d, "libamdhip64.so"))


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["lib_first", "torch_first"])
def test_library_and_torch_share_one_runtime(order):
    code = LIB_FIRST if order == "lib_first" else "import torch\n" + LIB_FIRST
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=180, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert "ok" in r.stdout
