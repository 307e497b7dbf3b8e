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
