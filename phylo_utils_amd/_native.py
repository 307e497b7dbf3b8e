"""ctypes binding of libphylo_hip.so (C ABI declared in include/phylo_hip.h).

The shared object is built in-tree (``phylo_utils_amd/libphylo_hip.so``, see
``phylo_utils_amd/csrc/Makefile``).  There is no CPU fallback: if the library is
missing or a device call fails, the error is raised -- callers must never get
numbers that did not come from the HIP path.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(HERE, "libphylo_hip.so")
LIB_PATH = os.environ.get("PHYLO_HIP_LIB", _DEFAULT_LIB)

PU_KEEP_PARTIALS = 0x0
PU_LNL_ONLY = 0x1
PU_NO_REORDER = 0x2
# pu_ctx_set_stream: the context's own non-blocking stream (NULL is the HIP null stream)
PU_OWN_STREAM = ctypes.c_void_p(-1)

_c_int = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_dbl = ctypes.c_double
_P = ctypes.c_void_p

# name -> (restype, argtypes)
SIGNATURES = {
    "pu_version": (ctypes.c_char_p, []),
    "pu_last_error": (ctypes.c_char_p, [_P]),
    "pu_device_count": (_c_int, [_P]),
    "pu_clv": (_c_int, [_c_int, _c_int, _c_int, _c_i64, _P, _P, _P, _P, _P, _P, _P, _P]),
    "pu_lnl_node": (_c_int, [_c_int, _c_int, _c_int, _c_i64, _P, _P, _P, _P]),
    "pu_discrete_gamma": (_c_int, [_c_dbl, _c_int, _c_int, _P]),
    "pu_ctx_create": (_c_int, [_P, _c_int, _c_int, _c_int, _c_i64, _c_int, _c_int, _c_int]),
    "pu_ctx_destroy": (None, [_P]),
    "pu_set_tip_partials": (_c_int, [_P, _c_int, _P]),
    "pu_set_code_table": (_c_int, [_P, _c_int, _P]),
    "pu_set_tip_codes": (_c_int, [_P, _c_int, _P]),
    "pu_set_pattern_weights": (_c_int, [_P, _P]),
    "pu_set_model": (_c_int, [_P, _P, _P, _P, _P, _P, _P]),
    "pu_set_model_p": (_c_int, [_P, _P, _P, _P]),
    "pu_set_pmatrices": (_c_int, [_P, _P]),
    "pu_set_pmatrix_provider": (_c_int, [_P, _P, _P]),
    "pu_set_schedule": (_c_int, [_P, _c_int, _P, _P, _c_int, _c_int, _c_dbl]),
    "pu_set_branch_lengths": (_c_int, [_P, _P, _c_dbl]),
    "pu_run": (_c_int, [_P, _P, _P]),
    "pu_set_tips": (_c_int, [_P, _c_int, _P, _c_int, _P, _P, _P, _P]),
    "pu_set_tip_nodes": (_c_int, [_P, _c_int, _P]),
    "pu_share_tips": (_c_int, [_P, _P, _c_int, _P]),
    "pu_group_create": (_c_int, [_P, _c_int, _P, _c_int, _c_int, _c_i64, _c_int,
                                 _c_int, _c_int]),
    "pu_group_destroy": (None, [_P]),
    "pu_group_last_error": (ctypes.c_char_p, [_P]),
    "pu_group_size": (_c_int, [_P]),
    "pu_group_shard": (_c_int, [_P, _c_int, _P, _P]),
    "pu_group_ctx": (_P, [_P, _c_int]),
    "pu_group_set_tips": (_c_int, [_P, _c_int, _P, _c_int, _P, _P, _P, _P]),
    "pu_group_set_model": (_c_int, [_P, _P, _P, _P, _P, _P, _P]),
    "pu_group_set_schedule": (_c_int, [_P, _c_int, _P, _P, _c_int, _c_int, _c_dbl]),
    "pu_group_set_branch_lengths": (_c_int, [_P, _P, _c_dbl]),
    "pu_group_set_model_p": (_c_int, [_P, _P, _P, _P]),
    "pu_group_set_pmatrices": (_c_int, [_P, _P]),
    "pu_group_run": (_c_int, [_P, _P, _P]),
    "pu_enqueue": (_c_int, [_P]),
    "pu_synchronize": (_c_int, [_P, _P]),
    "pu_get_site_lnl": (_c_int, [_P, _P]),
    "pu_get_partials": (_c_int, [_P, _c_int, _P, _P]),
    "pu_get_root": (_c_int, [_P, _P, _P]),
    "pu_get_pmatrices": (_c_int, [_P, _P]),
    "pu_ctx_set_stream": (_c_int, [_P, _P]),
    "pu_set_lnl_device_output": (_c_int, [_P, _P]),
    "pu_plan_stats": (_c_int, [_c_int, _c_int, _P, _c_int, _c_int, _c_int, _c_int, _c_int, _P]),
    "pu_set_ascertainment": (_c_int, [_P, _c_int, _c_i64]),
    "pu_get_ascertainment_correction": (_c_int, [_P, _P]),
    "pu_edge_lnl": (_c_int, [_P, _c_int, _c_int, _P, _P]),
    "pu_edge_derivs": (_c_int, [_P, _c_int, _c_int, _c_dbl, _P]),
    "pu_update_partials": (_c_int, [_P, _c_int, _P, _P]),
    "pu_optimise_edge": (_c_int, [_P, _c_int, _c_int, _c_dbl, _c_int, _P, _P]),
    "pu_minimise_edge": (_c_int, [_P, _c_int, _c_int, _c_int, _c_dbl, _c_dbl, _c_dbl, _c_dbl,
                                  _P]),
    "pu_optimise_sweep": (_c_int, [_P, _c_int, _P, _c_dbl, _c_int, _P, _P]),
    "pu_get_branch_lengths": (_c_int, [_P, _P, _P]),
    "pu_lnl_branch": (_c_int, [_c_int, _c_int, _c_i64, _c_int, _P, _P, _P, _P, _P, _P, _P, _P]),
    "pu_lnl_branch_derivs": (_c_int, [_c_int, _c_int, _c_i64, _c_int, _P, _P, _P, _P, _P, _P,
                                      _P, _P]),
    "pu_compress_patterns": (_c_int, [_c_int, _P, _c_int, _c_i64, _c_int, _P, _P, _P, _P]),
    "pu_compress_patterns_device": (_c_int, [_c_int, _P, _P, _c_int, _c_i64, _c_int, _P,
                                             _c_i64, _P, _P, _P]),
    "pu_ctx_stream": (_P, [_P]),
    "pu_ctx_device_bytes": (_c_i64, [_P]),
    "pu_write_ceiling": (_c_int, [_c_int, _c_i64, _c_int, _P]),
    "pu_ctx_newton_stats": (_c_int, [_P, _P, _P]),
    "pu_ctx_profile": (_c_int, [_P, _c_int]),
    "pu_ctx_kernel_ms": (_c_int, [_P, _P, _P, _P]),
    "pu_ctx_kernel_times": (_c_int, [_P, _P, _P, _c_int, _P]),
    "pu_ctx_traffic": (_c_int, [_P, _P]),
    "pu_ctx_plan_info": (_c_int, [_P, _P]),
    "pu_ctx_edge_kernel_ms": (_c_int, [_P, _P, _P]),
    "pu_ctx_edge_kernel_ms2": (_c_int, [_P, _P, _P, _P]),
    "pu_batch_create": (_c_int, [_P, _c_int, _P]),
    "pu_batch_destroy": (None, [_P]),
    "pu_batch_last_error": (ctypes.c_char_p, [_P]),
    "pu_batch_set_stream": (_c_int, [_P, _P]),
    "pu_batch_enqueue": (_c_int, [_P, _P]),
    "pu_batch_synchronize": (_c_int, [_P]),
    "pu_batch_profile": (_c_int, [_P, _c_int]),
    "pu_batch_kernel_times": (_c_int, [_P, _P, _P, _c_int, _P]),
}

_lib = None
_lock = threading.Lock()


class PhyloHipError(RuntimeError):
    """A libphylo_hip call returned a negative status (message = pu_last_error)."""


def _preload_hip_runtime():
    """One HIP runtime per process, whichever of torch and this library the caller loads
    first.

    libphylo_hip.so is built with ROCm 7.2 and needs libamdhip64.so.7 /
    libhsa-runtime64.so.1 / librccl.so.1; PyTorch ships its own runtime under the same
    sonames (ROCm 7.0).  The dynamic linker binds a soname to the first library loaded under
    it, so loading this library first used to put the system runtime in the process and torch
    then saw no GPU.  When torch is installed it is imported here, before this library, so
    the process always runs torch's runtime -- the order bench.py and the GPU tests use.
    (Preloading torch's runtime files without importing torch worked until process exit,
    where torch's later initialisation freed runtime state twice.)  PU_HIP_RUNTIME=system
    keeps the system runtime.  Returns torch's library directory, or None."""
    if os.environ.get("PU_HIP_RUNTIME") == "system":
        return None
    try:
        import torch
    except ImportError:
        return None
    return os.path.join(os.path.dirname(torch.__file__), "lib")


def lib():
    """Load libphylo_hip.so once; raise if it is absent (no fallback path exists)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(
                        "libphylo_hip.so not found at %s -- build it with "
                        "`python -c 'import __graft_entry__ as g; g.build()'` or "
                        "`make -C phylo_utils_amd/csrc`" % LIB_PATH)
                _preload_hip_runtime()
                so = ctypes.CDLL(LIB_PATH)
                for name, (res, args) in SIGNATURES.items():
                    # an A/B build from an older round may lack a newer diagnostic entry
                    # point (PHYLO_HIP_LIB); calling it then raises AttributeError
                    fn = getattr(so, name, None)
                    if fn is None and LIB_PATH != _DEFAULT_LIB:
                        continue
                    fn = getattr(so, name)
                    fn.restype = res
                    fn.argtypes = args
                _lib = so
    return _lib


# return codes (include/phylo_hip.h)
PU_OK, PU_E_ARG, PU_E_HIP, PU_E_STATE, PU_E_SCHED, PU_E_NOMEM, PU_E_COMM = 0, -1, -2, -3, -4, -5, -6


def last_error(ctx=None):
    msg = lib().pu_last_error(ctx)
    return msg.decode() if msg else ""


def check(rc, ctx=None, what=""):
    if rc != 0:
        raise PhyloHipError("%s failed (%d): %s" % (what or "libphylo_hip call", rc,
                                                     last_error(ctx)))


def ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


# int (*)(void *user, int order, int n, const double *t, double *out)
PMAT_PROVIDER = ctypes.CFUNCTYPE(_c_int, _P, _c_int, _c_int, ctypes.POINTER(_c_dbl),
                                 ctypes.POINTER(_c_dbl))


def device_count():
    n = ctypes.c_int(0)
    check(lib().pu_device_count(ctypes.byref(n)))
    return n.value


def plan_stats(n_nodes, ops, root_edge, R, L, flags=0):
    """Host-only planner statistics (pu_plan_stats): dict of children per source; R is the
    split target (PU_SPLIT, 0: one task)."""
    ops = np.ascontiguousarray(ops, dtype=np.int32)
    st = np.zeros(8, dtype=np.int32)
    check(lib().pu_plan_stats(n_nodes, len(ops), ptr(ops), int(root_edge[0]),
                              int(root_edge[1]), R, L, flags, ptr(st)), what="pu_plan_stats")
    return dict(mem=int(st[0]), chains=int(st[1]), lds=int(st[2]), tip=int(st[3]),
                store=int(st[4]), max_live=int(st[5]), cur=int(st[6]), top=int(st[7]))


def ctx_plan(ctx):
    """The traversal plan of a context's schedule (pu_ctx_plan_info): launch grid, k_prune
    build, variant bits, LDS stash slots, chunks, LDS pad, tiles, blocks, the extra tiles per
    row (PU_PITCH_EXTRA) and the row pitch."""
    out = np.zeros(10, dtype=np.int32)
    check(lib().pu_ctx_plan_info(ctx, ptr(out)), ctx, "pu_ctx_plan_info")
    return dict(grid=int(out[0]), waves=int(out[1]), variant=int(out[2]), lds=int(out[3]),
                chunks=int(out[4]), pad=int(out[5]), tiles=int(out[6]), blocks=int(out[7]),
                pitch_extra=int(out[8]), pitch=int(out[9]))
