"""r06 debug: one cfg2-size device Newton with per-evaluation stamps (PU_NT_TIMING=1 prints
them from the library), and the host loop for comparison."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from phylo_utils_amd import TreeModel  # noqa: E402
from phylo_utils_amd import substitution_models as SM  # noqa: E402
from phylo_utils_amd.rate_models import GammaRateModel  # noqa: E402
from phylo_utils_amd.synthetic import CFG2_FREQS, CFG2_GTR_RATES, make_problem  # noqa: E402

m = SM.GTR(CFG2_GTR_RATES, CFG2_FREQS)
rm = GammaRateModel(4, 0.5)
tree, names, st = make_problem(50, int(os.environ.get("SITES", "100000")), m, rm.rates, seed=3)
tm = TreeModel(device=0)
tm.set_alignment_codes(st.astype(np.uint8), np.eye(4), names)
tm.set_substitution_model(m)
tm.set_rate_model(rm)
tm.set_tree(tree)
tm.initialise()
a, b = tm.traversal.root_edge
key = tuple(sorted((a, b)))
t0 = tm.traversal.brlens[key]
import ctypes  # noqa: E402
from phylo_utils_amd import _native as N  # noqa: E402
lib = N.lib()
for mode in ("1", "0", "1", "plain"):
    os.environ["PU_NT_PLAIN"] = "1" if mode == "plain" else "0"
    if mode == "plain":
        mode = "1"
    os.environ["PU_EDGE_DEVICE_NEWTON"] = mode
    ts = []
    for k in range(5):
        tm.traversal.brlens[key] = t0 * (0.5 + 0.25 * k)
        tm.update_branch_lengths()
        tm.likelihood()
        os.environ["PU_NT_TIMING"] = "1" if (mode == "1" and k == 2) else "0"
        c = time.perf_counter()
        t, lnl = tm.optimise_edge(a, b)
        ts.append(time.perf_counter() - c)
    raw = []
    for k in range(5):  # the C call alone, back to back (no traversal between)
        out_t, out_l = ctypes.c_double(), ctypes.c_double()
        c = time.perf_counter()
        N.check(lib.pu_optimise_edge(tm._ctx, a, b, 1e-8, 50, ctypes.byref(out_t), ctypes.byref(out_l)), tm._ctx)
        raw.append(time.perf_counter() - c)
    print("  raw pu_optimise_edge back to back us:", [round(x * 1e6, 1) for x in raw], flush=True)
    print("device" if mode == "1" else "host", "optimise_edge us:", [round(x * 1e6, 1) for x in ts],
          flush=True)
