"""How long the host takes to enqueue one cfg5 step (125 trees x pu_enqueue) against the step's
wall time: if the two are close, the step is host-bound."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import CONFIGS, make_model  # noqa: E402
from phylo_utils_amd import TreeModel  # noqa: E402
from phylo_utils_amd import _native as N  # noqa: E402
from phylo_utils_amd.rate_models import GammaRateModel  # noqa: E402
from phylo_utils_amd.synthetic import random_tree, simulate_states  # noqa: E402

cfg = CONFIGS["cfg5"]
model = make_model(cfg)
rm = GammaRateModel(4, 0.5)
S, ntax, T = cfg["sites"], cfg["ntax"], cfg["trees"]
tt = random_tree(np.random.default_rng(1234), ntax)
st = simulate_states(np.random.default_rng(999), tt, model, rm.rates, S)
names = sorted(st, key=lambda s: int(s[1:]))
codes = np.stack([st[n] for n in names]).astype(np.uint8)
dev = torch.device("cuda", 0)
streams = [torch.cuda.Stream(dev) for _ in range(4)]
lnl = torch.zeros(T, dtype=torch.float64, device=dev)
tms = []
for i in range(T):
    tm = TreeModel(keep_partials=False)
    tm.set_alignment_codes(codes, np.eye(4), names)
    tm.set_substitution_model(model)
    tm.set_rate_model(rm)
    tm.set_tree(random_tree(np.random.default_rng(10_000 + i), ntax))
    tm.initialise()
    N.check(N.lib().pu_ctx_set_stream(tm._ctx, ctypes.c_void_p(streams[i % 4].cuda_stream)))
    N.check(N.lib().pu_set_lnl_device_output(tm._ctx, ctypes.c_void_p(lnl.data_ptr() + 8 * i)))
    tms.append(tm)
lib = N.lib()
for rep in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for tm in tms:
        lib.pu_enqueue(tm._ctx)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("enqueue %.2f ms  step %.2f ms" % ((t1 - t0) * 1e3, (t2 - t0) * 1e3), flush=True)
