#!/usr/bin/env python
"""HBM calibration on one GPU: achievable write-only, read-only and copy bandwidth.

    python scripts/hbm_calib.py [--mb 800]

The traversal kernel in KEEP mode is a write stream (every internal CLV is stored
once); this measures what a plain store stream reaches on the same card so the
roofline fraction can be read against both the datasheet peak and the practical one.
"""
import argparse
import json

import torch


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=800)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    n = a.mb * (1 << 20) // 8
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    x.fill_(1.0)
    nbytes = n * 8
    out = {}
    ms = timed(lambda: x.fill_(2.0), a.reps)
    out["write_GBps"] = nbytes / ms / 1e6
    ms = timed(lambda: y.copy_(x), a.reps)
    out["copy_GBps"] = 2 * nbytes / ms / 1e6
    ms = timed(lambda: x.sum(), a.reps)
    out["read_GBps"] = nbytes / ms / 1e6
    out["mb"] = a.mb
    print(json.dumps(out))


if __name__ == "__main__":
    main()
