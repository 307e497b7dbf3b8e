"""Golden fixtures for the 1-D optimisers from the REFERENCE's own compiled module.

    make -C oracle ref_optim              # cythonizes /root/reference/src/optimisation.pyx
    python tests/golden/make_golden_optim.py   # -> tests/golden/optimisation.npz

oracle/_ref/optimisation*.so is the reference's src/optimisation.pyx, compiled where it lies
(generated C and the module go to oracle/_ref/ only).  For every case of tests/optim_cases.py
it records the out triple of brent_wrap / dbrent_wrap and every abscissa fn / dfn were
called at, plus simplex_encode/decode, transform_params/decode_params and quad_interp.
"""
import importlib.util
import glob
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import optim_cases as oc  # noqa: E402


def load_ref():
    so = glob.glob(os.path.join(ROOT, "oracle", "_ref", "optimisation*.so"))
    if not so:
        raise SystemExit("build the reference module first: make -C oracle ref_optim")
    spec = importlib.util.spec_from_file_location("optimisation", so[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ref = load_ref()
    out = {}
    for i, (name, guess, lb, rb, tol) in enumerate(oc.CASES):
        f, df = oc.FUNCS[name]
        g, xs = oc.traced(f)
        out["brent_%d_out" % i] = ref.brent_wrap(guess, lb, rb, g, tol)
        out["brent_%d_fx" % i] = np.array(xs)
        g, xs = oc.traced(f)
        dg, dxs = oc.traced(df)
        out["dbrent_%d_out" % i] = ref.dbrent_wrap(guess, lb, rb, g, dg, tol)
        out["dbrent_%d_fx" % i] = np.array(xs)
        out["dbrent_%d_dfx" % i] = np.array(dxs)
    for i, p in enumerate(oc.SIMPLEX):
        th = ref.simplex_encode(np.ascontiguousarray(p))
        out["simplex_%d_p" % i] = p
        out["simplex_%d_theta" % i] = th
        out["simplex_%d_back" % i] = ref.simplex_decode(np.ascontiguousarray(th))
        q = ref.transform_params(np.ascontiguousarray(p))
        out["simplex_%d_q" % i] = q
        out["simplex_%d_decoded" % i] = ref.decode_params(q)
    out["quad"] = np.array([ref.quad_interp(*a) for a in oc.QUAD])
    np.savez(os.path.join(HERE, "optimisation.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
