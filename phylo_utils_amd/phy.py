"""``phy`` -- lnL of an alignment on a tree (counterpart of the reference's ``bin/phy.py``,
SURVEY 8(f) N2).

    python -m phylo_utils_amd.phy -t tree.nwk -s aln.fasta -m 'GTR{1.0,2.0,1.0,1.0,2.0,1.0}+G4{0.5}'

Same options and output as ``bin/phy.py:13-19, 146`` (``lnL = <value>``).  The model
string grammar is ``bin/phy.py:41-56``: a model name, optional ``{parameters}``, then up to
two of ``+F{freqs}`` and ``+G<ncat>{alpha}``.  Differences, all deliberate:

* the reference passes every model ``(rates=..., freqs=...)`` (``:128``), which only
  ``GTR`` accepts -- the others raise TypeError; here each model gets its parameters in
  its own constructor's order (K80/HKY85/F84: kappa; TN93: alpha_y, alpha_r[, beta]);
* ``JC``/``JC69`` runs (the reference's ``JC69.p`` has no ``rates`` argument and cannot go
  through TreeModel);
* parameters may be written as integers (``{2}``) as well as ``{2.0}``, and model names
  may contain digits (the reference's ``Word(alphas)`` reads ``HKY85{2.0}`` as ``HKY`` and
  drops the rest of the string);
* Newick and FASTA are read without dendropy / Biopython (``tree.parse_newick``,
  ``alignment.read_fasta``).
Extensions: ``--optimise`` runs branch-length optimisation passes on the GPU first
(``--optimiser newton|brent|dbrent``)
(SURVEY 8(f) N1); ``--ascertainment`` applies the Lewis correction (N3); ``--device``.
"""
from __future__ import annotations

import argparse
import os
import re
import sys

from . import alignment as A
from . import rate_models as RM
from . import substitution_models as SM
from .tree import parse_newick
from .tree_model import TreeModel

PROTEIN_MODELS = ("JTT", "Dayhoff", "WAG", "LG")
_PART = re.compile(r"\+(F|G(\d+))(\{[^}]*\})?")
_HEAD = re.compile(r"([A-Za-z][A-Za-z0-9]*)(\{[^}]*\})?")


def _reals(braces):
    if braces is None:
        return None
    body = braces[1:-1].strip()
    if not body:
        raise ValueError("empty parameter list {}")
    return [float(x) for x in body.split(",")]


def parse_model_string(text):
    """bin/phy.py:41-56 -> dict(subs_model, model_params, freq_params, rate_model,
    rate_cats, rate_param); absent parts are None."""
    text = text.strip().replace(" ", "")
    m = _HEAD.match(text)
    if not m:
        raise ValueError("model string %r does not start with a model name" % text)
    out = dict(subs_model=m.group(1), model_params=_reals(m.group(2)), freq_params=None,
               rate_model=None, rate_cats=None, rate_param=None)
    rest, n = text[m.end():], 0
    while rest:
        p = _PART.match(rest)
        if not p or n == 2:
            raise ValueError("cannot parse %r in model string %r" % (rest, text))
        if p.group(1) == "F":
            out["freq_params"] = _reals(p.group(3))
        else:
            out["rate_model"] = "G"
            out["rate_cats"] = int(p.group(2))
            vals = _reals(p.group(3))
            out["rate_param"] = vals
        rest, n = rest[p.end():], n + 1
    return out


def _one(vals):
    """bin/phy.py:83-91 unpack: a single value is a scalar."""
    if vals is None:
        return None
    return vals[0] if len(vals) == 1 else vals


def build_model(desc):
    """Substitution model from a parsed model string (bin/phy.py:59-80, 119-128)."""
    name, p, f = desc["subs_model"], desc["model_params"], desc["freq_params"]
    freqs = None if f is None else list(f)
    try:
        if name == "GTR":
            return SM.GTR(rates=p, freqs=freqs)
        if name in ("JC", "JC69"):
            return SM.JC69()
        if name == "K80":
            return SM.K80(*(p or [2.0]))
        if name in ("HKY", "HKY85"):
            return SM.HKY85((p or [2.0])[0], freqs if freqs else [0.25] * 4)
        if name == "F81":
            return SM.F81(freqs if freqs else [0.25] * 4)
        if name == "F84":
            return SM.F84((p or [2.0])[0], freqs if freqs else [0.25] * 4)
        if name == "TN93":
            q = list(p or [2.0, 2.0])
            return SM.TN93(*q, freqs=freqs if freqs else [0.25] * 4)
        if name in PROTEIN_MODELS:
            return getattr(SM, name)(freqs=freqs)
    except TypeError as e:
        raise ValueError("bad parameters for model %s: %s" % (name, e))
    raise ValueError("Unrecognised model %s; valid options are GTR, HKY, HKY85, K80, F81, F84, "
                     "JC, JC69, TN93, LG, WAG, JTT, Dayhoff" % name)


def build_rate_model(desc):
    """bin/phy.py:130-138: +G<ncat>{alpha} -> Gamma (defaults 4, 0.5), else uniform."""
    if desc["rate_model"] == "G":
        ncat = desc["rate_cats"] if desc["rate_cats"] is not None else 4
        alpha = _one(desc["rate_param"])
        return RM.GammaRateModel(ncat, alpha if alpha is not None else 0.5)
    return RM.UniformRateModel()


def parse_cli(argv=None):
    ap = argparse.ArgumentParser("phy - calculate likelihood of an alignment given a "
                                 "phylogenetic model")
    ap.add_argument("-t", "--tree", type=str, help="File path to a tree in newick format")
    ap.add_argument("-s", "--alignment", type=str, help="File path to an alignment in fasta "
                    "format")
    ap.add_argument("-m", "--model", type=str, default="JC", help="Model specification string")
    ap.add_argument("--device", type=int, default=0, help="HIP device")
    ap.add_argument("--optimise", type=int, default=0, metavar="PASSES",
                    help="optimise branch lengths first (passes of the optimising traversal)")
    ap.add_argument("--optimiser", default="newton", choices=["newton", "brent", "dbrent"],
                    help="per-edge method of --optimise (brent / dbrent: the reference's "
                         "src/optimisation.pyx minimisers)")
    ap.add_argument("--ascertainment", choices=["reference", "weighted"], default=None,
                    help="Lewis ascertainment-bias correction")
    return ap.parse_args(argv)


def validate_args(args):
    """bin/phy.py:22-30."""
    if args.tree is None:
        raise ValueError("Tree file not specified")
    if args.alignment is None:
        raise ValueError("Alignment file not specified")
    if not os.path.exists(args.tree):
        raise FileNotFoundError("Tree file {} does not exist".format(args.tree))
    if not os.path.exists(args.alignment):
        raise FileNotFoundError("Alignment file {} does not exist".format(args.alignment))


def run(args, out=None):
    out = sys.stdout if out is None else out
    with open(args.tree) as fh:
        tree = parse_newick(fh.read())
    aln = A.read_fasta(args.alignment)
    desc = parse_model_string(args.model)
    alphabet = A.PROTEIN if desc["subs_model"] in PROTEIN_MODELS else A.DNA
    tm = TreeModel(device=args.device)
    tm.set_tree(tree)
    tm.set_alignment(aln, alphabet)
    tm.set_rate_model(build_rate_model(desc))
    tm.set_substitution_model(build_model(desc))
    if args.ascertainment:
        tm.set_ascertainment_bias_correction(weighted=args.ascertainment == "weighted")
    tm.initialise()
    if args.optimise:
        tm.optimise_branch_lengths(sweeps=args.optimise, method=args.optimiser)
    lnl = tm.compute_likelihood_at_edge(*tm.traversal.root_edge).sum()
    out.write("lnL = {}\n".format(lnl))
    return lnl


def main(argv=None):
    args = parse_cli(argv)
    try:
        validate_args(args)
    except (ValueError, FileNotFoundError) as e:
        sys.stderr.write("ERROR: {}\n".format(e))
        return 1
    try:
        run(args)
    except ValueError as e:
        sys.stderr.write("ERROR: {}\n".format(e))
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
