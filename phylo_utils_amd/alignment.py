"""Alignment ingest: character -> partial vectors, pattern compression, FASTA.

Mirrors ``phylo_utils/alignment/`` (``alignment.py:26-66``, ``charmaps.py``,
``alphabets.py``) without Biopython:

* ``DNA``, ``PROTEIN``, ``BINARY`` alphabet constants (``alphabets.py:1-3``);
  ``seq_to_partials`` also accepts the names ``"dna"``/``"protein"``/``"binary"``.
* charmaps: IUPAC nucleotide ambiguity (gap, N = all states), the 20 amino
  acids plus ``- ? X`` (all states), binary ``0 1 - N``; upper and lower case.
* ``alignment_to_numpy`` compresses identical columns with
  ``np.unique(axis=1, return_inverse, return_counts)`` exactly as the reference
  (patterns come out in lexicographic order).
* ``alignment_to_codes`` is the engine's compact form: every distinct tip
  vector gets a uint8 code (``pu_set_code_table`` / ``pu_set_tip_codes``).
"""
from __future__ import annotations

from functools import reduce

import numpy as np

from .data import DNA_STATES, PROTEIN_STATES

DNA = 0
PROTEIN = 1
BINARY = 2

_NAMES = {"dna": DNA, "nt": DNA, "nucleotide": DNA, "protein": PROTEIN, "aa": PROTEIN,
          "binary": BINARY}

_IUPAC = {
    "A": "A", "C": "C", "G": "G", "T": "T", "U": "T",
    "R": "AG", "Y": "CT", "M": "AC", "K": "GT", "W": "AT", "S": "CG",
    "B": "CGT", "D": "AGT", "H": "ACT", "V": "ACG", "N": "ACGT", "-": "ACGT",
}


def _build_charmap(states, codes, extra_all, case=True):
    cmap = {}
    for ch, members in codes.items():
        v = [1.0 if s in members else 0.0 for s in states]
        cmap[ch] = v
        if case and ch.isalpha():
            cmap[ch.lower()] = list(v)
    for ch in extra_all:
        cmap[ch] = [1.0] * len(states)
    return cmap


dna_charmap = _build_charmap(DNA_STATES, _IUPAC, [])
protein_charmap = _build_charmap(PROTEIN_STATES, {s: s for s in PROTEIN_STATES},
                                 ["-", "?", "X", "x"])
binary_charmap = {"-": [1.0, 1.0], "N": [1.0, 1.0], "0": [1.0, 0.0], "1": [0.0, 1.0]}

CHARMAPS = {DNA: dna_charmap, PROTEIN: protein_charmap, BINARY: binary_charmap}
NSTATES = {DNA: 4, PROTEIN: 20, BINARY: 2}


def alphabet_code(alphabet):
    if isinstance(alphabet, str):
        try:
            return _NAMES[alphabet.lower()]
        except KeyError:
            raise ValueError("unknown alphabet %r" % alphabet)
    return int(alphabet)


def seq_to_partials(seq, alphabet):
    """[len(seq)][K] 0/1 partial vectors for one sequence (alignment.py:26-37)."""
    cmap = CHARMAPS.get(alphabet_code(alphabet))
    if cmap is None:
        raise ValueError("unknown alphabet %r" % alphabet)
    try:
        return np.ascontiguousarray([cmap[ch] for ch in seq], dtype=np.float64)
    except KeyError as e:
        raise ValueError("character %s is not in the alphabet" % e)


def _records(alignment):
    """Accept [(name, seq)], {name: seq}, or objects with .name/.seq (Biopython records)."""
    if isinstance(alignment, dict):
        return list(alignment.items())
    out = []
    for rec in alignment:
        if isinstance(rec, (tuple, list)):
            out.append((rec[0], str(rec[1])))
        else:
            out.append((rec.name, str(rec.seq)))
    return out


def alignment_to_numpy(alignment, alphabet, compress=True):
    """(partials [ntaxa][S][K], siteweights [S], inverse_index [S_orig], names {name: row})
    -- alignment.py:40-57."""
    recs = _records(alignment)
    aln = np.stack([seq_to_partials(s, alphabet) for _, s in recs])
    names = {n: i for i, (n, _) in enumerate(recs)}
    n_sites = aln.shape[1]
    if compress:
        aln, inverse, weights = np.unique(aln, return_inverse=True, return_counts=True, axis=1)
        inverse = np.asarray(inverse).reshape(-1)
    else:
        weights = np.ones(n_sites, dtype=np.int64)
        inverse = np.arange(n_sites)
    return aln, weights, inverse, names


def partials_to_codes(aln):
    """Compact form of tip partials: (codes [ntaxa][S] uint8, table [n_codes][K]) or None
    when there are more than 256 distinct tip vectors."""
    K = aln.shape[-1]
    flat = aln.reshape(-1, K)
    table, inv = np.unique(flat, axis=0, return_inverse=True)
    if len(table) > 256:
        return None
    return (np.asarray(inv).reshape(aln.shape[:-1]).astype(np.uint8),
            np.ascontiguousarray(table, dtype=np.float64))


def alignment_to_codes(alignment, alphabet, compress=True):
    """alignment_to_numpy + partials_to_codes."""
    aln, w, inv, names = alignment_to_numpy(alignment, alphabet, compress)
    enc = partials_to_codes(aln)
    return aln, enc, w, inv, names


def invariant_sites(alignment):
    """Boolean per column: some state is allowed in every taxon (alignment.py:59-66)."""
    return [bool(np.any(reduce(np.logical_and, alignment[:, i, :], np.ones(alignment.shape[2]))))
            for i in range(alignment.shape[1])]


def read_fasta(path_or_text):
    """Minimal FASTA reader -> [(name, seq)] (stands in for Bio.AlignIO, alignment.py:15-17);
    the name is the first whitespace-delimited token of the header."""
    if "\n" in path_or_text or path_or_text.lstrip().startswith(">"):
        text = path_or_text
    else:
        with open(path_or_text) as fh:
            text = fh.read()
    recs, name, buf = [], None, []
    for line in text.splitlines():
        line = line.strip()
        if not line:
            continue
        if line.startswith(">"):
            if name is not None:
                recs.append((name, "".join(buf)))
            name, buf = line[1:].split()[0] if line[1:].split() else "", []
        else:
            buf.append(line)
    if name is not None:
        recs.append((name, "".join(buf)))
    lens = {len(s) for _, s in recs}
    if len(lens) > 1:
        raise ValueError("sequences have different lengths: %s" % sorted(lens))
    return recs


def guess_alphabet(seqs):
    chars = set("".join(s for _, s in _records(seqs))) if not isinstance(seqs, set) else seqs
    return PROTEIN if len(chars - set(dna_charmap)) > 0 else DNA
