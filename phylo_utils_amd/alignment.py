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
* ``alignment_to_codes`` is the engine's compact form: characters map to uint8 codes
  through a per-alphabet code table ordered like the partial vectors, and the pattern
  compression runs on the GPU (``pu_compress_patterns``) with np.unique's exact result.
"""
from __future__ import annotations

import ctypes
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


def code_table(alphabet):
    """(table [n_codes][K], lut [256] uint8) of an alphabet: the distinct partial vectors of
    its charmap in lexicographic order (np.unique(axis=0)), and per character byte its code
    (255: not in the alphabet).  Codes numbered this way compare like their vectors, so the
    byte order of code columns is the order np.unique gives float partial columns."""
    cmap = CHARMAPS.get(alphabet_code(alphabet))
    if cmap is None:
        raise ValueError("unknown alphabet %r" % alphabet)
    chars = sorted(cmap)
    vecs = np.array([cmap[c] for c in chars], dtype=np.float64)
    table, inv = np.unique(vecs, axis=0, return_inverse=True)
    lut = np.full(256, 255, dtype=np.uint8)
    for c, k in zip(chars, np.asarray(inv).reshape(-1)):
        lut[ord(c)] = k
    return np.ascontiguousarray(table), lut


def char_codes(alignment, alphabet):
    """(codes [ntaxa][S] uint8, table [n_codes][K], names {name: row}): every character
    through the alphabet's code table (seq_to_partials, alignment.py:26-37, as codes)."""
    recs = _records(alignment)
    table, lut = code_table(alphabet)
    if not recs:
        raise ValueError("empty alignment")
    raw = np.stack([np.frombuffer(s.encode("latin-1"), dtype=np.uint8) for _, s in recs])
    codes = lut[raw]
    if (codes == 255).any():
        t, j = np.argwhere(codes == 255)[0]
        raise ValueError("character '%s' is not in the alphabet" % chr(raw[t, j]))
    return codes, table, {n: i for i, (n, _) in enumerate(recs)}


def compress_codes(codes, n_codes, device=0):
    """Site-pattern compression of code columns on the GPU (pu_compress_patterns): the
    (unique [ntaxa][U], counts [U], inverse [S]) of np.unique(codes, axis=1,
    return_inverse=True, return_counts=True) -- alignment.py:40-57's call, bit for bit."""
    from . import _native as N
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    nt, S = codes.shape
    uniq = np.empty(nt * S, dtype=np.uint8)
    counts = np.empty(S, dtype=np.int64)
    inverse = np.empty(S, dtype=np.int64)
    U = ctypes.c_int64()
    N.check(N.lib().pu_compress_patterns(int(device), N.ptr(codes), nt, S, int(n_codes),
                                          N.ptr(uniq), N.ptr(counts), N.ptr(inverse),
                                          ctypes.byref(U)), None, "pu_compress_patterns")
    U = U.value
    return uniq[:nt * U].reshape(nt, U), counts[:U].copy(), inverse


def alignment_to_codes(alignment, alphabet, compress=True, device=0):
    """The engine's form of alignment_to_numpy: (codes [ntaxa][S'], table, siteweights,
    inverse_index, names), with table[codes] equal to alignment_to_numpy's partials and the
    same weights and inverse index.  Pattern compression runs on the GPU."""
    codes, table, names = char_codes(alignment, alphabet)
    if compress:
        codes, weights, inverse = compress_codes(codes, len(table), device)
    else:
        weights = np.ones(codes.shape[1], dtype=np.int64)
        inverse = np.arange(codes.shape[1])
    return codes, table, weights, inverse, names


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
