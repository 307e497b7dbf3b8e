"""GPU site-pattern compression (pu_compress_patterns) against the
reference's own call, np.unique(..., axis=1, return_inverse=True, return_counts=True)
(phylo_utils/alignment/alignment.py:40-57): unique columns, inverse index and counts
bit for bit, over the edge cases of the packing (1 to 8 bits per code, taxa not filling
the last 64-bit word, one site, one taxon, all columns equal or all distinct) and at the
BASELINE cfg4 shard size."""
import numpy as np
import pytest

from phylo_utils_amd import alignment as A
from phylo_utils_amd import _native as N

pytestmark = pytest.mark.gpu


def _ref(codes):
    u, inv, cnt = np.unique(codes, axis=1, return_inverse=True, return_counts=True)
    return u, np.asarray(inv).reshape(-1), cnt


def _check(codes, n_codes):
    u, cnt, inv = A.compress_codes(codes, n_codes)
    ru, rinv, rcnt = _ref(codes)
    np.testing.assert_array_equal(u, ru)
    np.testing.assert_array_equal(inv, rinv)
    np.testing.assert_array_equal(cnt, rcnt)
    assert inv.dtype == np.int64 and cnt.dtype == np.int64


def _with_dups(rng, nt, S, n_codes, frac=0.3):
    codes = rng.integers(0, n_codes, size=(nt, S), dtype=np.uint8)
    dup = rng.random(S) < frac
    codes[:, dup] = codes[:, rng.integers(0, S, size=int(dup.sum()))]
    return codes


@pytest.mark.parametrize("nt,S,n_codes", [
    (5, 1000, 4), (37, 5000, 15), (32, 4000, 15), (16, 3000, 16), (50, 2000, 21),
    (21, 3000, 8), (22, 3000, 5), (9, 2000, 256), (8, 4096, 256), (3, 1000, 2),
    (64, 500, 2), (65, 500, 2), (1, 50, 15), (200, 1, 15), (7, 3000, 1),
    # column pitch padded to 16 words: odd column count (one column per lane), 8-bit codes
    (400, 1001, 15), (700, 3000, 256)])
def test_compress_matches_numpy_unique(nt, S, n_codes):
    rng = np.random.default_rng(nt * 1000 + S + n_codes)
    _check(_with_dups(rng, nt, S, n_codes), n_codes)


def test_compress_degenerate_columns():
    rng = np.random.default_rng(5)
    same = np.tile(rng.integers(0, 15, size=(40, 1), dtype=np.uint8), (1, 777))
    _check(same, 15)                                  # one pattern
    distinct = np.stack([np.arange(600) % 15, np.arange(600) // 15]).astype(np.uint8)
    _check(distinct, 41)                              # every column its own pattern
    # columns equal in all but the last taxon of a partly filled last word
    base = rng.integers(0, 4, size=(70, 1), dtype=np.uint8)
    c = np.tile(base, (1, 64))
    c[-1] = rng.integers(0, 4, size=64)
    _check(c, 4)


def test_compress_conserved_taxa():
    # the first 40 taxa identical in every column: ties survive several refinement rounds
    rng = np.random.default_rng(9)
    c = _with_dups(rng, 100, 20_000, 4)
    c[:40] = c[:40, :1]
    c[60:70] = rng.integers(0, 2, size=(10, 1))
    _check(c, 4)


def test_compress_near_duplicates():
    # duplicated columns then a few changed cells: pairs of columns that differ in one taxon
    # stay tied through many refinement rounds (bench.py --workload patterns's generator)
    rng = np.random.default_rng(7)
    nt, S = 1000, 100_000
    c = rng.integers(0, 4, size=(nt, S), dtype=np.uint8)
    dup = rng.random(S) < 0.3
    c[:, dup] = c[:, rng.integers(0, S, size=int(dup.sum()))]
    amb = rng.random((nt, S)) < 0.001
    c[amb] = rng.integers(0, 15, size=int(amb.sum()))
    _check(c, 15)


@pytest.mark.parametrize("two_sorts,no_settle,no_tail,colmajor", [
    (False, False, False, False), (True, False, False, False), (False, True, False, False),
    (False, False, True, False), (False, False, False, True)])
def test_compress_near_duplicate_families(monkeypatch, two_sorts, no_settle, no_tail, colmajor):
    """Families of near-duplicates: several copies of a column, each changed in one or two
    cells (some at the same word, some to the same value), exact copies among them, and
    copies of copies -- one refinement round orders a family by (side of its first column,
    first differing word, that word); ties go on to the next round.  Both sort forms: the
    (rank, class) composite key and the two 32-bit sorts (taken when the composite does not
    fit 32 bits); with every group sorted (PU_PAT_NO_SETTLE), not settled by k_settle; and
    without the one-workgroup tail (PU_PAT_NO_TAIL); and with the packed words column-major
    (PU_PAT_COLMAJOR) instead of in 16-word slabs."""
    if two_sorts:
        monkeypatch.setenv("PU_PAT_TWO_SORTS", "1")
    if no_settle:
        monkeypatch.setenv("PU_PAT_NO_SETTLE", "1")
    if no_tail:
        monkeypatch.setenv("PU_PAT_NO_TAIL", "1")
    if colmajor:
        monkeypatch.setenv("PU_PAT_COLMAJOR", "1")
    rng = np.random.default_rng(17)
    nt, base = 300, 2000
    c = rng.integers(0, 4, size=(nt, base), dtype=np.uint8)
    fam = [c]
    for k in range(6):
        d = c[:, rng.integers(0, base, size=base)].copy()
        n_ch = rng.integers(0, 3, size=base)          # 0, 1 or 2 changed cells per copy
        for j in range(base):
            for _ in range(n_ch[j]):
                t = rng.integers(0, 40) if k % 2 else rng.integers(0, nt)  # early words, often
                d[t, j] = rng.integers(0, 15)
        fam.append(d)
    c = np.concatenate(fam, axis=1)
    c = np.concatenate([c, c[:, rng.integers(0, c.shape[1], size=3000)]], axis=1)
    _check(c, 15)


def test_compress_big_and_small_groups_in_one_round():
    """One refinement round with both kinds of group (k_settle, r06): groups of up to 16
    members ordered in place by one thread, larger ones by the round's sorts -- here families
    of 2-40 near-duplicates and exact copies around a few base columns, some differing at the
    same word with the same value (ties left for the next round), plus distinct columns."""
    rng = np.random.default_rng(23)
    nt = 150
    parts = [rng.integers(0, 4, size=(nt, 3000), dtype=np.uint8)]
    for size in (2, 3, 15, 16, 17, 18, 40, 40):
        base = rng.integers(0, 4, size=(nt, 1), dtype=np.uint8)
        fam = np.tile(base, (1, size))
        for j in range(size):
            kind = j % 4
            if kind == 1:                                   # one changed cell anywhere
                fam[rng.integers(0, nt), j] = rng.integers(0, 15)
            elif kind == 2:                                 # the same cell, the same value
                fam[5, j] = 9
            elif kind == 3:                                 # the same cell + one more later
                fam[5, j] = 9
                fam[rng.integers(20, nt), j] = rng.integers(0, 15)
        parts.append(fam)
    c = np.concatenate(parts, axis=1)
    c = c[:, rng.permutation(c.shape[1])]
    _check(c, 15)


@pytest.mark.parametrize("no_tail", [False, True])
def test_compress_big_groups_then_tail(monkeypatch, no_tail):
    """Families of 20 and 24 columns equal in word 0 (groups for the round's sorts), whose
    sorted runs (changed at the same late taxa) go on as small groups into the one-workgroup
    tail (k_tail, once at most 1024 columns are tied and no group has more than 16)."""
    if no_tail:
        monkeypatch.setenv("PU_PAT_NO_TAIL", "1")
    rng = np.random.default_rng(29)
    nt = 120
    parts = [rng.integers(0, 4, size=(nt, 4000), dtype=np.uint8)]
    for size in (20, 24, 3):
        base = rng.integers(0, 4, size=(nt, 1), dtype=np.uint8)
        fam = np.tile(base, (1, size))
        fam[3, :] = 7                 # all differ from the base column at word 0 the same way
        fam[100, : size // 2] = 11    # then half of them again, late
        fam[110, ::3] = 12
        parts += [base, fam]
    c = np.concatenate(parts, axis=1)
    c = c[:, rng.permutation(c.shape[1])]
    _check(c, 15)


def test_compress_cfg4_shard_size():
    # BASELINE cfg4 per-GPU shard: 1000 taxa x 125k DNA columns, 30% duplicated
    rng = np.random.default_rng(1)
    _check(_with_dups(rng, 1000, 125_000, 15), 15)


def test_compress_rejects_bad_codes():
    codes = np.zeros((3, 10), dtype=np.uint8)
    codes[1, 4] = 7
    with pytest.raises(N.PhyloHipError, match="n_codes"):
        A.compress_codes(codes, 5)


def test_alignment_to_codes_matches_alignment_to_numpy():
    rng = np.random.default_rng(3)
    pool = np.array(list("ACGTRYN-"))
    cols = pool[rng.integers(0, len(pool), size=(12, 150))]
    seqs = cols[:, rng.integers(0, 150, size=900)]
    recs = [("s%d" % i, "".join(r)) for i, r in enumerate(seqs)]
    parts, w, inv, names = A.alignment_to_numpy(recs, A.DNA)
    codes, table, w2, inv2, names2 = A.alignment_to_codes(recs, A.DNA)
    np.testing.assert_array_equal(table[codes], parts)
    np.testing.assert_array_equal(w2, w)
    np.testing.assert_array_equal(inv2, inv)
    assert names2 == names


def test_compress_device_api_strides():
    """pu_compress_patterns_device on device buffers: compact rows (ld 0, the 1-byte store
    path when U % 4 != 0), padded rows (ld % 4 == 0, wide stores) and an odd output base."""
    import ctypes
    import torch
    rng = np.random.default_rng(21)
    nt, S = 45, 3001
    codes = _with_dups(rng, nt, S, 15)
    ru, rinv, rcnt = _ref(codes)
    dev = torch.device("cuda", 0)
    d_codes = torch.from_numpy(codes).to(dev)
    for ld, off in ((0, 0), (3008, 0), (3008, 1)):
        # off 1: an odd output base (a tensor slice) must not take the 2-byte stores
        d_u = torch.zeros(nt * max(ld, S) + off, dtype=torch.uint8, device=dev)[off:]
        d_c = torch.empty(S, dtype=torch.int64, device=dev)
        d_i = torch.empty(S, dtype=torch.int64, device=dev)
        U = ctypes.c_int64()
        N.check(N.lib().pu_compress_patterns_device(
            0, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream),
            ctypes.c_void_p(d_codes.data_ptr()), nt, S, 15, ctypes.c_void_p(d_u.data_ptr()), ld,
            ctypes.c_void_p(d_c.data_ptr()), ctypes.c_void_p(d_i.data_ptr()), ctypes.byref(U)))
        U = U.value
        rows = ld or U
        u = d_u.cpu().numpy()[:nt * rows].reshape(nt, rows)[:, :U]
        np.testing.assert_array_equal(u, ru)
        np.testing.assert_array_equal(d_c.cpu().numpy()[:U], rcnt)
        np.testing.assert_array_equal(d_i.cpu().numpy(), rinv)
