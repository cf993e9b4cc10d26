"""The CPU restatement (oracle/) against scheme-independent truths.

Pins the oracle's P-set (qid, seq_id, pos) -> min e to a brute-force DP
(orc_bruteforce) on small texts, and its suffix array / BWT / locate to naive
definitions. The reference has no tests of its own, so these are
the pins; the exact multiset semantics (policy P0) remain unpinned against
upstream fmindex-collection.
"""
import numpy as np
import pytest

import oracle as O
from helpers import hits_as_rows, mutate_reads, pset, random_records


def naive_sa(recs):
    T = []
    for r in recs:
        T += [int(x) for x in r] + [0]
    n = len(T)
    return sorted(range(n), key=lambda i: T[i:]), T


@pytest.mark.parametrize("sigma", [5, 6])
def test_suffix_array_bwt_and_samples(sigma):
    rng = np.random.default_rng(3)
    recs = random_records(rng, [50, 1, 77, 20], sigma, repeats=False)
    recs[0][10:30] = recs[0][0]  # a homopolymer run
    idx = O.Index.build(recs, sigma, 4)
    ex = idx.export()
    sa, T = naive_sa(recs)
    assert ex["sa"].tolist() == sa
    n = len(T)
    assert ex["bwt_f"].tolist() == [T[(p - 1) % n] for p in sa]
    # reverse text = records reversed one by one, same order
    R = []
    for r in recs:
        R += [int(x) for x in r[::-1]] + [0]
    sar = sorted(range(n), key=lambda i: R[i:])
    assert ex["bwt_r"].tolist() == [R[(p - 1) % n] for p in sar]
    # C array
    for c in range(sigma + 1):
        assert ex["C"][c] == sum(1 for x in T if x < c)
    # samples: rows whose in-record offset is a multiple of the rate, and delimiters
    starts = np.cumsum([0] + [len(r) + 1 for r in recs])[:-1]
    exp = []
    for row, p in enumerate(sa):
        rid = np.searchsorted(starts, p, side="right") - 1
        if (p - starts[rid]) % 4 == 0 or p - starts[rid] == len(recs[rid]):
            exp.append(p)
            assert (int(ex["sampled"][row // 64]) >> (row % 64)) & 1
    assert ex["samples"].tolist() == exp


def test_exact_search_matches_string_find():
    rng = np.random.default_rng(5)
    recs = random_records(rng, [400, 300], 6)
    idx = O.Index.build(recs, 6, 16)
    m = 8
    pats = np.stack([recs[i % 2][j:j + m] for i, j in enumerate(rng.integers(0, 290, 30))])
    sch = O.scheme("backtracking", 0, 0, m)
    hits, cnt = idx.search(pats, sch, edit=True)
    got = set(map(tuple, hits_as_rows(hits)[:, :3].tolist()))
    exp = set()
    for q, p in enumerate(pats):
        for s, r in enumerate(recs):
            for i in range(len(r) - m + 1):
                if np.array_equal(r[i:i + m], p):
                    exp.add((q, s, i))
    assert got == exp
    assert cnt["rows"] == len(hits)


CASES = [  # (sigma, edit, k, m, with_n, repeats)
    (6, True, 0, 20, False, False),
    (6, True, 1, 24, True, False),
    (6, True, 2, 24, False, True),
    (6, True, 3, 30, True, False),
    (5, True, 2, 24, False, False),
    (6, False, 1, 24, False, True),
    (6, False, 2, 24, True, False),
    (5, False, 3, 30, False, False),
]


@pytest.mark.parametrize("sigma,edit,k,m,with_n,repeats", CASES)
@pytest.mark.parametrize("gen", ["backtracking", "pigeon", "h2-k1", "h2-k2", "h2-k3", "lam", "kucherov-k1",
                                 "kucherov-k2", "pigeon_opt", "suffix", "01*0", "kianfar", "pex-td", "pex-td-l",
                                 "pex-bu", "pex-bu-l"])
def test_pset_equals_bruteforce(sigma, edit, k, m, with_n, repeats, gen):
    if gen in ("lam", "kucherov-k1", "kucherov-k2", "kianfar") and k > 2:
        return  # tables for k <= 2
    rng = np.random.default_rng(1000 * k + m + sigma + (7 if edit else 0))
    recs = random_records(rng, [600, 250, 400], sigma, with_n=with_n, repeats=repeats)
    pats = mutate_reads(rng, recs, 25, m, k, sigma)
    sch = O.scheme(gen, 0, k, m, hamming=not edit)
    idx = O.Index.build(recs, sigma, 16)
    hits, _ = idx.search(pats, sch, edit=edit)
    bf = O.bruteforce(recs, pats, k, edit=edit)
    assert pset(hits_as_rows(hits)) == pset(hits_as_rows(bf))


def test_threads_do_not_change_the_multiset():
    rng = np.random.default_rng(9)
    recs = random_records(rng, [3000, 2000], 6)
    pats = mutate_reads(rng, recs, 60, 40, 2)
    sch = O.scheme("h2-k2", 0, 2, 40)
    idx = O.Index.build(recs, 6, 16)
    a, ca = idx.search(pats, sch, edit=True, nthreads=1)
    b, cb = idx.search(pats, sch, edit=True, nthreads=4)
    assert np.array_equal(hits_as_rows(a), hits_as_rows(b))
    assert ca == cb


def test_idx_roundtrip(tmp_path):
    rng = np.random.default_rng(11)
    recs = random_records(rng, [500, 90], 6, with_n=True)
    idx = O.Index.build(recs, 6, 16)
    p = tmp_path / "x.idx"
    idx.write(p)
    with open(p, "rb") as f:
        assert int.from_bytes(f.read(8), "little") == 6  # leading size_t sigma (index.cpp:98)
    idx2 = O.Index.read(p)
    a, b = idx.export(with_sa=False), idx2.export(with_sa=False)
    for key in ("bwt_f", "bwt_r", "sampled", "samples", "C"):
        assert np.array_equal(a[key], b[key]), key
    pats = mutate_reads(rng, recs, 10, 20, 1)
    sch = O.scheme("h2-k2", 0, 1, 20)
    assert np.array_equal(hits_as_rows(idx.search(pats, sch)[0]), hits_as_rows(idx2.search(pats, sch)[0]))
