"""Search schemes: completeness, validity, and product == oracle restatement
(search.cpp:174-212 generator/expand, :226 limitToHamming)."""
import numpy as np
import pytest

import oracle as O
import sahara_amd as sa

GENS = ["backtracking", "pigeon", "h2-k1", "h2-k2", "h2-k3", "lam", "kucherov-k1", "kucherov-k2", "pigeon_opt",
        "suffix", "01*0", "kianfar", "pex-td", "pex-td-l", "pex-bu", "pex-bu-l"]
# published tables for k <= 2 only (unknown generator beyond, like upstream's
# generators outside their tables)
KMAX = {"lam": 2, "kucherov-k1": 2, "kucherov-k2": 2, "kianfar": 2}
# the reference's listing (search_scheme.cpp:192); the rest stay unknown here
REFERENCE_ORDER = ["backtracking", "optimum", "01*0", "01*0_opt", "pigeon", "pigeon_opt", "suffix", "h2-k1", "h2-k2",
                   "h2-k3", "kianfar", "kucherov-k1", "kucherov-k2", "lam", "hato", "pex-td", "pex-td-l", "pex-bu",
                   "pex-bu-l"]


def covers(pi, l, u, d):
    acc = 0
    for i, part in enumerate(pi):
        acc += d[part]
        if acc < l[i] or acc > u[i]:
            return False
    return True


def dists(P, lo, hi):
    out = []

    def rec(cur):
        if len(cur) == P:
            if lo <= sum(cur) <= hi:
                out.append(list(cur))
            return
        for e in range(0, hi - sum(cur) + 1):
            rec(cur + [e])
    rec([])
    return out


@pytest.mark.parametrize("gen", GENS)
@pytest.mark.parametrize("k", [0, 1, 2, 3, 4, 5, 6])
def test_complete_and_valid(gen, k):
    if k > KMAX.get(gen, 99):
        with pytest.raises(sa.SaharaError):
            sa.scheme_parts(gen, 0, k)
        return
    for mink in range(0, k + 1):
        pi, l, u = sa.scheme_parts(gen, mink, k)
        P = pi.shape[1]
        for s in range(pi.shape[0]):
            assert sorted(pi[s].tolist()) == list(range(P))
            lo = hi = pi[s][0]
            for x in pi[s][1:]:
                assert x in (lo - 1, hi + 1)
                lo, hi = min(lo, x), max(hi, x)
            assert all(l[s][i] <= u[s][i] for i in range(P))
            assert all(l[s][i] <= l[s][i + 1] and u[s][i] <= u[s][i + 1] for i in range(P - 1))
        for d in dists(P, mink, k):
            assert any(covers(pi[s], l[s], u[s], d) for s in range(pi.shape[0])), (d, gen, mink, k)
        assert O.scheme_complete(gen, mink, k)


@pytest.mark.parametrize("gen", GENS)
@pytest.mark.parametrize("k", [0, 1, 2, 3])
@pytest.mark.parametrize("length", [7, 32, 100, 101, 250])
@pytest.mark.parametrize("ham", [False, True])
def test_product_scheme_equals_oracle(gen, k, length, ham):
    if k > KMAX.get(gen, 99):
        return
    P = sa.scheme_parts(gen, 0, k)[0].shape[1]
    if length < P:
        return
    a = sa.search_scheme(gen, 0, k, length, hamming=ham)
    b = O.scheme(gen, 0, k, length, hamming=ham)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    pi = a[0]
    for s in range(pi.shape[0]):
        assert sorted(pi[s].tolist()) == list(range(length))


def test_default_generator_shape():
    # h2-k2 at k=2: 4 parts, every search starts with an exact part
    pi, l, u = sa.scheme_parts("h2-k2", 0, 2)
    assert pi.shape[1] == 4
    assert all(u[s][0] == 0 for s in range(pi.shape[0]))


def test_unknown_generator_and_short_pattern():
    with pytest.raises(sa.SaharaError, match="valid generators are"):
        sa.search_scheme("nope", 0, 2, 50)
    with pytest.raises(sa.SaharaError):
        sa.search_scheme("h2-k2", 0, 2, 3)  # 4 parts do not fit 3 positions


def test_counts_monotone_in_k():
    prev = 0
    for k in range(0, 4):
        nc, wnc = sa.scheme_counts(sa.search_scheme("h2-k2", 0, k, 100), True, 6, 3e9)
        assert nc > prev and wnc > 0
        prev = nc


@pytest.mark.parametrize("gen,k,m,n", [("h2-k2", 2, 40, 5e3), ("h2-k1", 1, 30, 2e3), ("pigeon", 2, 36, 1e4),
                                       ("h2-k3", 3, 48, 3e3), ("h2-k2", 2, 100, 3e9)])
def test_dynamic_partition(gen, k, m, n):
    """--dynamic_generator: sizes sum to m, no empty part, WNC never above the uniform split,
    and the hit set equals brute force (the sizes only move the search effort)."""
    import numpy as np
    import oracle
    import sahara_amd as sa
    from helpers import mutate_reads, pset, random_records
    (pi, l, u), sizes = sa.search_scheme_dynamic(gen, 0, k, m, text_len=n)
    assert sizes.sum() == m and sizes.min() >= 1
    wd = sa.scheme_counts((pi, l, u), True, 6, n)[1]
    wu = sa.scheme_counts(sa.search_scheme(gen, 0, k, m), True, 6, n)[1]
    assert wd <= wu * (1 + 1e-9)
    if n < 1e6:
        rng = np.random.default_rng(m)
        recs = random_records(rng, [int(n) // 2, int(n) // 2], 6, repeats=True)
        pats = mutate_reads(rng, recs, 40, m, k)
        I = oracle.Index.build(recs, 6)
        h, _ = I.search(pats, (pi, l, u), edit=True)
        assert pset(h) == pset(oracle.bruteforce(recs, pats, k, edit=True))


def test_generators_listed_in_reference_order():
    """list-generators / the error text name the registered generators in the
    reference's order (search_scheme.cpp:192), a subsequence of it."""
    names = list(sa.scheme_generators())
    assert names == [n for n in REFERENCE_ORDER if n in names]
    assert set(GENS) == set(names)


@pytest.mark.parametrize("gen,k,want", [
    ("lam", 2, [([0, 1, 2], [0, 0, 0], [0, 2, 2]), ([2, 1, 0], [0, 0, 0], [0, 1, 2]), ([1, 0, 2], [0, 0, 1], [0, 1, 2])]),
    ("kucherov-k1", 1, [([0, 1], [0, 0], [0, 1]), ([1, 0], [0, 1], [0, 1])]),
    ("pigeon_opt", 2, [([0, 1, 2], [0, 0, 0], [0, 2, 2]), ([1, 2, 0], [0, 0, 1], [0, 1, 2]),
                       ([2, 1, 0], [0, 1, 2], [0, 1, 2])]),
    ("suffix", 2, [([0, 1, 2], [0, 0, 0], [0, 1, 2]), ([1, 2, 0], [0, 0, 0], [0, 1, 2]), ([2, 1, 0], [0, 0, 0], [0, 2, 2])]),
])
def test_published_shapes(gen, k, want):
    """Spot values: Lam et al.'s k = 2 scheme and KST's non-redundant k = 1
    scheme as Kucherov, Salikhov and Tsur (2016) print them (1-based there);
    the pigeonhole and suffix-filter constructions at k = 2."""
    pi, l, u = sa.scheme_parts(gen, 0, k)
    got = [(pi[s].tolist(), l[s].tolist(), u[s].tolist()) for s in range(pi.shape[0])]
    assert got == want


def test_redundancy_where_published_schemes_differ():
    """pigeon_opt's bounds (the parts left of the first error-free part hold
    errors) cover each error distribution at most as often as pigeon's, and
    in total less often; KST's k = 1 scheme is non-redundant, Lam's is not
    (both search the exact match twice)."""
    def multiplicity(gen, k):
        pi, l, u = sa.scheme_parts(gen, 0, k)
        return [sum(covers(pi[s], l[s], u[s], d) for s in range(pi.shape[0])) for d in dists(pi.shape[1], 0, k)]
    for k in (1, 2, 3):
        opt, plain = multiplicity("pigeon_opt", k), multiplicity("pigeon", k)
        assert min(opt) == 1 and all(a <= b for a, b in zip(opt, plain)) and sum(opt) < sum(plain)
    assert set(multiplicity("kucherov-k1", 1)) == {1}
    assert max(multiplicity("lam", 1)) == 2


@pytest.mark.parametrize("gen,k,want", [
    ("pex-td", 2, [([0, 1, 2], [0, 0, 0], [0, 1, 2]), ([1, 0, 2], [0, 0, 0], [0, 1, 2]), ([2, 1, 0], [0, 0, 0], [0, 2, 2])]),
    ("pex-td-l", 2, [([0, 1, 2], [0, 0, 0], [0, 1, 2]), ([1, 0, 2], [0, 1, 1], [0, 1, 2]),
                     ([2, 1, 0], [0, 0, 2], [0, 2, 2])]),
    # K = 4: bottom-up pairs (0 1)(2 3) then merges them, leaf 4 joins last;
    # top-down splits 3 + 2 leaves at the root
    ("pex-bu", 4, [([0, 1, 2, 3, 4], [0] * 5, [0, 1, 3, 3, 4]), ([1, 0, 2, 3, 4], [0] * 5, [0, 1, 3, 3, 4]),
                   ([2, 3, 1, 0, 4], [0] * 5, [0, 1, 3, 3, 4]), ([3, 2, 1, 0, 4], [0] * 5, [0, 1, 3, 3, 4]),
                   ([4, 3, 2, 1, 0], [0] * 5, [0, 4, 4, 4, 4])]),
    ("pex-td", 4, [([0, 1, 2, 3, 4], [0] * 5, [0, 1, 2, 4, 4]), ([1, 0, 2, 3, 4], [0] * 5, [0, 1, 2, 4, 4]),
                   ([2, 1, 0, 3, 4], [0] * 5, [0, 2, 2, 4, 4]), ([3, 4, 2, 1, 0], [0] * 5, [0, 1, 4, 4, 4]),
                   ([4, 3, 2, 1, 0], [0] * 5, [0, 1, 4, 4, 4])]),
    ("kianfar", 2, [([0, 1, 2, 3], [0, 0, 1, 1], [0, 0, 2, 2]), ([2, 1, 0, 3], [0, 0, 0, 0], [1, 1, 2, 2]),
                    ([3, 2, 1, 0], [0, 0, 0, 2], [0, 1, 2, 2])]),
])
def test_pex_and_kianfar_shapes(gen, k, want):
    """The PEX trees (top-down: a node of budget e keeps floor(e / 2) + 1
    leaves on the left; bottom-up: neighbours paired level by level) and
    Kianfar et al.'s K = 2 optimum table, as part-level schemes."""
    pi, l, u = sa.scheme_parts(gen, 0, k)
    got = [(pi[s].tolist(), l[s].tolist(), u[s].tolist()) for s in range(pi.shape[0])]
    assert got == want


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5])
def test_pex_lower_bounds_cut_redundancy(k):
    """With lower bounds (ties to the left child) a PEX scheme covers every
    error distribution at most as often as without, and in total less often;
    for k <= 2 exactly once. (Beyond, cumulative bounds cannot say "the left
    child alone is over its budget", so some overlap stays.)"""
    def mult(gen):
        pi, l, u = sa.scheme_parts(gen, 0, k)
        return [sum(covers(pi[s], l[s], u[s], d) for s in range(pi.shape[0])) for d in dists(pi.shape[1], 0, k)]
    for tree in ("td", "bu"):
        low, plain = mult(f"pex-{tree}-l"), mult(f"pex-{tree}")
        assert min(low) == 1 and all(a <= b for a, b in zip(low, plain)) and sum(low) < sum(plain)
        if k <= 2:
            assert set(low) == {1}
