"""Shared test helpers: seeded synthetic inputs and multiset comparison."""
import numpy as np

# dna5 codes: A=1 C=2 G=3 N=4 T=5 ; dna4: A=1 C=2 G=3 T=4
ACGT5 = np.array([1, 2, 3, 5], np.uint8)
ACGT4 = np.array([1, 2, 3, 4], np.uint8)


def acgt(sigma):
    return ACGT5 if sigma == 6 else ACGT4


def random_records(rng, lengths, sigma=6, with_n=False, repeats=False):
    recs = []
    for L in lengths:
        r = acgt(sigma)[rng.integers(0, 4, size=L)]
        if repeats and L > 200:
            # plant tandem/interspersed repeats so intervals get large
            unit = r[:rng.integers(3, 12)].copy()
            for _ in range(4):
                p = rng.integers(0, L - 60)
                r[p:p + 60] = np.resize(unit, 60)
        if with_n and sigma == 6 and L > 50:
            p = rng.integers(0, L - 10)
            r[p:p + rng.integers(1, 8)] = 4
        recs.append(r.astype(np.uint8))
    return recs


def mutate_reads(rng, recs, n, m, k, sigma=6):
    """Reads of length m sampled from the records with up to k random S/I/D."""
    out = np.zeros((n, m), np.uint8)
    alpha = acgt(sigma)
    for i in range(n):
        while True:
            r = recs[rng.integers(len(recs))]
            if len(r) >= m + k + 1:
                break
        p = rng.integers(0, len(r) - m - k)
        s = list(r[p:p + m + k])
        for _ in range(k):
            t = rng.integers(3)
            j = rng.integers(len(s))
            if t == 0:
                s[j] = alpha[rng.integers(4)]
            elif t == 1:
                s.insert(j, alpha[rng.integers(4)])
            else:
                del s[j]
        out[i] = np.array(s[:m], np.uint8)
    return out


def hits_as_rows(h):
    """HIT_DTYPE array or (n,4) u64 array -> sorted (n,4) array (qid, seq_id, pos, e)."""
    if h.dtype.names:
        a = np.stack([h["qid"].astype(np.uint64), h["seq_id"].astype(np.uint64),
                      h["pos"].astype(np.uint64), h["err"].astype(np.uint64)], axis=1)
    else:
        a = np.asarray(h, dtype=np.uint64).reshape(-1, 4)
    if len(a) == 0:
        return a
    order = np.lexsort((a[:, 3], a[:, 2], a[:, 1], a[:, 0]))
    return a[order]


def pset(rows):
    """(qid, seq_id, pos) -> min e."""
    d = {}
    for q, s, p, e in rows.tolist():
        k = (q, s, p)
        if k not in d or e < d[k]:
            d[k] = e
    return d
