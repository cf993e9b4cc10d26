"""Generate the golden fixtures in tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`). Requires oracle/liboracle.so.

The reference ships no test vectors ("parity unpinned"), so
the fixtures are produced by the CPU restatement in oracle/ and, before being
written, cross-checked against the scheme-independent brute-force DP
(P-set, §8c). What they pin is that every later build — the oracle itself,
the HIP library and the `sahara` CLI — keeps producing exactly these bytes
and hit multisets.

Files:
  ref_a.fa            3 records (1500/800/400 bp, dna5, N runs, planted repeats)
  ref_a.fa.idx        `sahara index ref_a.fa` as written by the restatement
  reads_a.fa          60 reads x 40 bp, up to 2 S/I/D each, plus 4 random reads
  ref_b.fa            1 record 2000 bp (ACGT only)
  ref_b.fa.dna4.idx   `sahara index --dna4 ref_b.fa`
  reads_b.fa          40 reads x 48 bp with 3 S/I/D + 20 with 0-2 substitutions
  hits_*.txt          "qid seqId pos e" per located row, sorted; one file per
                      (fixture, -d, -e, -g, -m) case listed in CASES
  manifest.json       the cases, file sizes and sha256 of every fixture
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402
from helpers import mutate_reads, random_records  # noqa: E402

CHARS = {6: "$ACGNT", 5: "$ACGT"}

# (name, fixture, sigma, metric, k, generator, mode, reverse)
CASES = [
    ("a_lev_k0", "a", 6, "lev", 0, "h2-k2", "all", True),
    ("a_lev_k1", "a", 6, "lev", 1, "h2-k2", "all", True),
    ("a_lev_k2", "a", 6, "lev", 2, "h2-k2", "all", True),
    ("a_ham_k2", "a", 6, "ham", 2, "h2-k2", "all", True),
    ("a_lev_k2_pigeon_norev", "a", 6, "lev", 2, "pigeon", "all", False),
    ("a_best_k2", "a", 6, "lev", 2, "h2-k2", "besthits", True),
    ("b_lev_k3", "b", 5, "lev", 3, "h2-k3", "all", True),
    ("b_ham_k2_backtracking", "b", 5, "ham", 2, "backtracking", "all", True),
]


def write_fasta(path, names, seqs, sigma, width=60):
    with open(path, "w") as f:
        for n, s in zip(names, seqs):
            txt = "".join(CHARS[sigma][c] for c in s)
            f.write(f">{n}\n")
            for i in range(0, len(txt), width):
                f.write(txt[i:i + width] + "\n")


def rc(p, sigma):
    comp = {6: [0, 5, 3, 2, 4, 1], 5: [0, 4, 3, 2, 1]}[sigma]
    return np.array([comp[c] for c in p[::-1]], np.uint8)


def patterns(reads, sigma, reverse):
    """search.cpp:111-124: qid 2i = read i, 2i+1 = its reverse complement."""
    out = []
    for r in reads:
        out.append(r)
        if reverse:
            out.append(rc(r, sigma))
    return np.array(out, np.uint8)


def make_inputs():
    rng = np.random.default_rng(20241015)
    ref_a = random_records(rng, [1500, 800, 400], sigma=6, with_n=True, repeats=True)
    reads_a = mutate_reads(rng, ref_a, 60, 40, 2, sigma=6)
    junk = np.array([1, 2, 3, 5], np.uint8)[rng.integers(0, 4, size=(4, 40))]
    reads_a = np.concatenate([reads_a, junk])
    ref_b = random_records(rng, [2000], sigma=5)
    reads_b = mutate_reads(rng, ref_b, 40, 48, 3, sigma=5)
    subs = []  # substitution-only reads so the Hamming cases have hits
    for _ in range(20):
        p = int(rng.integers(0, 2000 - 48))
        r = ref_b[0][p:p + 48].copy()
        for j in rng.choice(48, size=int(rng.integers(0, 3)), replace=False):
            r[j] = 1 + (r[j] + int(rng.integers(0, 3))) % 4
        subs.append(r)
    reads_b = np.concatenate([reads_b, np.array(subs, np.uint8)])
    return {"a": (ref_a, reads_a, 6), "b": (ref_b, reads_b, 5)}


def sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def main():
    inputs = make_inputs()
    files = {}
    idx = {}
    for key, (recs, reads, sigma) in inputs.items():
        ref = os.path.join(HERE, f"ref_{key}.fa")
        write_fasta(ref, [f"chr{i + 1} fixture {key}" for i in range(len(recs))], recs, sigma)
        write_fasta(os.path.join(HERE, f"reads_{key}.fa"), [f"read{i}" for i in range(len(reads))],
                    reads, sigma, width=1000)
        I = oracle.Index.build(recs, sigma=sigma, rate=16)
        ipath = ref + (".idx" if sigma == 6 else ".dna4.idx")
        I.write(ipath)
        idx[key] = I
        files[os.path.basename(ref)] = None
        files[f"reads_{key}.fa"] = None
        files[os.path.basename(ipath)] = None
    cases = []
    for name, key, sigma, metric, k, gen, mode, reverse in CASES:
        recs, reads, _ = inputs[key]
        pats = patterns(reads, sigma, reverse)
        edit = metric == "lev"
        m = pats.shape[1]
        if mode == "all":
            sch = oracle.scheme(gen, 0, k, m, hamming=not edit)
            hits, _ = idx[key].search(pats, sch, edit=edit)
            # P-set check against the brute-force DP before anything is written
            bf = oracle.bruteforce(recs, pats, k, edit=edit)
            got = {}
            for q, s, p, e in hits.tolist():
                got[(q, s, p)] = min(e, got.get((q, s, p), 99))
            want = {(q, s, p): e for q, s, p, e in bf.tolist()}
            assert got == want, f"{name}: restatement disagrees with brute force"
        else:
            schemes = [oracle.scheme(gen, j, j, m) for j in range(k + 1)]
            hits = oracle.search_best(idx[key], pats, schemes)
            bf = oracle.bruteforce(recs, pats, k, edit=True)
            best = {}
            for q, s, p, e in bf.tolist():
                best[q] = min(e, best.get(q, 99))
            assert {int(q) for q in hits[:, 0]} == set(best), f"{name}: besthits query set"
            for q, s, p, e in hits.tolist():
                assert e == best[q], f"{name}: besthits error count"
        hits = hits[np.lexsort((hits[:, 3], hits[:, 2], hits[:, 1], hits[:, 0]))]
        out = os.path.join(HERE, f"hits_{name}.txt")
        np.savetxt(out, hits, fmt="%d")
        files[os.path.basename(out)] = None
        cases.append(dict(name=name, fixture=key, sigma=sigma, metric=metric, k=k, generator=gen,
                          mode=mode, reverse=reverse, hits=len(hits), patterns=int(pats.shape[0])))
        print(f"{name:28s} patterns={pats.shape[0]:4d} hits={len(hits)}")
    for f in files:
        p = os.path.join(HERE, f)
        files[f] = dict(bytes=os.path.getsize(p), sha256=sha(p))
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(dict(cases=cases, files=files), f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
