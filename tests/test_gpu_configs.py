"""GPU parity at the shapes of BASELINE.json's configs (SURVEY §8, config shorthand).

Each case runs the read length, error budget, metric and scheme of one config
against a reference the CPU restatement indexes on its own (O.Index.build:
no part of the GPU's index reaches the checker), in all four execution modes:

- C1 exactly: 1,000 x 32 bp, k = 0, against 1 Mbp (search.cpp:221-231, k = 0);
- C2: k = 1 Hamming (`-d ham`, limitToHamming, search.cpp:226-227), 100 bp,
  substitution-only reads, against a 10 Mbp single-record reference;
- C3 (the bench's workload, reduced): k = 2 Levenshtein, 100 bp, h2-k2 (3
  searches), against a 12 Mbp reference in 24 records, also through the
  streamed packed call the bench times (search.cpp:221-250);
- C5: k = 3 Levenshtein, 250 bp, h2-k2 expanded to 5 searches, against a
  10 Mbp reference in 24 records (GRCh38 proportions, like bench.py).

The bar is P-strict: the multiset of (qid, seq_id, pos, e) equals the
oracle's. Origin recall (every simulated read found on its forward strand
within k positions of where it was sampled) is checked on top.
"""
import numpy as np
import pytest

import oracle as O
import sahara_amd as sa
from helpers import hits_as_rows

pytestmark = pytest.mark.gpu

MODES = [(True, True), (False, False), (True, False), (False, True)]  # (verify, locate_sa)
GRCH38 = [248956422, 242193529, 198295559, 190214555, 181538259, 170805979, 159345973, 145138636,
          138394717, 133797422, 135086622, 133275309, 114364328, 107043718, 101991189, 90338345,
          83257441, 80373285, 58617616, 64444167, 46709983, 50818468, 156040895, 57227415]


def _lens(total, n):
    if n == 1:
        return np.array([total], np.uint64)
    w = np.array(GRCH38[:n], np.float64)
    lens = np.floor(w / w.sum() * total).astype(np.uint64)
    lens[0] += np.uint64(total - int(lens.sum()))
    return lens


def _records(flat, lens):
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    return [flat[offs[i]:offs[i + 1]] for i in range(len(lens))]


def _origin_recall(rows, origin, k):
    """Fraction of reads with a forward-strand hit in their own record within
    k positions of the sampled start (a leading D/I moves the start by <= k)."""
    fwd = rows[rows[:, 0] % 2 == 0]
    read = (fwd[:, 0] // 2).astype(np.int64)
    ok = (fwd[:, 1] == origin[read, 0]) & (np.abs(fwd[:, 2].astype(np.int64) - origin[read, 1].astype(np.int64)) <= k)
    found = np.zeros(len(origin), bool)
    found[read[ok]] = True
    return found.mean()


def _check_config(gpu_device, ref_len, n_rec, n_reads, m, k, edit, n_searches, check_index=False, streamed=False):
    flat, lens = sa.synth_reference(_lens(ref_len, n_rec), sigma=6, seed=42)
    reads, origin = sa.synth_reads(flat, lens, n_reads, m, k if edit else 0, sigma=6, seed=7, with_origin=True,
                                   substitutions=0 if edit else k)
    pats = sa.interleave_rc(reads, 6)
    sch = sa.search_scheme("h2-k2", 0, k, m, hamming=not edit)
    assert sch[0].shape == (n_searches, m)
    # the checker's scheme is the oracle's own expansion of the same generator
    osch = O.scheme("h2-k2", 0, k, m, hamming=not edit)
    assert all(np.array_equal(a, b) for a, b in zip(sch, osch))
    ref = O.Index.build(_records(flat, lens), 6, 16)
    want, _ = ref.search(pats, sch, edit=edit, nthreads=16)
    want = hits_as_rows(want)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    if check_index:  # independent construction at 10 Mbp: the GPU index equals the oracle's
        a, b = ref.export(), gpu.export()
        assert np.array_equal(gpu.export_sa(), a["sa"])
        for key in ("bwt_f", "bwt_r", "sampled", "samples"):
            assert np.array_equal(a[key], b[key]), key
    for verify, locate_sa in MODES:
        gpu.set_mode(verify=verify, locate_sa=locate_sa)
        got = hits_as_rows(sa.search(gpu, pats, sch, edit=edit))
        assert len(got) == len(want), (verify, locate_sa, len(got), len(want))
        assert np.array_equal(got, want), (verify, locate_sa)
    if streamed:  # the bench's call: 2-bit reads in page-locked memory in, compact records out
        gpu.set_mode(verify=True, locate_sa=True)
        rec = sa.search_packed_compact(gpu, sa.pack_reads(reads, 6, pinned=True), sch, edit=edit)
        got = hits_as_rows(rec.to_hits())
        rec.close()
        assert np.array_equal(got, want)
    assert _origin_recall(want, origin, k) == 1.0
    return want


def test_c1_exact_shape(gpu_device):
    """C1: k=0, 1k x 32 bp vs 1 Mbp (BASELINE configs[0])."""
    want = _check_config(gpu_device, 1_000_000, 1, 1000, 32, 0, True, 1)
    assert (want[:, 3] == 0).all()


def test_c2_shape_hamming(gpu_device):
    """C2: k=1 Hamming, 100 bp substitution-only reads, single record."""
    want = _check_config(gpu_device, 10_000_000, 1, 20_000, 100, 1, False, 2, check_index=True)
    assert want[:, 3].max() <= 1


def test_c3_shape_k2_edit_100bp(gpu_device):
    """C3: k=2 Levenshtein, 100 bp, h2-k2 (3 searches), 24 GRCh38-proportioned records."""
    want = _check_config(gpu_device, 12_000_000, 24, 50_000, 100, 2, True, 3, streamed=True)
    assert want[:, 3].max() <= 2 and len(np.unique(want[:, 1])) > 12


def test_c5_shape_k3_250bp(gpu_device):
    """C5: k=3 Levenshtein, 250 bp (two-word text stack, 8+ window blocks), 5 searches, 24 records."""
    want = _check_config(gpu_device, 10_000_000, 24, 5000, 250, 3, True, 5)
    assert want[:, 3].max() <= 3 and len(np.unique(want[:, 1])) > 12
