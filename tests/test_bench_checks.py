"""bench.py's full-size checks, run on CPU against the oracle's index.

bench.verify_index checks the GPU index of the 3 Gbp bench text with torch
ops (suffix order of every adjacent row pair, BWT, samples, C); here the same
function runs on torch's CPU device over an index the CPU restatement built,
and must pass it and catch planted corruptions. bench.origin_recall is held
to reads simulated with their origins.
"""
import sys
import os

import numpy as np
import pytest
import torch

import oracle as O
import sahara_amd as sa
from helpers import hits_as_rows

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


class _OracleIdx:
    """The BiFMIndex calls verify_index makes, served from the oracle: one
    index, or (refs a list) the parts of a multi-part index, each over its
    own records; corrupt(ex) plants an error in part `bad_part`."""

    def __init__(self, ref, lens, sigma=6, rate=16, corrupt=None, bad_part=0):
        refs = ref if isinstance(ref, list) else [ref]
        self.exs = [r.export() for r in refs]
        self.lens, self.sigma, self.rate, self.part = lens, sigma, rate, 0
        if corrupt:
            corrupt(self.exs[bad_part])

    def info(self):
        return {"n": sum(len(e["bwt_f"]) for e in self.exs), "sampling_rate": self.rate, "sigma": self.sigma,
                "n_parts": len(self.exs)}

    def select_part(self, p):
        self.part = p

    def part_info(self, p=None):
        e = self.exs[self.part if p is None else p]
        return {"n": len(e["bwt_f"]), "sampling_rate": self.rate, "sigma": self.sigma, "n_parts": len(self.exs),
                "n_records": len(e["rec_lens"]) if "rec_lens" in e else int((e["bwt_f"] == 0).sum())}

    def export(self):
        e = dict(self.exs[self.part])
        e["C"] = e["C"][: self.sigma + 1]
        return e

    def export_sa(self):
        return self.exs[self.part]["sa"].copy()


def _text(seed=3, lengths=(3000, 17, 900, 2500)):
    flat, lens = sa.synth_reference(list(lengths), sigma=6, seed=seed)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    return flat, lens, [flat[offs[i]:offs[i + 1]] for i in range(len(lens))]


def test_verify_index_passes_on_a_correct_index():
    flat, lens, recs = _text()
    ref = O.Index.build(recs, 6, 16)
    out = bench.verify_index(_OracleIdx(ref, lens), flat, lens, torch, "cpu", W=5)
    assert out["sa_probe_ok"], out
    assert out["index_check_rows"] == len(flat) + len(lens)


def test_verify_index_repetitive_text_needs_many_key_blocks():
    flat, lens, recs = _text()
    flat[:2000] = 1  # long poly-A run (recs are views of flat): adjacent suffixes agree for hundreds of symbols
    ref = O.Index.build(recs, 6, 16)
    out = bench.verify_index(_OracleIdx(ref, lens), flat, lens, torch, "cpu", W=21)
    assert out["sa_probe_ok"], out
    assert out["index_check_max_lcp_blocks"] > 50


def _swap_sa(ex):
    ex["sa"][[100, 2000]] = ex["sa"][[2000, 100]]


def _bwt(ex):
    ex["bwt_f"][77] = 1 if ex["bwt_f"][77] != 1 else 2


def _sample(ex):
    ex["samples"][5] += 1


def _bit(ex):
    ex["sampled"][3] ^= np.uint64(1 << 9)


def _c(ex):
    ex["C"][2] += 1


@pytest.mark.parametrize("corrupt,key", [(_swap_sa, "sa_sorted"), (_bwt, "bwt"), (_sample, "samples"),
                                         (_bit, "samples"), (_c, "C")])
def test_verify_index_catches_corruption(corrupt, key):
    flat, lens, recs = _text()
    ref = O.Index.build(recs, 6, 16)
    out = bench.verify_index(_OracleIdx(ref, lens, corrupt=corrupt), flat, lens, torch, "cpu", W=5)
    assert not out["sa_probe_ok"] and not out["index_checks"][key], out


@pytest.mark.parametrize("corrupt,key", [(None, None), (_swap_sa, "sa_sorted"), (_sample, "samples")])
def test_verify_index_over_parts(corrupt, key):
    """A multi-part index (texts beyond 32-bit rows): every part is checked
    against its own records' text; an error in the second part is caught."""
    flat, lens, recs = _text(lengths=(3000, 17, 900, 2500, 1200))
    refs = [O.Index.build(recs[:2], 6, 16), O.Index.build(recs[2:], 6, 16)]
    out = bench.verify_index(_OracleIdx(refs, lens, corrupt=corrupt, bad_part=1), flat, lens, torch, "cpu", W=5)
    assert out["index_parts"] == 2 and out["index_check_rows"] == len(flat) + len(lens)
    if corrupt is None:
        assert out["sa_probe_ok"], out
    else:
        assert not out["sa_probe_ok"] and not out["index_checks"][key], out


def test_origin_recall():
    flat, lens, recs = _text(lengths=(200_000, 100_000))
    reads, origin = sa.synth_reads(flat, lens, 400, 60, 2, sigma=6, seed=9, with_origin=True)
    pats = sa.interleave_rc(reads, 6)
    sch = sa.search_scheme("h2-k2", 0, 2, 60)
    rows = hits_as_rows(O.Index.build(recs, 6, 16).search(pats, sch, nthreads=4)[0])
    h = np.zeros(len(rows), sa.HIT_DTYPE)
    h["qid"], h["seq_id"], h["pos"], h["err"] = rows[:, 0], rows[:, 1], rows[:, 2], rows[:, 3]
    assert bench.origin_recall(h, origin, 2) == 1.0
    drop = h[h["qid"] != 10]  # read 5's forward hits gone
    assert bench.origin_recall(drop, origin, 2) == pytest.approx(399 / 400)
    moved = h.copy()
    moved["pos"][moved["qid"] == 10] += 50
    assert bench.origin_recall(moved, origin, 2) == pytest.approx(399 / 400)


def _mix64(x):
    M = (1 << 64) - 1
    x ^= x >> 30
    x = (x * 0xbf58476d1ce4e5b9) & M
    x ^= x >> 27
    x = (x * 0x94d049bb133111eb) & M
    return x ^ (x >> 31)


def test_hits_digest_restates_kdigest():
    """bench.hits_digest (numpy, wrapping u64) against the kDigest formula in
    plain Python integers (search.hip kDigest), order-independent."""
    rng = np.random.default_rng(5)
    h = np.zeros(3000, sa.HIT_DTYPE)
    h["qid"] = rng.integers(0, 1 << 40, len(h), dtype=np.uint64)
    h["seq_id"] = rng.integers(0, 1 << 20, len(h), dtype=np.uint32)
    h["pos"] = rng.integers(0, 1 << 33, len(h), dtype=np.uint64)
    h["err"] = rng.integers(0, 16, len(h), dtype=np.uint32)
    M = (1 << 64) - 1
    want = 0
    for r in h.tolist():
        q, s, e, p = r
        inner = _mix64(((s << 40) ^ (p << 4) ^ e) & M)
        want = (want + _mix64(((q * 0x9E3779B97F4A7C15) & M) ^ inner)) & M
    assert bench.hits_digest(h) == want
    assert bench.hits_digest(h[::-1].copy()) == want
    assert bench.hits_digest(h[:-1]) != want
