"""Multi-part indexes: texts of 2^32 - 2 symbols or more are indexed as parts
split at record boundaries (index_build.hip splitRecords; capi.cpp run merges
the parts' hits), because rows, SA entries and cursors are 32-bit while the
reference's index is size_t-addressed (/root/reference/src/sahara/index.cpp:87).

SAHARA_PART_SYMBOLS lowers the part size so that small texts take the same
path. The bar: every part is the oracle's index of its own records, and the
hits over all parts are exactly the oracle's over one index of all records
(qid, seq_id, pos, err), in every execution mode and through every call
(device-resident, streamed reads, besthits, --max_hits, .idx round trip, CLI).
"""
import os
import subprocess

import numpy as np
import pytest

import oracle as O
import sahara_amd as sa
from helpers import hits_as_rows, mutate_reads, random_records

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LENS = [9000, 40, 7000, 7000, 120, 15000, 3000, 64, 5000]


def _records(seed=11):
    rng = np.random.default_rng(seed)
    recs = random_records(rng, LENS, 6, with_n=True, repeats=True)
    reads = mutate_reads(rng, recs, 900, 70, 2)
    return recs, reads


def _parts_of(lens, limit):
    first, n = [0], 0
    for r, L in enumerate(lens):
        if n and n + L + 1 > limit:
            first.append(r)
            n = 0
        n += L + 1
    return first + [len(lens)]


@pytest.mark.parametrize("limit", [20000, 9001, 1])
def test_parts_are_the_oracle_index_of_their_records(gpu_device, monkeypatch, limit):
    monkeypatch.setenv("SAHARA_PART_SYMBOLS", str(limit))
    recs, _ = _records()
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    first = _parts_of(LENS, max(limit, 2))
    inf = gpu.info()
    assert inf["n_parts"] == len(first) - 1 > 1
    assert inf["n"] == sum(L + 1 for L in LENS) and inf["n_records"] == len(LENS)
    for p in range(len(first) - 1):
        gpu.select_part(p)
        ref = O.Index.build(recs[first[p]:first[p + 1]], 6, 16).export()
        got = gpu.export()
        assert np.array_equal(gpu.export_sa(), ref["sa"])
        for key in ("bwt_f", "bwt_r", "sampled", "samples"):
            assert np.array_equal(got[key], ref[key]), (p, key)
        assert gpu.part_info(p)["kmer_depth"] == inf["kmer_depth"]


@pytest.mark.parametrize("verify,locate_sa", [(True, True), (False, False), (True, False), (False, True)])
def test_multi_part_hits_equal_one_index(gpu_device, monkeypatch, verify, locate_sa):
    monkeypatch.setenv("SAHARA_PART_SYMBOLS", "16000")
    monkeypatch.setenv("SAHARA_BATCH", "301")
    recs, reads = _records()
    pats = sa.interleave_rc(reads, 6)
    sch = sa.search_scheme("h2-k2", 0, 2, reads.shape[1])
    want = hits_as_rows(O.Index.build(recs, 6, 16).search(pats, sch, nthreads=8)[0])
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    assert gpu.info()["n_parts"] > 1
    gpu.set_mode(verify=verify, locate_sa=locate_sa)
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats, sch)), want)
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch)), want)
    gpu.stage(pats, sch)
    assert gpu.run() == len(want)
    assert np.array_equal(hits_as_rows(gpu.fetch()), want)


def test_multi_part_besthits_max_hits_and_hamming(gpu_device, monkeypatch):
    recs, reads = _records(5)
    pats = sa.interleave_rc(reads, 6)
    m = reads.shape[1]
    one = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    monkeypatch.setenv("SAHARA_PART_SYMBOLS", "12000")
    parts = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    assert parts.info()["n_parts"] > 1
    best = [sa.search_scheme("h2-k2", j, j, m) for j in range(3)]
    assert np.array_equal(hits_as_rows(sa.search_best(parts, pats, best)), hits_as_rows(sa.search_best(one, pats, best)))
    sch = sa.search_scheme("h2-k2", 0, 2, m)
    for n in (1, 3):
        assert np.array_equal(hits_as_rows(sa.search(parts, pats, sch, max_hits=n)),
                              hits_as_rows(sa.search(one, pats, sch, max_hits=n)))
    ham = sa.search_scheme("h2-k1", 0, 1, m, hamming=True)
    assert np.array_equal(hits_as_rows(sa.search(parts, pats, ham, edit=False)),
                          hits_as_rows(sa.search(one, pats, ham, edit=False)))


def test_multi_part_idx_round_trip(gpu_device, monkeypatch, tmp_path):
    monkeypatch.setenv("SAHARA_PART_SYMBOLS", "10000")
    recs, reads = _records(7)
    pats = sa.interleave_rc(reads, 6)
    sch = sa.search_scheme("h2-k2", 0, 2, reads.shape[1])
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    np_ = gpu.info()["n_parts"]
    assert np_ > 2
    path = tmp_path / "multi.idx"
    gpu.save(path)
    raw = path.read_bytes()
    assert int.from_bytes(raw[:8], "little") == 6  # the reference's leading size_t sigma (search.cpp:278-283)
    assert int.from_bytes(raw[16:24], "little") == np_
    monkeypatch.delenv("SAHARA_PART_SYMBOLS")
    back = sa.BiFMIndex.load(path, device=gpu_device)
    assert back.info()["n_parts"] == np_
    want = hits_as_rows(O.Index.build(recs, 6, 16).search(pats, sch, nthreads=8)[0])
    assert np.array_equal(hits_as_rows(sa.search(back, pats, sch)), want)
    back2 = sa.BiFMIndex.from_bytes(raw, device=gpu_device)
    assert np.array_equal(hits_as_rows(sa.search(back2, pats, sch)), want)
    with pytest.raises(sa.SaharaError, match="truncated|trailing"):
        sa.BiFMIndex.from_bytes(raw[:-3], device=gpu_device)


def test_multi_part_cli(gpu_device, tmp_path):
    """`sahara index` splits a text into parts (here forced small) and `sahara
    search` over the multi-part .idx prints the same hit lines as over one part."""
    sahara = os.path.join(ROOT, "bin", "sahara")
    recs, reads = _records(3)
    fa = tmp_path / "ref.fa"
    chars = np.frombuffer(b"$ACGNT", np.uint8)
    fa.write_text("".join(f">rec{i} x\n{chars[r].tobytes().decode()}\n" for i, r in enumerate(recs)))
    q = tmp_path / "q.fa"
    q.write_text("".join(f">q{i}\n{chars[r].tobytes().decode()}\n" for i, r in enumerate(reads[:300])))
    outs = []
    for env in ({}, {"SAHARA_PART_SYMBOLS": "15000"}):
        e = dict(os.environ, **env)
        subprocess.run([sahara, "index", str(fa)], check=True, env=e, capture_output=True)
        idx = tmp_path / f"ref{len(env)}.idx"
        os.replace(tmp_path / "ref.fa.idx", idx)
        p = subprocess.run([sahara, "search", "-q", str(q), "-i", str(idx), "-e", "2", "-o", str(tmp_path / "o.txt")],
                           env=e, capture_output=True, text=True)
        assert p.returncode == 0, p.stderr
        outs.append((tmp_path / "o.txt").read_text())
    assert outs[0] == outs[1] and len(outs[0].splitlines()) > 300
    raw = (tmp_path / "ref1.idx").read_bytes()
    assert int.from_bytes(raw[16:24], "little") > 1  # the second index has parts
