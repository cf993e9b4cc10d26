"""Streamed query upload at two bits per symbol (capi.cpp uploadChunk,
pack2Avx2 / pack2Scalar; search.hip kUnpack2 / kPatchRank).

CPU: the host packer against a numpy restatement of the format (symbol i at
bits 2 (i % 4) of byte i / 4, A C G T = 0 1 2 3, dna5's N listed by position),
AVX2 and scalar alike, and its rank check.
GPU: sahara_gpu_search[_reads] at 2, 4 and 8 bits per symbol give the
oracle's hits, also with N in the reads and with a chunk so N-rich that it goes
up as nibbles instead.
"""
import numpy as np
import pytest

import oracle as O
import sahara_amd as sa
from helpers import hits_as_rows


def _model_pack2(r, sigma):
    r = np.asarray(r, np.int64)
    code = (r - 1) & 3
    if sigma == 6:
        code = np.where(r == 5, 3, np.where(r == 4, 0, code))
    pad = (-len(code)) % 4
    c = np.concatenate([code, np.zeros(pad, np.int64)]).reshape(-1, 4)
    packed = (c[:, 0] | c[:, 1] << 2 | c[:, 2] << 4 | c[:, 3] << 6).astype(np.uint8)
    npos = np.flatnonzero(r == 4).astype(np.uint32) if sigma == 6 else np.zeros(0, np.uint32)
    return packed, npos


@pytest.mark.parametrize("sigma", [5, 6])
@pytest.mark.parametrize("n", [0, 1, 3, 4, 63, 64, 65, 127, 128, 129, 1000, 4099])
@pytest.mark.parametrize("scalar", [False, True, 2])
def test_pack_2bit_matches_model(sigma, n, scalar):
    rng = np.random.default_rng(n * 7 + sigma)
    r = rng.integers(1, sigma, n).astype(np.uint8)
    if sigma == 6 and n:
        r[rng.integers(0, n, max(1, n // 20))] = 4  # some N
    got, pos, bad = sa.pack_2bit(r, sigma, scalar=scalar)
    want, wpos = _model_pack2(r, sigma)
    assert not bad
    assert np.array_equal(got, want)
    assert np.array_equal(np.sort(pos), wpos)


@pytest.mark.parametrize("sigma", [5, 6])
@pytest.mark.parametrize("value", [0, 7, 200])
@pytest.mark.parametrize("where", [0, 63, 130, 999])
def test_pack_2bit_flags_bad_ranks(sigma, value, where):
    r = np.full(1000, 2, np.uint8)
    r[where] = value
    assert sa.pack_2bit(r, sigma)[2]
    assert sa.pack_2bit(r, sigma, scalar=True)[2]
    assert sa.pack_2bit(r, sigma, scalar=2)[2]
    r[where] = sigma  # one past the alphabet
    assert sa.pack_2bit(r, sigma)[2]


def _inputs(with_n, m=60, n_reads=2000):
    flat, lens = sa.synth_reference([300_000, 200_000], sigma=6, seed=23)
    reads = sa.synth_reads(flat, lens, n_reads, m, 2, sigma=6, seed=29)
    if with_n:
        rng = np.random.default_rng(3)
        mask = rng.random(reads.shape) < 0.01
        reads[mask] = 4
        reads[200:240] = 4  # reads of N only: with 32-read chunks, chunk 6 is N-rich
    pats = sa.interleave_rc(reads, 6)
    sch = sa.search_scheme("h2-k2", 0, 2, m)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ref = O.Index.build([flat[offs[i]:offs[i + 1]] for i in range(len(lens))], 6, 16)
    return flat, lens, reads, pats, sch, ref


@pytest.mark.gpu
@pytest.mark.parametrize("bits", ["2", "4", "8"])
@pytest.mark.parametrize("with_n", [False, True])
def test_streamed_upload_encodings(gpu_device, monkeypatch, bits, with_n):
    """2 bits: straight into the pattern forms (kPackFrom2); 4: nibbles; 8: bytes."""
    monkeypatch.setenv("SAHARA_UPLOAD_BITS", bits)
    monkeypatch.setenv("SAHARA_UPLOAD_CHUNK", "64")
    monkeypatch.setenv("SAHARA_BATCH", "997")
    flat, lens, reads, pats, sch, ref = _inputs(with_n)
    want = hits_as_rows(ref.search(pats, sch, nthreads=8)[0])
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch)), want)
    chunks = gpu.stats()["upload_chunks"]
    assert sum(chunks) == (len(reads) + 31) // 32
    if bits == "2" and with_n:
        assert chunks[1] >= 1 and chunks[0] > chunks[1]  # the N-rich chunk went as nibbles
    else:
        assert chunks[{"2": 0, "4": 1, "8": 2}[bits]] == sum(chunks)
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats, sch)), want)
    odd = pats[:, :59].copy()  # odd length: chunks start mid-byte of the 2-bit stream
    sch59 = sa.search_scheme("h2-k2", 0, 2, 59)
    want59 = hits_as_rows(ref.search(odd, sch59, nthreads=8)[0])
    assert np.array_equal(hits_as_rows(sa.search(gpu, odd, sch59)), want59)


@pytest.mark.gpu
def test_2bit_upload_refuses_bad_rank(gpu_device, monkeypatch):
    monkeypatch.setenv("SAHARA_UPLOAD_BITS", "2")
    monkeypatch.setenv("SAHARA_UPLOAD_CHUNK", "64")
    flat, lens, reads, pats, sch, ref = _inputs(False)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    for v in (0, 6, 9):
        bad = reads.copy()
        bad[1500, 3] = v
        with pytest.raises(sa.SaharaError, match="out of range"):
            sa.search_reads(gpu, bad, sch)
    want = hits_as_rows(ref.search(pats, sch, nthreads=8)[0])
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch)), want)


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"SAHARA_FULL_DOWNLOAD": "1"}, {"SAHARA_HITCAP": "300", "SAHARA_TASKCAP": "200"},
                                 {"SAHARA_PIN_MIN": "0"}, {"SAHARA_PIN_MIN": "0", "SAHARA_COMPACT_DOWNLOAD": "1"}])
def test_hit_download_forms(gpu_device, monkeypatch, env):
    """Hits leave the device whole into a pinned sink, or as 8-B records per
    batch that host threads expand into a pageable one (capi.cpp Expander;
    more batches than staging slots); also through an overflow re-run, with
    every sink pinned (SAHARA_PIN_MIN=0), compact into a pinned sink, and with
    no sink at all (SAHARA_FULL_DOWNLOAD=1 with pageable buffers: copied
    after the pass). Same hits, first call and steady state alike."""
    monkeypatch.setenv("SAHARA_BATCH", "211")
    monkeypatch.setenv("SAHARA_UPLOAD_CHUNK", "100")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    flat, lens, reads, pats, sch, ref = _inputs(True)
    want = hits_as_rows(ref.search(pats, sch, nthreads=8)[0])
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    for _ in range(3):
        assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch)), want)
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats[:777], sch)), want[want[:, 0] < 777])


@pytest.mark.gpu
@pytest.mark.parametrize("m", [17, 32, 33, 250])
def test_2bit_pattern_forms_any_length(gpu_device, monkeypatch, m):
    """kPackFrom2 at lengths with one partial block, exactly one block, one
    symbol more, and C5's 250 (8 blocks): same hits as the byte upload, N
    included, reads and reverse complements alike."""
    monkeypatch.setenv("SAHARA_UPLOAD_CHUNK", "50")
    flat, lens = sa.synth_reference([200_000, 100_000], sigma=6, seed=31)
    reads = sa.synth_reads(flat, lens, 600, m, 2, sigma=6, seed=37)
    reads[np.random.default_rng(m).random(reads.shape) < 0.02] = 4
    sch = sa.search_scheme("h2-k2", 0, 2, m)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    monkeypatch.setenv("SAHARA_UPLOAD_BITS", "8")
    want = hits_as_rows(sa.search_reads(gpu, reads, sch))
    monkeypatch.setenv("SAHARA_UPLOAD_BITS", "2")
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch)), want)
    assert gpu.stats()["upload_chunks"][0] > 1
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ref = O.Index.build([flat[offs[i]:offs[i + 1]] for i in range(len(lens))], 6, 16)
    assert np.array_equal(want, hits_as_rows(ref.search(sa.interleave_rc(reads, 6), sch, nthreads=8)[0]))


@pytest.mark.gpu
@pytest.mark.parametrize("bits", ["2", "4"])
def test_streamed_upload_dna4(gpu_device, monkeypatch, bits):
    """A dna4 index (sigma 5, A C G T = 1..4): the 2-bit codes unpack through
    the dna4 table, no N exists, and an N (rank 5 here) is out of range."""
    monkeypatch.setenv("SAHARA_UPLOAD_BITS", bits)
    monkeypatch.setenv("SAHARA_UPLOAD_CHUNK", "128")
    flat, lens = sa.synth_reference([200_000, 150_000], sigma=5, seed=41)
    reads = sa.synth_reads(flat, lens, 1500, 64, 2, sigma=5, seed=43)
    pats = sa.interleave_rc(reads, 5)
    sch = sa.search_scheme("h2-k2", 0, 2, 64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ref = O.Index.build([flat[offs[i]:offs[i + 1]] for i in range(len(lens))], 5, 16)
    want = hits_as_rows(ref.search(pats, sch, nthreads=8)[0])
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=5, device=gpu_device)
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch)), want)
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats, sch)), want)
    assert gpu.stats()["upload_chunks"][0 if bits == "2" else 1] > 0
    bad = reads.copy()
    bad[700, 9] = 5
    with pytest.raises(sa.SaharaError, match="out of range"):
        sa.search_reads(gpu, bad, sch)
