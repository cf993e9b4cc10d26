"""Reads two bits per symbol (include/sahara_hip.h sahara_gpu_search_packed,
sahara_gpu_search_packed_compact; sahara_read_fasta form 2): the FASTA ingest
writes the packed form straight from the file, and the search calls take it
as it is. CPU: the packed ingest equals the rank ingest packed afterwards.
GPU: the packed calls equal the rank calls (and the oracle) through many
chunks and batches, shards that start inside a byte, N, --no-reverse,
--limit_queries and --max_hits; refused inputs fail loudly."""
import numpy as np
import pytest

import oracle as O
import sahara_amd as sa
from helpers import hits_as_rows


def _write_fasta(path, recs, chars="$ACGNT", width=None, rng=None):
    with open(path, "w") as f:
        for i, r in enumerate(recs):
            s = "".join(chars[c] for c in r)
            if rng is not None and i % 3 == 1:
                s = s.lower()
            f.write(f">read{i} x\n")
            w = width or max(1, len(s))
            for j in range(0, len(s), w):
                f.write(s[j:j + w] + ("\r\n" if i % 4 == 3 else "\n"))


def _model_codes(ranks, sigma):
    code = np.zeros(256, np.uint8)
    code[1], code[2], code[3] = 0, 1, 2
    code[5 if sigma == 6 else 4] = 3
    c = code[ranks]
    c = np.concatenate([c, np.zeros((-len(c)) % 4, np.uint8)]).reshape(-1, 4)
    packed = (c[:, 0] | (c[:, 1] << 2) | (c[:, 2] << 4) | (c[:, 3] << 6)).astype(np.uint8)
    npos = np.flatnonzero(ranks == 4).astype(np.uint64) if sigma == 6 else np.zeros(0, np.uint64)
    return packed, npos


@pytest.mark.parametrize("sigma", [5, 6])
@pytest.mark.parametrize("threads", [1, 3])
def test_packed_fasta_ingest_equals_rank_ingest(tmp_path, sigma, threads):
    rng = np.random.default_rng(sigma * 10 + threads)
    hi = sigma
    recs = [rng.integers(1, hi, int(n)).astype(np.uint8) for n in rng.integers(1, 300, 400)]
    chars = "$ACGNT" if sigma == 6 else "$ACGT"
    p = tmp_path / "q.fa"
    _write_fasta(p, recs, chars, width=37, rng=rng)
    one = sa.read_fasta(str(p), sigma, form=1, threads=threads)
    two = sa.read_fasta(str(p), sigma, form=2, threads=threads)
    flat = np.concatenate(recs)
    assert one["bad"] is None and two["bad"] is None
    assert np.array_equal(one["data"], flat)
    assert np.array_equal(one["offs"], two["offs"]) and two["n_symbols"] == flat.size
    want, wpos = _model_codes(flat, sigma)
    assert np.array_equal(two["data"], want) and np.array_equal(two["n_pos"], wpos)
    # the library packer over the rank form gives the same bytes
    codes, pos, bad = sa.pack_2bit(one["data"], sigma)
    assert not bad and np.array_equal(codes, two["data"]) and np.array_equal(pos.astype(np.uint64), wpos)


@pytest.mark.parametrize("form", [1, 2])
def test_fasta_ingest_reports_first_invalid_character(tmp_path, form):
    p = tmp_path / "bad.fa"
    p.write_text(">a\nACGT\n>b second\nACGNT\nAXG\n>c\nQ\n")
    r = sa.read_fasta(str(p), 6, form=form)
    assert r["bad"] == (1, 6, "X", "b second")
    r = sa.read_fasta(str(p), 5, form=form)  # dna4: the N comes first
    assert r["bad"] == (1, 3, "N", "b second")
    with pytest.raises(sa.SaharaError):
        sa.read_fasta(str(tmp_path / "missing.fa"), 6, form=form)


def _setup(sigma=6, n_reads=3000, m=100, k=2, seed=11, n_frac=0.004):
    flat, lens = sa.synth_reference([200_000, 150_000], sigma=sigma, seed=seed)
    reads = sa.synth_reads(flat, lens, n_reads, m, k, sigma=sigma, seed=seed + 1)
    if sigma == 6 and n_frac:
        reads[np.random.default_rng(seed).random(reads.shape) < n_frac] = 4
    return flat, lens, reads, sa.search_scheme("h2-k2", 0, k, m)


def _ordered(h):
    return np.stack([h["qid"], h["seq_id"], h["pos"], h["err"]], 1).astype(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("batch,chunk,ramp,ramp_end", [(None, None, None, None), ("997", "64", None, None),
                                                       ("211", "100", None, None), ("997", "64", None, "0"),
                                                       ("997", "150", "300:7", "500:1:3")])
def test_packed_calls_equal_rank_calls(gpu_device, monkeypatch, batch, chunk, ramp, ramp_end):
    """(streamed calls end on smaller batches by default, pass.cpp; SAHARA_RAMP /
    SAHARA_RAMP_END set the first and last batches, "0": none)"""
    for var, val in (("SAHARA_BATCH", batch), ("SAHARA_UPLOAD_CHUNK", chunk), ("SAHARA_RAMP", ramp),
                     ("SAHARA_RAMP_END", ramp_end)):
        if val:
            monkeypatch.setenv(var, val)
    flat, lens, reads, sch = _setup()
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    pk = sa.pack_reads(reads, 6)
    assert pk.n_pos.size > 0
    full = sa.search_reads(gpu, reads, sch)
    for _ in range(2):
        c = sa.search_packed_compact(gpu, pk, sch)
        assert np.array_equal(_ordered(c.to_hits()), _ordered(full))
        c.close()
    assert np.array_equal(_ordered(sa.search_packed(gpu, pk, sch)), _ordered(full))
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ref = O.Index.build([flat[offs[i]:offs[i + 1]] for i in range(len(lens))], 6, 16)
    assert np.array_equal(hits_as_rows(full), hits_as_rows(ref.search(sa.interleave_rc(reads, 6), sch, nthreads=8)[0]))


@pytest.mark.gpu
@pytest.mark.parametrize("m", [61, 100, 250])
def test_packed_shards_start_inside_a_byte(gpu_device, monkeypatch, m):
    """Shards of one packed stream (sym0 = r0 * m, any value mod 4), with the
    whole stream's N list: each shard's hits equal the rank call on its reads."""
    monkeypatch.setenv("SAHARA_UPLOAD_CHUNK", "64")
    flat, lens, reads, sch = _setup(n_reads=900, m=m, k=3 if m == 250 else 2, n_frac=0.01)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    pk = sa.pack_reads(reads, 6)
    for r0, r1 in ((0, 300), (3, 301), (301, 602), (601, 900), (899, 900)):
        want = _ordered(sa.search_reads(gpu, reads[r0:r1], sch))
        got = sa.search_packed_compact(gpu, pk.shard(r0, r1), sch)
        assert np.array_equal(_ordered(got.to_hits()), want), (r0, r1)
        got.close()


@pytest.mark.gpu
@pytest.mark.parametrize("reverse,limit", [(False, 0), (True, 777), (False, 500)])
def test_packed_limit_no_reverse_and_max_hits(gpu_device, reverse, limit):
    flat, lens, reads, sch = _setup(n_reads=1200)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    pk = sa.pack_reads(reads, 6)
    want = _ordered(sa.search_reads(gpu, reads, sch, reverse=reverse, limit=limit))
    got = sa.search_packed_compact(gpu, pk, sch, reverse=reverse, limit=limit)
    assert np.array_equal(_ordered(got.to_hits()), want)
    for n in (1, 3):
        assert np.array_equal(_ordered(sa.search_packed(gpu, pk, sch, reverse=reverse, limit=limit, max_hits=n)),
                              _ordered(sa.search_reads(gpu, reads, sch, reverse=reverse, limit=limit, max_hits=n)))


@pytest.mark.gpu
def test_packed_from_fasta_and_dna4(gpu_device, tmp_path):
    """FASTA -> form 2 -> packed call equals FASTA -> ranks -> reads call, on a
    dna5 and a dna4 index; a dna4 index refuses N, and unordered N positions
    are refused; the context stays usable."""
    for sigma in (6, 5):
        flat, lens, reads, sch = _setup(sigma=sigma, n_reads=700, m=64)
        p = tmp_path / f"q{sigma}.fa"
        _write_fasta(p, reads, "$ACGNT" if sigma == 6 else "$ACGT", width=50)
        two = sa.read_fasta(str(p), sigma, form=2)
        gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=sigma, device=gpu_device)
        pk = sa.PackedReads(two["data"], len(reads), 64, two["n_pos"])
        got = sa.search_packed_compact(gpu, pk, sch)
        assert np.array_equal(_ordered(got.to_hits()), _ordered(sa.search_reads(gpu, reads, sch)))
        got.close()
        if sigma == 5:
            bad = sa.PackedReads(two["data"], len(reads), 64, np.array([5], np.uint64))
            with pytest.raises(sa.SaharaError):
                sa.search_packed_compact(gpu, bad, sch)
        else:
            assert two["n_pos"].size > 1
            swapped = two["n_pos"].copy()
            swapped[[0, 1]] = swapped[[1, 0]]
            with pytest.raises(sa.SaharaError):
                sa.search_packed(gpu, sa.PackedReads(two["data"], len(reads), 64, swapped), sch)
        again = sa.search_packed_compact(gpu, pk, sch)  # still usable
        assert len(again) == len(sa.search_reads(gpu, reads, sch))
        again.close()


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"SAHARA_CHUNK_SEEDS": "0"}, {"SAHARA_BATCH": "997"},
                                 {"SAHARA_CHUNK_SEEDS": "0", "SAHARA_BATCH": "997"},
                                 {"SAHARA_UPLOAD_CHUNK": str(1 << 20)}])
def test_packed_first_batch_seeds_in_parts(gpu_device, monkeypatch, env):
    """The first batch's text phase started on its seed tasks (also for a lone
    batch), its seeds in parts, chunk by chunk as each is up (small chunks:
    16 parts; the default chunk size on a call this small: four, as a lone
    C2 batch is cut, staging.cpp); and with one seed launch per batch
    (SAHARA_CHUNK_SEEDS=0)."""
    monkeypatch.setenv("SAHARA_UPLOAD_CHUNK", "150")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    flat, lens, reads, sch = _setup(n_reads=1200)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    want = _ordered(sa.search_reads(gpu, reads, sch))
    pk = sa.pack_reads(reads, 6, pinned=True)
    for _ in range(2):
        got = sa.search_packed_compact(gpu, pk, sch)
        assert np.array_equal(_ordered(got.to_hits()), want)
        got.close()
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ref = O.Index.build([flat[offs[i]:offs[i + 1]] for i in range(len(lens))], 6, 16)
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch)),
                          hits_as_rows(ref.search(sa.interleave_rc(reads, 6), sch, nthreads=8)[0]))
