"""sahara_gpu_search_reads_compact: the hits as 8-B records the device writes
into pinned host memory batch by batch (include/sahara_hip.h
sahara_hit_blocks), decoded on the host. Same multiset and order as
sahara_gpu_search_reads (and the oracle) through many batches and upload
chunks, --limit_queries / --no-reverse, a sink sized too small by the previous
call, many records, dna4; multi-part indexes are refused."""
import os

import numpy as np
import pytest

import oracle as O
import sahara_amd as sa
from helpers import hits_as_rows
from test_cli import read_hits, run
from test_golden import GOLD, IDX


def _setup(sigma=6, nrec=2, n_reads=3000, m=100, k=2, seed=11):
    lens = [200_000 // nrec] * nrec if nrec > 2 else [200_000, 150_000][:nrec]
    flat, lens = sa.synth_reference(lens, sigma=sigma, seed=seed)
    reads = sa.synth_reads(flat, lens, n_reads, m, k, sigma=sigma, seed=seed + 1)
    if sigma == 6:
        reads[np.random.default_rng(seed).random(reads.shape) < 0.005] = 4
    return flat, lens, reads, sa.search_scheme("h2-k2", 0, k, m)


def _rows(c):
    return hits_as_rows(c.to_hits())


def _ordered(h):
    return np.stack([h["qid"], h["seq_id"], h["pos"], h["err"]], 1).astype(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("batch,chunk", [(None, None), ("997", "64"), ("211", "100")])
def test_compact_equals_full_records(gpu_device, monkeypatch, batch, chunk):
    for var, val in (("SAHARA_BATCH", batch), ("SAHARA_UPLOAD_CHUNK", chunk)):
        if val:
            monkeypatch.setenv(var, val)
    flat, lens, reads, sch = _setup()
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    full = sa.search_reads(gpu, reads, sch)
    for _ in range(3):  # first call (sink from the estimate), then from the pool
        c = sa.search_reads_compact(gpu, reads, sch)
        h = c.to_hits()
        assert len(c) == len(full)
        assert np.array_equal(_ordered(h), _ordered(full))  # canonical order, record for record
        assert c.block_end[-1] == len(c) and np.all(np.diff(c.block_end.astype(np.int64)) >= 0)
        c.close()
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ref = O.Index.build([flat[offs[i]:offs[i + 1]] for i in range(len(lens))], 6, 16)
    want = hits_as_rows(ref.search(sa.interleave_rc(reads, 6), sch, nthreads=8)[0])
    assert np.array_equal(hits_as_rows(full), want)


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"SAHARA_PACK_BIND": "1"}, {"SAHARA_PACK_AHEAD": "0"},
                                 {"SAHARA_PACK_AHEAD": "7", "SAHARA_PACK_PIECE": "4096"}])
def test_compact_host_path_settings(gpu_device, monkeypatch, env):
    """The streamed call's host-side variants give the same records:
    packers bound to the GPU's NUMA node, packing on demand (no chunks ahead)
    and many small pieces seven chunks ahead; small batches and chunks so
    that the ring wraps."""
    monkeypatch.setenv("SAHARA_BATCH", "701")
    monkeypatch.setenv("SAHARA_UPLOAD_CHUNK", "96")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    flat, lens, reads, sch = _setup(n_reads=2400)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    want = _ordered(sa.search_reads(gpu, reads, sch))
    for _ in range(2):
        c = sa.search_reads_compact(gpu, reads, sch)
        assert np.array_equal(_ordered(c.to_hits()), want)
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("reverse,limit", [(True, 0), (True, 1999), (False, 0), (False, 777)])
def test_compact_limit_and_no_reverse(gpu_device, monkeypatch, reverse, limit):
    monkeypatch.setenv("SAHARA_BATCH", "500")
    flat, lens, reads, sch = _setup(n_reads=1500)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    want = _ordered(sa.search_reads(gpu, reads, sch, reverse=reverse, limit=limit))
    got = _ordered(sa.search_reads_compact(gpu, reads, sch, reverse=reverse, limit=limit).to_hits())
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_compact_sink_too_small_is_refilled(gpu_device, monkeypatch):
    """A call with far more hits than the last one: the sink (sized from the
    last call) overflows mid-pass; every batch's records are rewritten into
    one that fits, same result."""
    monkeypatch.setenv("SAHARA_BATCH", "300")
    monkeypatch.setenv("SAHARA_PIN_MIN", "0")
    flat, lens, reads, sch = _setup(n_reads=2500)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    small = sa.search_reads_compact(gpu, reads[:40], sch)
    assert np.array_equal(_ordered(small.to_hits()), _ordered(sa.search_reads(gpu, reads[:40], sch)))
    small.close()
    sa.search_reads_compact(gpu, reads[:40], sch).close()  # lastHits = a few hundred
    big = sa.search_reads_compact(gpu, reads, sch)
    assert np.array_equal(_ordered(big.to_hits()), _ordered(sa.search_reads(gpu, reads, sch)))


@pytest.mark.gpu
def test_compact_records_view_outlives_its_call(gpu_device, monkeypatch):
    """`recs` taken from a call's result stays valid after the result object
    is dropped and later calls reuse the library's pinned pool: the view
    keeps its owner (and so the memory) alive."""
    import gc
    monkeypatch.setenv("SAHARA_PIN_MIN", "0")  # every sink comes from the pinned pool
    flat, lens, reads, sch = _setup(n_reads=1500)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    recs = sa.search_reads_compact(gpu, reads, sch).recs
    saved = recs.copy()
    gc.collect()
    for _ in range(3):  # same-size calls: a freed sink would be handed out again here
        sa.search_reads_compact(gpu, reads[::-1].copy(), sch).close()
    assert not recs.flags.writeable
    assert np.array_equal(recs, saved)
    del recs
    # a result dropped without close() frees its memory at once (no cycle
    # keeps it for the garbage collector): the next call reuses the pool
    import weakref
    r = sa.search_reads_compact(gpu, reads, sch)
    owner = weakref.ref(r._own)
    del r
    assert owner() is None
    # close() with a view still alive: the view keeps the memory (the pool
    # cannot hand it to the next calls), and it goes with the view
    r = sa.search_reads_compact(gpu, reads, sch)
    owner = weakref.ref(r._own)
    view = r.recs[::2]
    saved = view.copy()
    r.close()
    assert owner() is not None
    for _ in range(3):
        sa.search_reads_compact(gpu, reads[::-1].copy(), sch).close()
    assert np.array_equal(view, saved)
    del view
    assert owner() is None


@pytest.mark.gpu
@pytest.mark.parametrize("sigma,nrec", [(6, 300), (5, 24)])
def test_compact_many_records_and_dna4(gpu_device, sigma, nrec):
    flat, lens, reads, sch = _setup(sigma=sigma, nrec=nrec, n_reads=2000, m=64)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=sigma, device=gpu_device)
    want = _ordered(sa.search_reads(gpu, reads, sch))
    c = sa.search_reads_compact(gpu, reads, sch)
    assert len(c.rec_starts) == nrec + 1 and c.rec_starts[-1] == gpu.info()["n"]
    assert np.array_equal(_ordered(c.to_hits()), want)
    assert len(np.unique(want[:, 1])) > nrec // 2


@pytest.mark.gpu
def test_compact_refuses_multi_part_index(gpu_device, monkeypatch):
    monkeypatch.setenv("SAHARA_PART_SYMBOLS", "250000")
    flat, lens, reads, sch = _setup(n_reads=100)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    assert gpu.info()["n_parts"] == 2
    with pytest.raises(sa.SaharaError, match="single-part"):
        sa.search_reads_compact(gpu, reads, sch)
    assert len(sa.search_reads(gpu, reads, sch)) > 0  # the context stays usable


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["-e", 2], ["-e", 2, "--no-reverse"], ["-e", 2, "--limit_queries", 71]])
def test_cli_compact_and_full_records_write_the_same_file(args, tmp_path, gpu_device):
    """bin/sahara formats compact records by default (all mode, no
    --max_hits); SAHARA_CLI_FULL_HITS=1 takes whole records: byte-identical
    output files."""
    base = ["search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", os.path.join(GOLD, IDX["a"]), "--emit-errors"]
    a, b = tmp_path / "a.txt", tmp_path / "b.txt"
    rc, _, err = run(*base, "-o", a, *args)
    assert rc == 0, err
    os.environ["SAHARA_CLI_FULL_HITS"] = "1"
    try:
        rc, _, err = run(*base, "-o", b, *args)
    finally:
        del os.environ["SAHARA_CLI_FULL_HITS"]
    assert rc == 0, err
    assert a.read_bytes() == b.read_bytes() and len(read_hits(a, 4)) > 0
