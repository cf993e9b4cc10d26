"""GPU (HIP, gfx950) vs the CPU restatement: bit-exact multisets.

Every test runs through the C ABI of sahara_amd/lib/libsahara_hip.so.
Parity bar: the multiset of (qid, seq_id, pos, e) records is identical to the
oracle's (oracle/oracle.cpp), and the GPU-built index (SA, both BWTs, C,
samples) equals the oracle's construction byte for byte.
"""
import numpy as np
import pytest

import oracle as O
import sahara_amd as sa
from helpers import hits_as_rows, mutate_reads, pset, random_records

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sigma", [5, 6])
@pytest.mark.parametrize("shape", ["multi", "repeats", "tiny"])
def test_gpu_index_equals_oracle(gpu_device, sigma, shape):
    rng = np.random.default_rng(hash((sigma, shape)) % 2**32)
    if shape == "multi":
        recs = random_records(rng, [5000, 1, 130, 4096, 63, 64, 65], sigma, with_n=True)
    elif shape == "repeats":
        recs = random_records(rng, [6000, 3000], sigma, repeats=True)
        recs[0][100:1100] = recs[0][0]  # long homopolymer: many doubling rounds
    else:
        recs = [np.array([1], np.uint8)]
    ref = O.Index.build(recs, sigma, 16)
    gpu = sa.BiFMIndex.build(recs, sigma=sigma, sampling_rate=16, device=gpu_device)
    a = ref.export()
    b = gpu.export()
    assert np.array_equal(gpu.export_sa(), a["sa"])
    text = np.concatenate([np.append(np.asarray(r, np.uint8), 0) for r in recs])
    assert np.array_equal(gpu.export_text(), text)
    for key in ("bwt_f", "bwt_r", "sampled", "samples"):
        assert np.array_equal(a[key], b[key]), key
    assert np.array_equal(a["C"][: sigma + 1], b["C"])


CASES = [  # sigma, edit, k, m, gen, with_n, repeats
    (6, True, 0, 32, "h2-k2", False, False),
    (6, True, 1, 40, "h2-k2", True, False),
    (6, True, 2, 50, "h2-k2", False, True),
    (6, True, 2, 50, "pigeon", False, False),
    (6, True, 2, 30, "backtracking", True, False),
    (6, True, 3, 60, "h2-k3", False, True),
    (6, True, 3, 60, "h2-k1", False, False),
    (5, True, 2, 50, "h2-k2", False, False),
    (5, True, 3, 40, "h2-k2", False, True),
    (6, False, 1, 40, "h2-k2", False, False),
    (6, False, 2, 50, "h2-k2", True, True),
    (5, False, 3, 60, "pigeon", False, False),
]


MODES = [(True, True), (False, False), (True, False), (False, True)]  # (verify, locate_sa)


@pytest.mark.gpu
@pytest.mark.parametrize("gen,k,edit", [("lam", 2, True), ("kucherov-k1", 1, True), ("kucherov-k2", 2, True),
                                        ("pigeon_opt", 3, True), ("suffix", 2, True), ("01*0", 2, True),
                                        ("01*0", 3, False), ("suffix", 3, False), ("kianfar", 2, True),
                                        ("kianfar", 1, False), ("pex-td", 3, True), ("pex-td-l", 2, True),
                                        ("pex-bu", 4, True), ("pex-bu-l", 3, False)])
def test_gpu_equals_oracle_published_generators(gpu_device, gen, k, edit):
    """Each of the published generators (search_scheme.cpp:192 names): GPU ==
    oracle multiset in every execution mode, seeds from the k-mer table and
    text tasks included."""
    rng = np.random.default_rng(k + len(gen))
    recs = random_records(rng, [20000, 9000], 6, repeats=True)
    reads = mutate_reads(rng, recs, 250, 60, k, 6)
    pats = sa.interleave_rc(reads, 6)
    scheme = sa.search_scheme(gen, 0, k, 60, hamming=not edit)
    want, _ = O.Index.build(recs, 6, 16).search(pats, scheme, edit=edit, nthreads=8)
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    for verify, locate_sa in MODES:
        gpu.set_mode(verify=verify, locate_sa=locate_sa)
        assert np.array_equal(hits_as_rows(sa.search(gpu, pats, scheme, edit=edit)), hits_as_rows(want)), \
            (verify, locate_sa)


@pytest.mark.parametrize("sigma,edit,k,m,gen,with_n,repeats", CASES)
def test_gpu_search_multiset_equals_oracle(gpu_device, sigma, edit, k, m, gen, with_n, repeats):
    rng = np.random.default_rng(7 * k + m + sigma + (1 if edit else 0))
    recs = random_records(rng, [20000, 7000, 3000], sigma, with_n=with_n, repeats=repeats)
    reads = mutate_reads(rng, recs, 300, m, k, sigma)
    pats = sa.interleave_rc(reads, sigma)
    scheme = sa.search_scheme(gen, 0, k, m, hamming=not edit)
    ref = O.Index.build(recs, sigma, 16)
    want, _ = ref.search(pats, scheme, edit=edit, nthreads=8)
    gpu = sa.BiFMIndex.build(recs, sigma=sigma, device=gpu_device)
    for verify, locate_sa in MODES:
        gpu.set_mode(verify=verify, locate_sa=locate_sa)
        got = sa.search(gpu, pats, scheme, edit=edit)
        assert len(got) == len(want), (verify, locate_sa)
        # canonical order out of the ABI
        rows = hits_as_rows(got)
        raw = np.stack([got["qid"], got["seq_id"], got["pos"], got["err"]], 1).astype(np.uint64)
        assert np.array_equal(rows, raw)
        assert np.array_equal(rows, hits_as_rows(want)), (verify, locate_sa)


def test_gpu_pset_equals_bruteforce(gpu_device):
    rng = np.random.default_rng(77)
    recs = random_records(rng, [900, 400], 6, with_n=True, repeats=True)
    reads = mutate_reads(rng, recs, 40, 24, 2)
    scheme = sa.search_scheme("h2-k2", 0, 2, 24)
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    got = sa.search(gpu, reads, scheme, edit=True)
    bf = O.bruteforce(recs, reads, 2, edit=True)
    assert pset(hits_as_rows(got)) == pset(hits_as_rows(bf))


def test_idx_files_cross_load(gpu_device, tmp_path):
    rng = np.random.default_rng(5)
    recs = random_records(rng, [3000, 500], 6, with_n=True)
    ref = O.Index.build(recs, 6, 16)
    p1 = tmp_path / "oracle.idx"
    ref.write(p1)
    g1 = sa.BiFMIndex.load(p1, device=gpu_device)          # oracle-written -> GPU
    # full SA and text densified from the rate-16 samples on load
    assert np.array_equal(g1.export_sa(), ref.export()["sa"])
    text = np.concatenate([np.append(np.asarray(r, np.uint8), 0) for r in recs])
    assert np.array_equal(g1.export_text(), text)
    g2 = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    p2 = tmp_path / "gpu.idx"
    g2.save(p2)
    r2 = O.Index.read(p2)                                    # GPU-written -> oracle
    a, b = ref.export(with_sa=False), r2.export(with_sa=False)
    for key in ("bwt_f", "bwt_r", "sampled", "samples", "C"):
        assert np.array_equal(a[key], b[key]), key
    assert open(p1, "rb").read() == open(p2, "rb").read()     # byte-identical files
    g3 = sa.BiFMIndex.from_bytes(open(p2, "rb").read(), device=gpu_device)
    reads = mutate_reads(rng, recs, 50, 30, 2)
    sch = sa.search_scheme("h2-k2", 0, 2, 30)
    want = hits_as_rows(ref.search(reads, sch)[0])
    for g in (g1, g2, g3):
        for verify, locate_sa in MODES:
            g.set_mode(verify, locate_sa)
            assert np.array_equal(hits_as_rows(sa.search(g, reads, sch)), want)


def test_hit_buffer_overflow_reruns(gpu_device, monkeypatch):
    rng = np.random.default_rng(8)
    recs = random_records(rng, [4000], 6, repeats=True)
    recs[0][:500] = 1  # poly-A: huge intervals, many cursors
    reads = np.vstack([np.full((20, 20), 1, np.uint8), mutate_reads(rng, recs, 30, 20, 1)])
    sch = sa.search_scheme("h2-k2", 0, 1, 20)
    want = hits_as_rows(O.Index.build(recs, 6, 16).search(reads, sch)[0])
    monkeypatch.setenv("SAHARA_HITCAP", "7")
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    got = sa.search(gpu, reads, sch)
    assert np.array_equal(hits_as_rows(got), want)


def test_no_hits_and_device_resident_path(gpu_device):
    rng = np.random.default_rng(9)
    recs = random_records(rng, [5000], 6)
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    sch = sa.search_scheme("h2-k2", 0, 1, 40)
    junk = np.array(rng.integers(1, 4, size=(10, 40)), np.uint8)  # random 40-mers: absent from 5 kbp
    assert len(sa.search(gpu, junk, sch)) == 0
    reads = mutate_reads(rng, recs, 100, 40, 1)
    gpu.set_mode(verify=False, locate_sa=False)  # the reference's own work: FM ranks + LF walks
    direct = sa.search(gpu, reads, sch)
    gpu.stage(reads, sch, edit=True)
    n = gpu.run(count=True)
    st = gpu.stats()
    assert n == len(direct) == st["hits"]
    assert np.array_equal(gpu.fetch(), direct)
    d1 = gpu.digest()
    gpu.run(count=False)
    assert gpu.digest() == d1
    # counters agree with the oracle's deterministic work counts
    ref = O.Index.build(recs, 6, 16)
    _, cnt = ref.search(reads, sch, edit=True)
    assert st["nodes"] == cnt["nodes"]
    assert st["rank_nodes"] == cnt["rank_nodes"]
    assert st["ext_lines"] == cnt["ext_lines"]
    assert st["lf_steps"] == cnt["lf_steps"]
    assert st["cursors"] == cnt["leaves"]
    # verify mode: fewer rank nodes, same hits
    gpu.set_mode(verify=True, locate_sa=True)
    gpu.run(count=True)
    st2 = gpu.stats()
    assert st2["rank_nodes"] < st["rank_nodes"] and st2["conversions"] > 0
    assert np.array_equal(gpu.fetch(), direct)
    # device-side copy for the cross-GPU hit gather: global qids, same records
    import torch
    from sahara_amd.dist import hit_rows_from_records
    buf = torch.full((len(direct) + 5, 3), -1, dtype=torch.int64, device=f"cuda:{gpu_device}")
    assert gpu.copy_hits(buf.data_ptr(), buf.shape[0], qid_offset=1000) == len(direct)
    rows = hit_rows_from_records(buf[: len(direct)].cpu().numpy())
    want = hits_as_rows(direct).copy()
    want[:, 0] += np.uint64(1000)
    assert np.array_equal(rows, want)
    assert (buf[len(direct):] == -1).all()
    with pytest.raises(sa.SaharaError):
        gpu.copy_hits(buf.data_ptr(), len(direct) - 1)


def test_errors_are_loud(gpu_device):
    rng = np.random.default_rng(10)
    recs = random_records(rng, [500], 6)
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    bad = np.zeros((2, 10), np.uint8)  # rank 0 ('$') is not a query symbol
    with pytest.raises(sa.SaharaError, match="rank out of range"):
        sa.search(gpu, bad, sa.search_scheme("h2-k2", 0, 1, 10))
    with pytest.raises(sa.SaharaError, match="no schemes"):
        sa.search_best(gpu, np.ones((1, 10), np.uint8), [])


@pytest.mark.parametrize("k,m,nreads,ref_len", [(2, 100, 20000, 2_000_000), (3, 150, 3000, 1_000_000)])
def test_medium_scale_parity(gpu_device, k, m, nreads, ref_len):
    flat, lens = sa.synth_reference([ref_len // 2, ref_len // 3, ref_len - ref_len // 2 - ref_len // 3],
                                    sigma=6, seed=42)
    reads = sa.synth_reads(flat, lens, nreads, m, k, sigma=6, seed=7)
    pats = sa.interleave_rc(reads, 6)
    sch = sa.search_scheme("h2-k2", 0, k, m)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    got = sa.search(gpu, pats, sch)
    gpu.set_mode(verify=False, locate_sa=False)
    assert np.array_equal(sa.search(gpu, pats, sch), got)
    ex = gpu.export()
    ref = O.Index.from_parts(6, ex["n"], lens, 16, ex["bwt_f"], ex["bwt_r"], ex["sampled"], ex["samples"])
    want, _ = ref.search(pats, sch, edit=True, nthreads=8)
    assert np.array_equal(hits_as_rows(got), hits_as_rows(want))
    # every simulated read is found (forward strand) with <= k errors
    found = np.zeros(nreads, bool)
    found[(got["qid"][got["qid"] % 2 == 0] // 2).astype(np.int64)] = True
    assert found.all()


@pytest.mark.parametrize("nrec", [256, 257, 700])
def test_decode_over_many_records(gpu_device, nrec):
    """Hits decoded to (seq_id, pos) over texts of many short records: the
    record starts sit in LDS for <= 256 records (kSortDecode) and are searched
    in global memory above that."""
    rng = np.random.default_rng(nrec)
    recs = random_records(rng, list(rng.integers(30, 160, size=nrec)), 6)
    m, k = 30, 2
    reads = mutate_reads(rng, recs, 3000, m, k)
    pats = sa.interleave_rc(reads, 6)
    sch = sa.search_scheme("h2-k2", 0, k, m)
    want = hits_as_rows(O.Index.build(recs, 6, 16).search(pats, sch, nthreads=8)[0])
    assert len(np.unique(want[:, 1])) > nrec // 2
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    assert gpu.info()["n_records"] == nrec
    for verify, locate_sa in MODES:
        gpu.set_mode(verify, locate_sa)
        assert np.array_equal(hits_as_rows(sa.search(gpu, pats, sch)), want), (verify, locate_sa)


def test_text_phase_at_record_and_text_boundaries(gpu_device, monkeypatch):
    """Occurrences that touch position 0, the last symbol of the text and
    record delimiters: the text-phase windows are clamped there."""
    rng = np.random.default_rng(21)
    recs = random_records(rng, [60, 45, 200, 33, 90], 6)
    m = 24
    pats = []
    for r in recs:
        pats.append(r[:m])            # record start (incl. text position 0)
        pats.append(r[len(r) - m:])   # record end (incl. the last text symbol)
    pats = np.array(pats, np.uint8)
    pats = np.vstack([pats, mutate_reads(rng, recs, 40, m, 2)])
    # mutate the boundary patterns too
    for i in range(0, 10, 3):
        pats[i, 0] = 1 if pats[i, 0] != 1 else 2
        pats[i + 1, -1] = 1 if pats[i + 1, -1] != 1 else 2
    monkeypatch.setenv("SAHARA_TASKCAP", "5")  # also exercises the task-buffer re-run
    for k in (1, 2, 3):
        sch = sa.search_scheme("h2-k2", 0, k, m)
        want = hits_as_rows(O.Index.build(recs, 6, 16).search(pats, sch)[0])
        gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
        for verify, locate_sa in MODES:
            gpu.set_mode(verify, locate_sa)
            assert np.array_equal(hits_as_rows(sa.search(gpu, pats, sch)), want), (k, verify, locate_sa)


def _repeat_case():
    rng = np.random.default_rng(5)
    unit = random_records(rng, [400], 6)[0]
    parts = []
    for i in range(40):
        u = unit.copy()
        u[rng.integers(0, 400, size=i % 3)] = 1  # near-identical copies: varying error counts
        parts += [u, random_records(rng, [rng.integers(50, 300)], 6)[0]]
    recs = [np.concatenate(parts[:40]), np.concatenate(parts[40:]), random_records(rng, [5000], 6)[0]]
    m, k = 40, 2
    reads = np.vstack([mutate_reads(rng, [unit], 150, m, k), mutate_reads(rng, recs[2:], 150, m, k),
                       random_records(rng, [m] * 40, 6)])
    pats = sa.interleave_rc(reads, 6)
    sch = sa.search_scheme("h2-k2", 0, k, m)
    want = hits_as_rows(O.Index.build(recs, 6, 16).search(pats, sch, nthreads=8)[0])
    return recs, pats, sch, want


def test_sort_decode_tile_holds_every_tier(gpu_device):
    """kSortDecode (search.hip) stages the rows of 256 consecutive queries in
    LDS when they fit its 1024-key tile. Here one such range mixes queries
    without hits with register-sorted (<= 8 rows), wave-sorted (9-64) and
    radix-sorted (> 64) segments, in shuffled order; the range before it holds
    > 1024 rows and takes the global-memory path."""
    recs, pats, sch, want = _repeat_case()
    per_q = np.bincount(want[:, 0].astype(np.int64), minlength=len(pats))
    rng = np.random.default_rng(9)
    pick = [np.flatnonzero(sel)[:n] for sel, n in (((per_q >= 1) & (per_q <= 8), 40), ((per_q > 8) & (per_q <= 64), 4),
                                                   ((per_q > 64) & (per_q <= 300), 1), (per_q == 0, 60))]
    assert all(len(p) for p in pick)
    tile = rng.permutation(np.concatenate(pick))
    assert per_q[tile].sum() <= 1024 and per_q[:256].sum() > 1024
    pats2 = np.vstack([pats[:256], pats[tile]])
    want2 = hits_as_rows(O.Index.build(recs, 6, 16).search(pats2, sch, nthreads=8)[0])
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    for verify, locate_sa in MODES:
        gpu.set_mode(verify, locate_sa)
        assert np.array_equal(hits_as_rows(sa.search(gpu, pats2, sch)), want2), (verify, locate_sa)


@pytest.mark.parametrize("batch", ["97", "1000000"])
def test_segment_sort_and_multi_batch_pipeline(gpu_device, monkeypatch, batch):
    """Per-query segments of every length: reads from a 40-fold repeated unit
    have > 8 located rows (segmented radix sort), unique reads 1-2 (register
    sort), random reads none. SAHARA_BATCH=97 runs many batches through the
    three-stream pipeline, with the per-query counters reused between them."""
    monkeypatch.setenv("SAHARA_BATCH", batch)
    recs, pats, sch, want = _repeat_case()
    per_q = np.bincount(want[:, 0].astype(np.int64), minlength=len(pats))
    assert per_q.max() > 8 and ((per_q >= 1) & (per_q <= 8)).any() and (per_q == 0).any()
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    for verify, locate_sa in MODES:
        gpu.set_mode(verify, locate_sa)
        for _ in range(2):
            assert np.array_equal(hits_as_rows(sa.search(gpu, pats, sch)), want), (verify, locate_sa)


@pytest.mark.parametrize("kmer", ["0", "8", "16"])
def test_kmer_depths_and_seed_tasks(gpu_device, monkeypatch, kmer):
    """The k-mer table only changes where searches start: no table, a shallow
    one, and one as deep as a 3 Gbp index gets (16: on this 1 Mbp text nearly
    every 16-mer is unique, so most searches become text tasks straight from
    kSeedItems). Every depth, with and without that seed-to-task shortcut,
    gives the oracle's multiset."""
    monkeypatch.setenv("SAHARA_KMER", kmer)
    flat, lens = sa.synth_reference([600_000, 400_000], sigma=6, seed=3)
    reads = sa.synth_reads(flat, lens, 4000, 100, 2, sigma=6, seed=11)
    pats = sa.interleave_rc(reads, 6)
    sch = sa.search_scheme("h2-k2", 0, 2, 100)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    ex = gpu.export()
    ref = O.Index.from_parts(6, ex["n"], lens, 16, ex["bwt_f"], ex["bwt_r"], ex["sampled"], ex["samples"])
    want = hits_as_rows(ref.search(pats, sch, edit=True, nthreads=8)[0])
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats, sch)), want)
    monkeypatch.setenv("SAHARA_SEED_TASKS", "0")
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats, sch)), want)


def test_nibble_upload_matches_byte_upload(gpu_device, monkeypatch):
    """Inputs of >= 64M symbols cross PCIe two symbols per byte (capi.cpp
    stageIn) and are expanded on the device: the hits equal those of the
    byte-for-byte upload (SAHARA_NIBBLE_UPLOAD=0), at an odd pattern length
    and an odd pattern count (a lone last nibble). A byte of 16 or more is no
    rank of any alphabet and is refused like any out-of-range rank."""
    flat, lens = sa.synth_reference([600_000, 400_000], sigma=6, seed=5)
    reads = sa.synth_reads(flat, lens, 350_000, 101, 2, sigma=6, seed=13)
    pats = np.ascontiguousarray(sa.interleave_rc(reads, 6)[:-1])
    assert pats.size >= 64 << 20 and pats.size % 2 == 1
    sch = sa.search_scheme("h2-k2", 0, 2, 101)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    monkeypatch.setenv("SAHARA_NIBBLE_UPLOAD", "1")
    got = hits_as_rows(sa.search(gpu, pats, sch))
    monkeypatch.setenv("SAHARA_NIBBLE_UPLOAD", "0")
    want = hits_as_rows(sa.search(gpu, pats, sch))
    assert len(want) >= len(pats) // 2 and np.array_equal(got, want)
    monkeypatch.setenv("SAHARA_NIBBLE_UPLOAD", "1")
    bad = pats.copy()
    bad[-1, -1] = 17
    with pytest.raises(Exception, match="out of range"):
        sa.search(gpu, bad, sch)
    bad[-1, -1] = 7  # a nibble, but no rank of sigma 6: the device check
    with pytest.raises(Exception, match="out of range"):
        sa.search(gpu, bad, sch)


def _streamed_inputs(n_reads=2000, m=60, k=2):
    flat, lens = sa.synth_reference([300_000, 200_000], sigma=6, seed=17)
    reads = sa.synth_reads(flat, lens, n_reads, m, k, sigma=6, seed=19)
    pats = sa.interleave_rc(reads, 6)
    sch = sa.search_scheme("h2-k2", 0, k, m)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ref = O.Index.build([flat[offs[i]:offs[i + 1]] for i in range(len(lens))], 6, 16)
    return flat, lens, reads, pats, sch, ref


@pytest.mark.parametrize("chunk,batch,nibble", [(None, None, "1"), ("64", "97", "1"), ("7", None, "1"),
                                                ("64", "97", "0")])
def test_search_reads_and_streamed_upload(gpu_device, monkeypatch, chunk, batch, nibble):
    """sahara_gpu_search_reads (reverse complements interleaved on the device,
    search.cpp:121-127) and sahara_gpu_search both upload the queries chunk by
    chunk while earlier batches search (SAHARA_UPLOAD_CHUNK patterns per
    chunk, SAHARA_BATCH per batch): same hits as the oracle over the
    interleaved patterns, also cut by --limit_queries (odd: the last read's
    reverse complement dropped) and with --no-reverse."""
    for var, val in (("SAHARA_UPLOAD_CHUNK", chunk), ("SAHARA_BATCH", batch)):
        if val:
            monkeypatch.setenv(var, val)
    monkeypatch.setenv("SAHARA_NIBBLE_UPLOAD", nibble)
    flat, lens, reads, pats, sch, ref = _streamed_inputs()
    want = hits_as_rows(ref.search(pats, sch, nthreads=8)[0])
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats, sch)), want)
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch)), want)
    lim = 2 * 1500 - 1
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch, limit=lim)), want[want[:, 0] < lim])
    fwd = hits_as_rows(ref.search(reads, sch, nthreads=8)[0])
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch, reverse=False)), fwd)
    # the device-resident run over what the streamed call left staged
    gpu.run()
    assert np.array_equal(hits_as_rows(gpu.fetch()), fwd)


@pytest.mark.parametrize("bad_value", [0, 6, 17])
def test_streamed_upload_refuses_bad_rank_in_a_late_chunk(gpu_device, monkeypatch, bad_value):
    """A byte that is no rank (0, >= sigma) in a chunk uploaded while earlier
    batches already search: the call fails loudly, nothing of the bad chunk is
    searched, and the context serves the next call."""
    monkeypatch.setenv("SAHARA_UPLOAD_CHUNK", "64")
    monkeypatch.setenv("SAHARA_BATCH", "97")
    flat, lens, reads, pats, sch, ref = _streamed_inputs()
    want = hits_as_rows(ref.search(pats, sch, nthreads=8)[0])
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    bad = reads.copy()
    bad[1900, 5] = bad_value
    with pytest.raises(sa.SaharaError, match="out of range"):
        sa.search_reads(gpu, bad, sch)
    badp = pats.copy()
    badp[3801, 7] = bad_value
    with pytest.raises(sa.SaharaError, match="out of range"):
        sa.search(gpu, badp, sch)
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch)), want)


def test_pinned_hit_sink_grows_and_is_recycled(gpu_device, monkeypatch):
    """Hits go to pinned host memory batch by batch (SAHARA_PIN_MIN=0 pins
    every size): a call with more hits than the last call's estimate falls
    back to a bigger buffer, freed buffers are reused, and every result is
    the oracle's."""
    monkeypatch.setenv("SAHARA_PIN_MIN", "0")
    monkeypatch.setenv("SAHARA_BATCH", "97")
    flat, lens, reads, pats, sch, ref = _streamed_inputs()
    want = hits_as_rows(ref.search(pats, sch, nthreads=8)[0])
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    small = sa.search_reads(gpu, reads[:40], sch)
    assert np.array_equal(hits_as_rows(small), want[want[:, 0] < 80])
    kept = sa.search_reads(gpu, reads, sch)  # more hits than the estimate from 40 reads
    assert np.array_equal(hits_as_rows(kept), want)
    for _ in range(3):  # steady state: the sink comes back from the pool
        assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch)), want)
    assert np.array_equal(hits_as_rows(kept), want)  # a held buffer is never handed out again
    del small, kept


@pytest.mark.parametrize("m,k,gen", [(400, 2, "h2-k2"), (1000, 2, "h2-k2"), (700, 3, "pigeon")])
def test_long_reads(gpu_device, m, k, gen):
    """Reads far beyond the bench's 100 / 250 bp: windows of more than eight
    blocks copied in rounds (m = 400: one text workgroup per CU), and reads
    whose window and pattern no longer fit the text phase's LDS (m = 700,
    1000), which stay in the FM phase to the end. Same hits as the oracle;
    every read found at its origin."""
    flat, lens = sa.synth_reference([400_000, 250_000], sigma=6, seed=m)
    reads, origin = sa.synth_reads(flat, lens, 300, m, k, sigma=6, seed=k, with_origin=True)
    pats = sa.interleave_rc(reads, 6)
    sch = sa.search_scheme(gen, 0, k, m)
    gpu = sa.BiFMIndex.build_flat(flat, lens, sigma=6, device=gpu_device)
    got = hits_as_rows(sa.search_reads(gpu, reads, sch))
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ref = O.Index.build([flat[offs[i]:offs[i + 1]] for i in range(len(lens))], 6, 16)
    assert np.array_equal(got, hits_as_rows(ref.search(pats, sch, nthreads=8)[0]))
    fwd = got[got[:, 0] % 2 == 0]
    hit = {(int(q) // 2, int(s), int(p)) for q, s, p, e in fwd}
    assert all(any((i, int(origin[i, 0]), int(origin[i, 1]) + d) in hit for d in range(-k, k + 1))
               for i in range(len(reads)))


@pytest.mark.gpu
@pytest.mark.parametrize("steal", ["0", "1", "8", "64"])
def test_text_phase_work_stealing(gpu_device, monkeypatch, steal):
    """Idle lanes of a wave take the bottom stack entry (and the window and
    pattern) of a busy lane once the task queue is dry (SAHARA_STEAL_AT):
    the hits are the oracle's whatever the threshold, on repeat-rich text
    (deep subtrees) with k = 3, several small batches (many launch ends)."""
    monkeypatch.setenv("SAHARA_STEAL_AT", steal)
    monkeypatch.setenv("SAHARA_BATCH", "333")
    rng = np.random.default_rng(77)
    recs = random_records(rng, [30000, 12000], 6, repeats=True)
    reads = mutate_reads(rng, recs, 400, 80, 3, 6)
    pats = sa.interleave_rc(reads, 6)
    scheme = sa.search_scheme("h2-k3", 0, 3, 80)
    want, _ = O.Index.build(recs, 6, 16).search(pats, scheme, edit=True, nthreads=8)
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats, scheme)), hits_as_rows(want))
    gpu.stage(pats, scheme)
    gpu.run()
    assert np.array_equal(hits_as_rows(gpu.fetch()), hits_as_rows(want))


@pytest.mark.gpu
@pytest.mark.parametrize("steal", ["1", "8", "64"])
def test_fm_phase_work_stealing(gpu_device, monkeypatch, steal):
    """kSearchFM: idle lanes of a wave take the bottom stack entry (pattern id
    and search by shuffle) of a busy lane once the seed queue is dry
    (SAHARA_FM_STEAL_AT; the stack is a ring whose bottom moves up). The
    oracle's hits whatever the threshold, in the reference execution (every
    node ranked from the root, LF locate), FM only (no text phase) and the
    default; the node and Occ-line counts equal those without stealing."""
    monkeypatch.setenv("SAHARA_BATCH", "333")
    rng = np.random.default_rng(78)
    recs = random_records(rng, [30000, 12000], 6, repeats=True)
    reads = mutate_reads(rng, recs, 400, 80, 3, 6)
    pats = sa.interleave_rc(reads, 6)
    scheme = sa.search_scheme("h2-k3", 0, 3, 80)
    want = hits_as_rows(O.Index.build(recs, 6, 16).search(pats, scheme, edit=True, nthreads=8)[0])
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    gpu.stage(pats, scheme)
    for mode, split in (((False, False), None), ((True, True), "0"), ((True, True), None)):
        if split:
            monkeypatch.setenv("SAHARA_SPLIT", split)
        else:
            monkeypatch.delenv("SAHARA_SPLIT", raising=False)
        gpu.set_mode(verify=mode[0], locate_sa=mode[1])
        counts = {}
        for at in ("0", steal):
            monkeypatch.setenv("SAHARA_FM_STEAL_AT", at)
            gpu.run(count=True)
            st = gpu.stats()
            counts[at] = (st["nodes"], st["ext_lines"], st["hits"])
            assert np.array_equal(hits_as_rows(gpu.fetch()), want), (mode, split, at)
        assert counts["0"] == counts[steal], (mode, split, counts)
    gpu.set_mode(verify=True, locate_sa=True)
    monkeypatch.delenv("SAHARA_SPLIT", raising=False)
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats, scheme)), want)


@pytest.mark.gpu
@pytest.mark.parametrize("n,batch", [(1, "257"), (2, "257"), (5, "257"), (3, "7")])
def test_max_hits_on_the_device(gpu_device, monkeypatch, n, batch):
    """--max_hits n limited per batch on the device (search.hip limitBatch)
    equals the documented policy (include/sahara_hip.h, test_golden's
    limit_rows) over the oracle's hits: repeat-rich text (queries with many
    positions and several error counts), several batches, reads and
    patterns calls, and besthits. Batches of 7 patterns: 143 batches, past
    the 64 whose per-batch host counters fit one page of pinned memory."""
    from test_golden import limit_rows
    monkeypatch.setenv("SAHARA_BATCH", batch)
    rng = np.random.default_rng(40 + n)
    recs = random_records(rng, [25000, 8000], 6, repeats=True)
    reads = mutate_reads(rng, recs, 500, 50, 2, 6)
    pats = sa.interleave_rc(reads, 6)
    scheme = sa.search_scheme("h2-k2", 0, 2, 50)
    ref = O.Index.build(recs, 6, 16)
    want, _ = ref.search(pats, scheme, edit=True, nthreads=8)
    want = limit_rows(hits_as_rows(want), n)
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats, scheme, max_hits=n)), want)
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, scheme, max_hits=n)), want)
    best = [sa.search_scheme("h2-k2", j, j, 50) for j in range(3)]
    bw = O.search_best(ref, pats, best, nthreads=8)
    assert np.array_equal(hits_as_rows(sa.search_best(gpu, pats, best, max_hits=n)), limit_rows(hits_as_rows(bw), n))


@pytest.mark.parametrize("n", [1, 3, 40])
def test_max_hits_repeats_and_exact_reads(gpu_device, monkeypatch, n):
    """--max_hits n equal to the policy over the oracle's full hits, with
    queries of every kind — exact repeats with hundreds of positions, exact
    reads with a few positions, and reads with 1-2 errors — over several batches, reads with and without reverse
    complements, and the patterns call."""
    from test_golden import limit_rows
    monkeypatch.setenv("SAHARA_BATCH", "173")
    rng = np.random.default_rng(90 + n)
    unit = random_records(rng, [60], 6)[0]
    rep = np.tile(unit, 300)
    rep[rng.integers(0, len(rep), 40)] = rng.integers(1, 6, 40)
    recs = [rep] + random_records(rng, [30000, 9000], 6)
    exact = mutate_reads(rng, recs, 300, 50, 0, 6)
    errs = mutate_reads(rng, recs, 300, 50, 2, 6)
    reads = np.concatenate([exact, errs])[rng.permutation(600)]
    scheme = sa.search_scheme("h2-k2", 0, 2, 50)
    ref = O.Index.build(recs, 6, 16)
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    for rc in (True, False):
        pats = sa.interleave_rc(reads, 6) if rc else reads
        want, _ = ref.search(pats, scheme, edit=True, nthreads=8)
        want = limit_rows(hits_as_rows(want), n)
        assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, scheme, reverse=rc, max_hits=n)), want)
        if rc:
            assert np.array_equal(hits_as_rows(sa.search(gpu, pats, scheme, max_hits=n)), want)
            q_with_n = np.bincount(want[:, 0].astype(np.int64), minlength=len(pats))
            assert (q_with_n == n).any() and (q_with_n < n).any()  # both kinds of query occur


@pytest.mark.parametrize("batch", [None, "37"])
def test_long_and_huge_segments(gpu_device, monkeypatch, batch):
    """Queries with 65..2048 located rows are sorted per workgroup in LDS
    (kSortBigLds, bitonic over the segment padded to a power of two), longer
    ones by the segmented radix sort (kScanTiles lists them): units tiled 90,
    700, 1500 and 2600 times give segments on both sides of 2048 and of every
    power of two, in one batch and across many."""
    if batch:
        monkeypatch.setenv("SAHARA_BATCH", batch)
    rng = np.random.default_rng(77)
    recs, pats = [], []
    for tiles in (90, 700, 1500, 2600):
        unit = random_records(rng, [50], 6)[0]
        r = np.tile(unit, tiles)
        r[rng.integers(0, len(r), tiles // 10)] = rng.integers(1, 6, tiles // 10)
        recs.append(r)
        for s in rng.integers(0, 50, 12):
            p = np.roll(unit, -int(s))[:24].copy()
            if s % 2:
                p[rng.integers(0, 24)] = rng.integers(1, 6)
            pats.append(p)
    pats = np.vstack(pats + random_records(rng, [24] * 8, 6)).astype(np.uint8)
    sch = sa.search_scheme("h2-k1", 0, 1, 24)
    want = hits_as_rows(O.Index.build(recs, 6, 16).search(pats, sch, nthreads=8)[0])
    per_q = np.bincount(want[:, 0].astype(np.int64), minlength=len(pats))
    assert ((per_q > 64) & (per_q <= 2048)).sum() >= 12 and (per_q > 2048).sum() >= 4
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    for verify, locate_sa in MODES:
        gpu.set_mode(verify, locate_sa)
        assert np.array_equal(hits_as_rows(sa.search(gpu, pats, sch)), want), (verify, locate_sa)


@pytest.mark.gpu
@pytest.mark.parametrize("m,k", [(100, 2), (250, 3), (100, 1)])
def test_text_shapes_with_dollar_and_n(gpu_device, monkeypatch, m, k):
    """The compile-time text shapes (m = 100: C2 / C3, m = 250 with k = 3: C5)
    on windows that hold a record delimiter '$' (short records) or an N of the
    text, and patterns that hold an N: the oracle's multiset, in one batch
    and many."""
    rng = np.random.default_rng(m + k)
    lens = [int(x) for x in rng.integers(m // 2, 3 * m, 60)] + [20000, 9000]
    recs = random_records(rng, lens, 6, with_n=True, repeats=True)
    reads = mutate_reads(rng, recs, 300, m, k, 6)
    reads[rng.random(reads.shape) < 0.002] = 4
    pats = sa.interleave_rc(reads, 6)
    scheme = sa.search_scheme("h2-k2", 0, k, m)
    want, _ = O.Index.build(recs, 6, 16).search(pats, scheme, edit=True, nthreads=8)
    want = hits_as_rows(want)
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    for batch in (None, "131"):
        if batch:
            monkeypatch.setenv("SAHARA_BATCH", batch)
        assert np.array_equal(hits_as_rows(sa.search(gpu, pats, scheme)), want), batch
        assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, scheme)), want), batch


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,gen", [(100, 2, "h2-k2"), (60, 3, "h2-k3"), (50, 1, "pigeon"), (80, 2, "pex-bu")])
def test_single_row_seeds_near_text_ends(gpu_device, m, k, gen):
    """Single-row k-mer seeds going straight to the text phase, on reads and
    their reverse complements (mostly random occurrences) and random reads,
    over short records and text ends: the oracle's multiset through the
    staged and the counting pass."""
    rng = np.random.default_rng(m * 10 + k)
    recs = random_records(rng, [60000, 30000, 700, 150], 6, with_n=True, repeats=True)
    reads = np.vstack([mutate_reads(rng, recs, 300, m, k, 6), random_records(rng, [m] * 60, 6)])
    pats = sa.interleave_rc(reads, 6)
    scheme = sa.search_scheme(gen, 0, k, m)
    want = hits_as_rows(O.Index.build(recs, 6, 16).search(pats, scheme, edit=True, nthreads=8)[0])
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats, scheme)), want)
    gpu.stage(pats, scheme)
    gpu.run(count=True)
    assert gpu.stats()["conversions"] > 0
    assert np.array_equal(hits_as_rows(gpu.fetch()), want)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", ["61", "1000"])
def test_text_phase_many_batches(gpu_device, monkeypatch, batch):
    """The text phase per batch (search.hip kSearchTextBatch) with more
    batches than slots (61 patterns per batch: 14 batches over 5 slots),
    repeat-rich text with k = 3 (long tasks, work stealing): the oracle's hits
    through the device-resident pass (plain and count mode), the rank-form
    reads call and the packed call; at least one text launch per batch."""
    monkeypatch.setenv("SAHARA_BATCH", batch)
    rng = np.random.default_rng(505)
    recs = random_records(rng, [30000, 12000], 6, repeats=True)
    reads = mutate_reads(rng, recs, 400, 80, 3, 6)
    pats = sa.interleave_rc(reads, 6)
    scheme = sa.search_scheme("h2-k3", 0, 3, 80)
    want = hits_as_rows(O.Index.build(recs, 6, 16).search(pats, scheme, edit=True, nthreads=8)[0])
    gpu = sa.BiFMIndex.build(recs, sigma=6, device=gpu_device)
    nbatch = -(-len(pats) // int(batch))
    gpu.stage(pats, scheme)
    for count in (False, True):
        gpu.run(count=count)
        st = gpu.stats()
        assert np.array_equal(hits_as_rows(gpu.fetch()), want), count
        assert st["batches"] == nbatch, st
        assert st["text_launches"] >= nbatch, st
    assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, scheme)), want)
    c = sa.search_packed_compact(gpu, sa.pack_reads(reads, 6, pinned=True), scheme)
    got = c.to_hits()
    c.close()
    assert np.array_equal(hits_as_rows(got), want)


@pytest.mark.gpu
def test_buffers_at_high_addresses(gpu_device, tmp_path):
    """Every device buffer placed at an address whose low 32-bit word has bit
    31 set (test hook SAHARA_TEST_HIGH_ADDR=1, device_index.h DevBuf): a
    kernel that rebuilds a 64-bit address from a sign-extended 32-bit half —
    the round-5 fault — would fault or read the wrong memory
    here whatever the allocator does. The oracle's hits in all four execution
    modes, through the streamed packed call, and the rank-form reads call."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "high.py"
    script.write_text(f"""
import sys
sys.path[:0] = {[root, os.path.join(root, "tests"), os.path.join(root, "oracle")]!r}
import numpy as np
import oracle as O
import sahara_amd as sa
from helpers import hits_as_rows, mutate_reads, random_records
rng = np.random.default_rng(3131)
recs = random_records(rng, [40000, 9000, 300], 6, with_n=True, repeats=True)
reads = mutate_reads(rng, recs, 500, 100, 2, 6)
pats = sa.interleave_rc(reads, 6)
sch = sa.search_scheme("h2-k2", 0, 2, 100)
want = hits_as_rows(O.Index.build(recs, 6, 16).search(pats, sch, edit=True, nthreads=8)[0])
gpu = sa.BiFMIndex.build(recs, sigma=6, device={gpu_device})
for verify, locate_sa in [(True, True), (False, False), (True, False), (False, True)]:
    gpu.set_mode(verify=verify, locate_sa=locate_sa)
    assert np.array_equal(hits_as_rows(sa.search(gpu, pats, sch)), want), (verify, locate_sa)
gpu.set_mode(verify=True, locate_sa=True)
rec = sa.search_packed_compact(gpu, sa.pack_reads(reads, 6, pinned=True), sch)
assert np.array_equal(hits_as_rows(rec.to_hits()), want)
rec.close()
assert np.array_equal(hits_as_rows(sa.search_reads(gpu, reads, sch)), want)
print("ok", len(want))
""")
    env = dict(os.environ, SAHARA_TEST_HIGH_ADDR="1", SAHARA_BATCH="301")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
