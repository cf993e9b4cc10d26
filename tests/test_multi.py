"""Multi-rank sharding on CPU: world size 2 over gloo.

Each rank searches its contiguous read shard (reads + reverse complements)
with the CPU restatement, the hits are gathered to rank 0 by
sahara_amd.dist.gather_hits, and the result must equal the single-process
search of all reads. The GPU path uses the same helpers over RCCL (bench.py).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from helpers import hits_as_rows, mutate_reads, random_records

K = 2
M = 40


def _inputs():
    rng = np.random.default_rng(77)
    recs = random_records(rng, [3000, 1200], sigma=6, repeats=True)
    reads = mutate_reads(rng, recs, 45, M, K)
    return recs, reads


def _with_rc(reads):
    comp = np.array([0, 5, 3, 2, 4, 1], np.uint8)
    out = np.empty((2 * len(reads), reads.shape[1]), np.uint8)
    out[0::2] = reads
    out[1::2] = comp[reads[:, ::-1]]
    return out


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import oracle
    from sahara_amd.dist import (gather_hit_records, gather_hits, hit_records_from_rows, hit_rows_from_records,
                                 max_over_ranks, shard_bounds, sum_over_ranks)

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        recs, reads = _inputs()
        lo, hi = shard_bounds(len(reads), world, rank)
        I = oracle.Index.build(recs, sigma=6)
        h, _ = I.search(_with_rc(reads[lo:hi]), oracle.scheme("h2-k2", 0, K, M), edit=True)
        allh = gather_hits(h, qid_offset=2 * lo)
        total = sum_over_ranks(len(h))
        t = max_over_ranks(float(rank + 1))
        # the bench's record gather: fill() writes global-qid records into the buffer
        rows = np.asarray(h, np.uint64).reshape(-1, 4).copy()
        rows[:, 0] += np.uint64(2 * lo)
        rec = hit_records_from_rows(rows)

        def fill(buf):
            buf[: len(rec)] = torch.from_numpy(rec)

        parts, counts = gather_hit_records(len(rec), fill)
        assert counts[rank] == len(rec)
        if rank == 0:
            got2 = np.concatenate([hit_rows_from_records(p.numpy()) for p in parts])
            np.save(os.path.join(outdir, "gathered2.npy"), got2)
            np.save(os.path.join(outdir, "gathered.npy"), allh)
            np.save(os.path.join(outdir, "meta.npy"), np.array([total, t]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_hit_record_layout_round_trip():
    import sahara_amd as sa
    from sahara_amd.dist import hit_records_from_rows, hit_rows_from_records
    rng = np.random.default_rng(3)
    rows = np.stack([rng.integers(0, 2**40, 50), rng.integers(0, 2**31, 50), rng.integers(0, 2**33, 50),
                     rng.integers(0, 4, 50)], 1).astype(np.uint64)
    rec = hit_records_from_rows(rows)
    assert np.array_equal(hit_rows_from_records(rec), rows)
    h = rec.view(sa.HIT_DTYPE).reshape(-1)  # same bytes as the C ABI's sahara_hit
    assert np.array_equal(h["qid"], rows[:, 0]) and np.array_equal(h["seq_id"], rows[:, 1])
    assert np.array_equal(h["pos"], rows[:, 2]) and np.array_equal(h["err"], rows[:, 3])


def test_shard_bounds_partition():
    from sahara_amd.dist import shard_bounds
    for n in (0, 1, 7, 10_000_000, 80_000_000):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1


@pytest.mark.parametrize("world", [2])
def test_two_rank_gather_equals_single_process(world):
    import oracle
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d), nprocs=world, join=True, start_method="spawn")
        got = np.load(os.path.join(d, "gathered.npy"))
        got2 = np.load(os.path.join(d, "gathered2.npy"))
        total, t = np.load(os.path.join(d, "meta.npy"))
    recs, reads = _inputs()
    I = oracle.Index.build(recs, sigma=6)
    want, _ = I.search(_with_rc(reads), oracle.scheme("h2-k2", 0, K, M), edit=True)
    assert len(want) > 0
    assert np.array_equal(hits_as_rows(got), hits_as_rows(want))
    assert np.array_equal(hits_as_rows(got2), hits_as_rows(want))
    assert int(total) == len(want)
    assert t == float(world)  # max over ranks


class _FakeCompact:
    """Stands in for a sahara_gpu_search_packed_compact result on CPU: the
    rank's rows (rank-local qids, sorted) as 8-B compact records with a block
    table of 16-qid batches."""

    def __init__(self, rows, rec_starts):
        from sahara_amd.dist import rows_to_records
        self.rec_starts = rec_starts
        self.recs, self.block_qid0, self.block_end = rows_to_records(rows, rec_starts, 16)


class _FakeWhole:
    """A whole-records result (multi-part index): to_hits() only."""

    def __init__(self, rows):
        import sahara_amd as sa
        self.h = np.zeros(len(rows), sa.HIT_DTYPE)
        for k, f in enumerate(("qid", "seq_id", "pos", "err")):
            self.h[f] = rows[:, k]

    def to_hits(self):
        return self.h


def _bench_gather_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from sahara_amd.dist import gather_compact_records, records_to_rows

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(100 + rank)
        n = 37 + 20 * rank  # ragged per-rank counts
        rec_starts = np.array([0, 1000, 5000, 2**32 - 10], np.uint64)
        seq = rng.integers(0, 3, n).astype(np.uint64)
        rows = np.stack([np.sort(rng.integers(0, 2 * 50, n)), seq,
                         rng.integers(0, 900, n), rng.integers(0, 3, n)], 1).astype(np.uint64)
        res = []
        for obj in (_FakeCompact(rows, rec_starts), _FakeWhole(rows)):
            g = bench.gather_step(obj, getattr(obj, "rec_starts", None), 50, world, rank, dist.barrier, dist, torch,
                                  device="cpu")
            res += [g.get("records", -1), int(bool(g["verified"]))]
        # the gathered records decode to every rank's rows, qids made global
        c = _FakeCompact(rows, rec_starts)
        parts = gather_compact_records(c.recs, c.block_qid0, c.block_end, 2 * 50 * rank)
        mine = rows.copy()
        mine[:, 0] += np.uint64(2 * 50 * rank)
        allrows = [torch.zeros((57, 4), dtype=torch.int64) for _ in range(world)]
        pad = torch.zeros((57, 4), dtype=torch.int64)
        pad[:n] = torch.from_numpy(mine.view(np.int64))
        dist.all_gather(allrows, pad)
        if rank == 0:
            got = np.concatenate([records_to_rows(r, q, e, rec_starts) for r, q, e in parts])
            want = np.concatenate([a.numpy()[: 37 + 20 * r].view(np.uint64) for r, a in enumerate(allrows)])
            res.append(int(np.array_equal(got, want)))
            np.save(os.path.join(outdir, "g.npy"), np.array(res))
    finally:
        dist.destroy_process_group()


def test_bench_gather_step_two_ranks():
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_bench_gather_worker, args=(2, _free_port(), d), nprocs=2, join=True,
                           start_method="spawn")
        r = np.load(os.path.join(d, "g.npy"))
    assert list(r) == [37 + 57, 1, 37 + 57, 1, 1]
