"""Query sharding across GPUs: one process per GPU, the index
replicated on every GPU, contiguous read ranges per rank (a read and its
reverse complement stay together, qids stay contiguous), and the only
communication is a gather of hit records over RCCL (xGMI) / gloo.

Used by bench.py (torchrun, backend "nccl" = RCCL on ROCm) and covered with
world size 2 on gloo by tests/test_multi.py.
"""
from __future__ import annotations

import numpy as np


def shard_bounds(n_reads: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous read range [lo, hi) of `rank`; sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return n_reads * rank // world, n_reads * (rank + 1) // world


def _tensor(a, device):
    import torch
    return torch.as_tensor(np.ascontiguousarray(a)).to(device)


def gather_hits(rows: np.ndarray, qid_offset: int, device="cpu") -> np.ndarray | None:
    """Gather per-rank hit rows (n, 4) u64 = (qid, seq_id, pos, e) with
    rank-local qids to rank 0, in rank order, qids made global.

    Two collectives: an all_gather of the per-rank counts (8 B each), then an
    all_gather of the records padded to the largest count. Returns the
    concatenation on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    rows = np.asarray(rows, dtype=np.uint64).reshape(-1, 4).copy()
    rows[:, 0] += np.uint64(qid_offset)
    cnt = _tensor(np.array([len(rows)], np.int64), device)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [int(c.item()) for c in counts]
    cap = max(max(counts), 1)
    pad = np.zeros((cap, 4), np.int64)
    pad[: len(rows)] = rows.view(np.int64)
    t = _tensor(pad, device)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    if rank != 0:
        return None
    out = [p.cpu().numpy()[:c].view(np.uint64) for p, c in zip(parts, counts)]
    return np.concatenate(out) if out else np.zeros((0, 4), np.uint64)


HIT_WORDS = 3  # a sahara_hit record (24 B) as three int64 words


def gather_hit_records(n_local: int, fill, device="cpu"):
    """Gather every rank's hit records to rank 0 in rank order: the hit
    record gather of SURVEY §8(e), over RCCL (xGMI) on GPUs, gloo on CPU.

    `fill(buf)` writes this rank's n_local records (global qids) into the
    first rows of `buf`, an int64 tensor (cap, 3) on `device` — on a GPU,
    BiFMIndex.copy_hits(buf.data_ptr(), cap, qid_offset) does it on the
    device. One all_gather of the counts (8 B per rank), then one gather of
    the records padded to the largest count. Returns (parts, counts) on rank
    0, parts[r] = rank r's records (counts[r], 3); (None, counts) elsewhere."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    cnt = torch.tensor([int(n_local)], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [int(c.item()) for c in counts]
    cap = max(max(counts), 1)
    buf = torch.zeros((cap, HIT_WORDS), dtype=torch.int64, device=device)
    fill(buf)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gather_list=parts, dst=0)
    if rank != 0:
        return None, counts
    return [p[:c] for p, c in zip(parts, counts)], counts


def gather_compact_records(recs, block_qid0, block_end, qid_offset: int, device="cpu"):
    """Gather every rank's compact hit records — the 8-B records a
    sahara_gpu_search_packed_compact / _reads_compact call leaves in host
    memory (qid - its batch's first qid << 36 | text position << 4 | e) with
    the per-batch block table (first qid, one past the last record) — to
    rank 0 in rank order, over RCCL (xGMI) on GPUs, gloo on CPU. The block
    qids are made global (+ qid_offset, the rank's first pattern) before they
    leave the rank. Three collectives: an all_gather of the counts (records,
    blocks), then a gather of the records and one of the block tables, each
    padded to the largest count. Returns [(recs, block_qid0, block_end)] per
    rank on rank 0, None elsewhere; records_to_rows decodes them."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    recs = np.ascontiguousarray(recs, dtype=np.uint64)
    q0 = np.asarray(block_qid0, dtype=np.uint64) + np.uint64(qid_offset)
    end = np.asarray(block_end, dtype=np.uint64)
    cnt = torch.tensor([len(recs), len(q0)], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [(int(c[0].item()), int(c[1].item())) for c in counts]
    cap = max(max(c[0] for c in counts), 1)
    bcap = max(max(c[1] for c in counts), 1)
    buf = torch.zeros(cap, dtype=torch.int64, device=device)
    if len(recs):
        buf[: len(recs)] = torch.from_numpy(recs.view(np.int64)).to(device)
    blk = torch.zeros((bcap, 2), dtype=torch.int64, device=device)
    if len(q0):
        blk[: len(q0)] = torch.from_numpy(np.stack([q0, end], 1).view(np.int64)).to(device)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    bparts = [torch.empty_like(blk) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gather_list=parts, dst=0)
    dist.gather(blk, gather_list=bparts, dst=0)
    if rank != 0:
        return None
    out = []
    for p, b, (n, nb) in zip(parts, bparts, counts):
        r = p[:n].cpu().numpy().view(np.uint64)
        bt = b[:nb].cpu().numpy().view(np.uint64)
        out.append((r, bt[:, 0].copy(), bt[:, 1].copy()))
    return out


def records_to_rows(recs, block_qid0, block_end, rec_starts) -> np.ndarray:
    """Compact hit records + block table -> (n, 4) u64 rows (qid, seq_id,
    pos, e), as sahara_amd.CompactHits.to_hits decodes them."""
    recs = np.asarray(recs, np.uint64)
    counts = np.diff(np.concatenate([[0], np.asarray(block_end, np.uint64)])).astype(np.int64)
    out = np.empty((len(recs), 4), np.uint64)
    out[:, 0] = np.repeat(np.asarray(block_qid0, np.uint64), counts) + (recs >> np.uint64(36))
    g = (recs >> np.uint64(4)) & np.uint64(0xFFFFFFFF)
    starts = np.asarray(rec_starts, np.uint64)
    seq = np.searchsorted(starts, g, side="right") - 1
    out[:, 1] = seq
    out[:, 2] = g - starts[seq]
    out[:, 3] = recs & np.uint64(15)
    return out


def rows_to_records(rows, rec_starts, batch: int):
    """(n, 4) u64 rows sorted by qid -> compact records and a block table,
    one block per `batch` consecutive qids (the layout of a compact call's
    result; tests build rank-local results with it)."""
    rows = np.asarray(rows, np.uint64).reshape(-1, 4)
    starts = np.asarray(rec_starts, np.uint64)
    q = rows[:, 0]
    q0 = (q // np.uint64(batch)) * np.uint64(batch)
    recs = ((q - q0) << np.uint64(36)) | ((starts[rows[:, 1].astype(np.int64)] + rows[:, 2]) << np.uint64(4)) | rows[:, 3]
    firsts = np.unique(q0)
    end = np.searchsorted(q0, firsts, side="right").astype(np.uint64)
    return recs, firsts, end


def hit_rows_from_records(rec) -> np.ndarray:
    """(n, 3) int64 sahara_hit records -> (n, 4) u64 rows (qid, seq_id, pos, e)."""
    a = np.ascontiguousarray(np.asarray(rec, dtype=np.int64)).view(np.uint64).reshape(-1, HIT_WORDS)
    out = np.empty((len(a), 4), np.uint64)
    out[:, 0] = a[:, 0]
    out[:, 1] = a[:, 1] & np.uint64(0xFFFFFFFF)
    out[:, 2] = a[:, 2]
    out[:, 3] = a[:, 1] >> np.uint64(32)
    return out


def hit_records_from_rows(rows) -> np.ndarray:
    """(n, 4) u64 rows (qid, seq_id, pos, e) -> (n, 3) int64 sahara_hit records."""
    r = np.asarray(rows, dtype=np.uint64).reshape(-1, 4)
    a = np.empty((len(r), HIT_WORDS), np.uint64)
    a[:, 0] = r[:, 0]
    a[:, 1] = (r[:, 1] & np.uint64(0xFFFFFFFF)) | (r[:, 3] << np.uint64(32))
    a[:, 2] = r[:, 2]
    return a.view(np.int64)


def max_over_ranks(x: float, device="cpu") -> float:
    """The slowest rank's time: the whole job's time (bench contract)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def values_of_ranks(x: float, device="cpu") -> list[float]:
    """Every rank's value of x, in rank order (per-rank timings: a slow or
    imbalanced rank shows up by name the first time N GPUs run)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def sum_over_ranks(x: int, device="cpu") -> int:
    import torch
    import torch.distributed as dist

    t = torch.tensor([int(x)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
