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
