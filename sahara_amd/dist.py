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


def max_over_ranks(x: float, device="cpu") -> float:
    """The slowest rank's time: the whole job's time (bench contract)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: int, device="cpu") -> int:
    import torch
    import torch.distributed as dist

    t = torch.tensor([int(x)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
