"""Multi-GPU sharding of a message batch.

With no_context_takeover every message is an independent DEFLATE stream, so
a batch splits into contiguous message ranges, one per rank, balanced by
bytes (Zipf-sized batches would be badly balanced by count).  No payload
ever crosses ranks: each rank copies its own slice to its own GPU and runs
the batch kernels there.  The only collectives are control-plane ones over
`torch.distributed` (RCCL on GPUs, gloo in the CPU tests): an all-gather of
per-rank output byte counts to place every rank's output in one global
layout, and a max-reduce of elapsed times.
"""
from __future__ import annotations

import numpy as np


def byte_balanced_ranges(lens: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous [start, end) message ranges, one per rank: rank r ends at
    the first message whose byte prefix sum reaches (r + 1) / world of the
    total, so every rank gets about the same number of bytes."""
    n = len(lens)
    if world <= 1:
        return [(0, n)]
    csum = np.cumsum(np.asarray(lens, dtype=np.int64))
    total = int(csum[-1]) if n else 0
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        cut = int(np.searchsorted(csum, target, side="left")) + 1 if total else (n * r) // world
        cuts.append(min(max(cut, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def local_slice(data: np.ndarray, off: np.ndarray, lens: np.ndarray, rng: tuple[int, int]):
    """Rank-local copy of messages [start, end): (data, off, lens) rebased
    to start at 0, ready for a host-to-device copy."""
    s, e = rng
    if e <= s:
        return np.zeros(0, np.uint8), np.zeros(0, np.int64), np.zeros(0, np.int32)
    o = np.asarray(off[s:e], dtype=np.int64)
    ln = np.asarray(lens[s:e], dtype=np.int64)
    base, end = int(o[0]), int(o[-1] + ln[-1])
    return (np.ascontiguousarray(data[base:end]), o - base, ln.astype(np.int32))


def global_output_offsets(local_out_bytes: int, group=None):
    """All-gather of every rank's output byte count -> (this rank's byte
    offset in the global output, global total)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    mine = torch.tensor([local_out_bytes], dtype=torch.int64, device=dev)
    allb = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(allb, mine, group=group)
    sizes = [int(t.item()) for t in allb]
    return sum(sizes[:rank]), sum(sizes)


def max_over_ranks(x: float, group=None) -> float:
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
