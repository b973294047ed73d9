"""Sharding of independent verification units across ranks (one process per GPU).

The hot path has no exchange step: each rank verifies a contiguous shard
and only the per-item verdict bitmaps come back — one gather of ceil(n/8) bytes, the
"trivial gather" of the north star. Shards are multiples of 64 items so the bitmap u64
words of consecutive shards concatenate without bit shifting.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int, align: int = 64) -> tuple[int, int]:
    """Contiguous [start, end) of n items for `rank`, boundaries on multiples of `align`."""
    if world <= 1:
        return 0, n
    blocks = (n + align - 1) // align
    per, extra = divmod(blocks, world)
    b0 = rank * per + min(rank, extra)
    b1 = b0 + per + (1 if rank < extra else 0)
    return min(n, b0 * align), min(n, b1 * align)


def gather_bitmaps(local_words: torch.Tensor, n_total: int, world: int,
                   group=None) -> torch.Tensor | None:
    """all_gather the u64 bitmap words of every rank's shard (int64 tensor; on the device
    for RCCL, which gathers device memory over xGMI directly; staged through host memory
    for gloo). Returns the concatenated bitmap as uint8 (ceil(n_total/8) bytes) on every
    rank, on local_words' device."""
    if world <= 1:
        return local_words.view(torch.uint8)[: (n_total + 7) // 8]
    return _gather_words(local_words, n_total, world, group)


def _gather_words(local_words: torch.Tensor, n_total: int, world: int,
                  group=None) -> torch.Tensor:
    """The all_gather of gather_bitmaps (also with world 1: tests/test_gpu_distributed.py
    runs it on a one-rank RCCL group)."""
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    max_words = max((e - s + 63) // 64 for s, e in sizes)
    comm_dev = local_words.device
    if dist.get_backend(group) == "gloo" and comm_dev.type != "cpu":
        comm_dev = torch.device("cpu")
    buf = torch.zeros(max_words, dtype=torch.int64, device=comm_dev)
    buf[: local_words.numel()] = local_words
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    parts = [o[: (e - s + 63) // 64] for o, (s, e) in zip(out, sizes)]
    return torch.cat(parts).to(local_words.device).view(torch.uint8)[: (n_total + 7) // 8]
