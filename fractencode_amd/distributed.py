"""Multi-GPU sharding of the range search (one process per GPU, RCCL over xGMI).

Range blocks are independent: every rank holds the full frame and
domain pool, searches a contiguous slice of the ranges, and the 64-byte winner
records (encode_item_t) are all-gathered — the path's only exchange step.
The same functions run on the ``gloo`` backend with CPU tensors (tests).
"""
from __future__ import annotations

import numpy as np

RECORD_BYTES = 64


def shard_bounds(n_items: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous equal-capacity shard [start, stop) of rank (the last may be shorter)."""
    per = (n_items + world - 1) // world if world > 0 else n_items
    start = min(n_items, rank * per)
    return start, min(n_items, start + per)


def shard_capacity(n_items: int, world: int) -> int:
    return (n_items + world - 1) // world


def gather_records(local, n_items: int, world: int, group=None):
    """All-gathers per-rank record buffers (torch uint8 tensors of shard_capacity*64 bytes,
    on the device for nccl or on the CPU for gloo) and returns the n_items*64 leading bytes
    in global range order (rank r's shard first for rank 0, ...)."""
    import torch
    import torch.distributed as dist

    cap = shard_capacity(n_items, world) * RECORD_BYTES
    assert local.numel() == cap and local.dtype == torch.uint8
    if world == 1:
        return local[: n_items * RECORD_BYTES]
    out = torch.empty(world * cap, dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    return out[: n_items * RECORD_BYTES]


def records_from_bytes(buf) -> np.ndarray:
    from . import ENCODE_ITEM

    a = buf.cpu().numpy() if hasattr(buf, "cpu") else np.asarray(buf)
    return np.frombuffer(a.tobytes(), dtype=ENCODE_ITEM)


def encode_sharded(engine, ranges: np.ndarray, rank: int, world: int, device=None, group=None):
    """Search this rank's shard of `ranges` on `engine` (frame and domains already set)
    and all-gather every rank's records; returns the full encode_item_t array on every rank."""
    import torch

    start, stop = shard_bounds(len(ranges), world, rank)
    cap = shard_capacity(len(ranges), world) * RECORD_BYTES
    local = torch.zeros(cap, dtype=torch.uint8, device=device)
    if local.is_cuda:
        torch.cuda.synchronize(local.device)  # the zero-fill must land before the engine's copy
    engine.set_ranges(ranges[start:stop])
    engine.run()
    if local.is_cuda:  # nccl: records stay on the device (frac_copy_results_device)
        if stop > start:
            engine.copy_results_device(local.data_ptr())
        engine.sync()
    elif stop > start:  # gloo: host records
        out, _ = engine.fetch()
        local[: (stop - start) * RECORD_BYTES] = torch.from_numpy(np.ascontiguousarray(out).view(np.uint8))
    return records_from_bytes(gather_records(local, len(ranges), world, group))
