"""Multi-GPU sharding of the range search (one process per GPU, RCCL over xGMI).

Range blocks are independent: every rank holds the full frame and
domain pool, searches a contiguous slice of the ranges, and the winners are
all-gathered as the 32-byte (domain, transform, s, o, rms) tuples north_star names
(frac_tuple) — the path's only exchange step.  Every rank knows the range and domain
grids, so the 64-byte encode_item_t records are rebuilt locally from the tuples
(records_from_tuples).  The same functions run on the ``gloo`` backend with CPU
tensors (tests).
"""
from __future__ import annotations

import numpy as np

TUPLE_BYTES = 32


def shard_bounds(n_items: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous equal-capacity shard [start, stop) of rank (the last may be shorter)."""
    per = (n_items + world - 1) // world if world > 0 else n_items
    start = min(n_items, rank * per)
    return start, min(n_items, start + per)


def shard_capacity(n_items: int, world: int) -> int:
    return (n_items + world - 1) // world


def gather_tuples(local, n_items: int, world: int, group=None):
    """All-gathers per-rank tuple buffers (torch uint8 tensors of shard_capacity*32 bytes, on
    the device for nccl or on the CPU for gloo) and returns the n_items*32 leading bytes in
    global range order (rank 0's shard first, ...)."""
    import torch
    import torch.distributed as dist

    cap = shard_capacity(n_items, world) * TUPLE_BYTES
    assert local.numel() == cap and local.dtype == torch.uint8
    if world == 1:
        return local[: n_items * TUPLE_BYTES]
    out = torch.empty(world * cap, dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    return out[: n_items * TUPLE_BYTES]


def tuples_from_bytes(buf) -> np.ndarray:
    from . import TUPLE

    a = buf.cpu().numpy() if hasattr(buf, "cpu") else np.asarray(buf)
    return np.frombuffer(a.tobytes(), dtype=TUPLE)


def records_from_tuples(tuples: np.ndarray, ranges: np.ndarray, domains: np.ndarray) -> np.ndarray:
    """encode_item_t records (fractencode_amd.ENCODE_ITEM) from gathered tuples: the range
    geometry from `ranges`, the winning domain's origin and size from `domains` (the list
    given to set_domains); a tuple without a domain is the reference's default record."""
    from . import ENCODE_ITEM, NO_DOMAIN

    assert len(tuples) == len(ranges)
    rec = np.zeros(len(tuples), dtype=ENCODE_ITEM)
    for k in ("x", "y", "w", "h"):
        rec[k] = ranges[k]
    for k in ("distance", "contrast", "brightness", "transform"):
        rec[k] = tuples[k]
    has = tuples["domain"] != NO_DOMAIN
    d = domains[tuples["domain"][has].astype(np.int64)]
    rec["dx"][has], rec["dy"][has], rec["sw"][has], rec["sh"][has] = d["x"], d["y"], d["w"], d["h"]
    return rec


def encode_sharded(engine, ranges: np.ndarray, domains: np.ndarray, rank: int, world: int, device=None,
                   group=None) -> np.ndarray:
    """Search this rank's shard of `ranges` on `engine` (frame and `domains` already set), all-gather
    every rank's tuples and return the full encode_item_t array on every rank."""
    import torch

    start, stop = shard_bounds(len(ranges), world, rank)
    cap = shard_capacity(len(ranges), world) * TUPLE_BYTES
    local = torch.zeros(cap, dtype=torch.uint8, device=device)
    if local.is_cuda:
        torch.cuda.synchronize(local.device)  # the zero-fill must land before the engine's pack
    engine.set_ranges(ranges[start:stop])
    engine.run()
    if local.is_cuda:  # nccl: tuples packed on the device (frac_copy_tuples_device)
        if stop > start:
            engine.copy_tuples_device(local.data_ptr())
        engine.sync()
    elif stop > start:  # gloo: host tuples
        t = engine.fetch_tuples()
        local[: (stop - start) * TUPLE_BYTES] = torch.from_numpy(np.ascontiguousarray(t).view(np.uint8))
    return records_from_tuples(tuples_from_bytes(gather_tuples(local, len(ranges), world, group)), ranges, domains)
