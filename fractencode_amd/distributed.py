"""Multi-GPU sharding of the range search (one process per GPU, RCCL over xGMI).

Range blocks are independent: every rank holds the full frame and
domain pool, searches a contiguous slice of the ranges, and the winners are
all-gathered as the 32-byte (domain, transform, s, o, rms) tuples north_star names
(frac_tuple) — the path's only exchange step.  Every rank knows the range and domain
grids, so the 64-byte encode_item_t records are rebuilt locally from the tuples
(records_from_tuples).  The same functions run on the ``gloo`` backend with CPU
tensors (tests).

Shards.  Without the classifier every range meets every domain, so equal-count slices
are equal-cost.  With the classifier a range only meets the domains of its own category
(Classifier2::compare, encode/Classifier2.cpp:70-81), so its cost is the size of its
bucket: the slices are cut at equal fractions of the cost prefix sum, and
the all-gather pads every shard to the largest one.
"""
from __future__ import annotations

import numpy as np

TUPLE_BYTES = 32
N_BUCKETS = 7  # category + 1: −1..5


def shard_bounds(n_items: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous equal-capacity shard [start, stop) of rank (the last may be shorter)."""
    per = (n_items + world - 1) // world if world > 0 else n_items
    start = min(n_items, rank * per)
    return start, min(n_items, start + per)


def shard_capacity(n_items: int, world: int) -> int:
    return (n_items + world - 1) // world


def range_costs(ranges: np.ndarray, domains: np.ndarray) -> np.ndarray:
    """Per-range search cost with the classifier on: the number of domains sharing the range's
    category (both grids classified, categories −1..5), plus one for the range's own fixed work."""
    cnt = np.bincount(np.asarray(domains["category"], np.int64) + 1, minlength=N_BUCKETS)
    return cnt[np.asarray(ranges["category"], np.int64) + 1].astype(np.int64) + 1


def shard_plan(n_items: int, world: int, costs: np.ndarray | None = None) -> list[tuple[int, int]]:
    """[start, stop) of every rank: equal counts (costs None), else contiguous slices cut where the
    cost prefix sum crosses k/world of the total (each rank's cost is within one range's cost of
    the mean)."""
    if costs is None:
        return [shard_bounds(n_items, world, r) for r in range(world)]
    costs = np.asarray(costs, np.int64)
    assert len(costs) == n_items
    csum = np.concatenate([[0], np.cumsum(costs)])
    total = int(csum[-1])
    cuts = [0]
    for k in range(1, world):
        # first boundary whose prefix reaches k/world of the total (ties to the nearer side)
        goal = total * k / world
        i = int(np.searchsorted(csum, goal, side="left"))
        if 0 < i <= n_items and goal - csum[i - 1] < csum[i] - goal:
            i -= 1
        cuts.append(min(max(i, cuts[-1]), n_items))
    cuts.append(n_items)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def plan_capacity(plan: list[tuple[int, int]]) -> int:
    return max((b - a for a, b in plan), default=0)


def gather_tuples(local, plan: list[tuple[int, int]], group=None):
    """All-gathers per-rank tuple buffers (torch uint8 tensors of plan_capacity·32 bytes, on the
    device for nccl or on the CPU for gloo) and returns the tuples of every rank's shard in
    global range order (rank 0's shard first, ...).  Runs the collective whenever a process group
    is initialised, world size 1 included."""
    import torch
    import torch.distributed as dist

    world = len(plan)
    cap = plan_capacity(plan) * TUPLE_BYTES
    assert local.numel() == cap and local.dtype == torch.uint8
    if world == 1 and not dist.is_initialized():
        return local[: (plan[0][1] - plan[0][0]) * TUPLE_BYTES]
    assert dist.get_world_size(group) == world
    out = torch.empty(world * cap, dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    if all(b - a == plan_capacity(plan) for a, b in plan[:-1]):  # equal shards: one view
        n = plan[-1][1]
        return out[: n * TUPLE_BYTES]
    parts = [out[r * cap: r * cap + (b - a) * TUPLE_BYTES] for r, (a, b) in enumerate(plan)]
    return torch.cat(parts)


class FrameStripes:
    """The frame onto every rank without N full uploads: rank r copies only rows [r·rows, (r+1)·rows) of the
    caller's host plane across its own PCIe link (rows = ⌈H / world⌉; the last stripe is padded) and one
    all_gather_into_tensor assembles the whole plane on every rank — over xGMI with RCCL, or on the CPU with
    gloo.  `frame`: a [H, W] uint8 torch tensor (pinned for an asynchronous copy) or numpy array; calling
    the object returns the [H, W] plane on `device` (a view of an internal buffer, valid until the next
    call), ordered on torch's current stream."""

    def __init__(self, frame, world: int, rank: int, device, group=None):
        import torch

        ft = frame if isinstance(frame, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(frame))
        self.H, W = int(ft.shape[0]), int(ft.shape[1])
        rows = -(-self.H // world)
        r0, r1 = min(self.H, rank * rows), min(self.H, (rank + 1) * rows)
        self.n = r1 - r0
        self.host = ft[r0:r1]  # a view: pinned when the caller's plane is
        self.stripe = torch.zeros((rows, W), dtype=torch.uint8, device=device)
        self.full = torch.empty((world * rows, W), dtype=torch.uint8, device=device)
        self.group = group

    def __call__(self, mark=None):
        """`mark` (optional): called with "frame_h2d" after the stripe's copy is enqueued and with
        "frame_allgather" after the all-gather (a phase clock's marks)."""
        import torch.distributed as dist

        if self.n:
            self.stripe[: self.n].copy_(self.host, non_blocking=True)
        if mark:
            mark("frame_h2d")
        dist.all_gather_into_tensor(self.full, self.stripe, group=self.group)
        if mark:
            mark("frame_allgather")
        return self.full[: self.H]


def _hip_runtime():
    """The process's HIP runtime (the one PyTorch loaded: dlopen by soname returns it)."""
    import ctypes as C

    import torch  # noqa: F401  (loads the runtime first)

    L = C.CDLL("libamdhip64.so.7")
    L.hipHostRegister.restype = C.c_int
    L.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
    L.hipHostUnregister.restype = C.c_int
    L.hipHostUnregister.argtypes = [C.c_void_p]
    L.hipHostGetDevicePointer.restype = C.c_int
    L.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]
    return L


class NodeTuples:
    """One host buffer of every range's 32-byte tuple, shared by all ranks of one node: rank 0 creates a
    file in /dev/shm, every rank maps it (MAP_SHARED) and, on a GPU, registers the mapping with HIP, so a
    rank's resolve writes its shard's tuples (frac_set_tuple_sink at `sink_ptr()`) straight into the one
    output every rank sees — no tuple all-gather and no N full downloads, each PCIe link carries only its
    own shard's tuples.  The file is unlinked once every rank holds its mapping (nothing is left behind
    however the job ends).  Only for ranks that share one host (the caller checks); with ranks on several
    hosts the all-gather path (gather_tuples) stays."""

    def __init__(self, plan: list[tuple[int, int]], rank: int, device, group=None):
        import mmap
        import os
        import secrets

        import torch
        import torch.distributed as dist

        self.plan, self.rank, self.device = plan, rank, device
        self.n = plan[-1][1] if plan else 0
        self.bytes = max(1, self.n * TUPLE_BYTES)
        size = -(-self.bytes // mmap.PAGESIZE) * mmap.PAGESIZE
        name = [f"/dev/shm/fracenc_tuples_{os.getpid()}_{secrets.token_hex(6)}" if rank == 0 else None]
        if rank == 0:
            try:
                fd = os.open(name[0], os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
                try:
                    os.ftruncate(fd, size)
                finally:
                    os.close(fd)
            except OSError as exc:  # every rank learns of it from the broadcast, none waits forever
                try:
                    os.unlink(name[0])
                except OSError:
                    pass
                name = [f"error: {exc}"]
        dist.broadcast_object_list(name, src=0, group=group)
        if name[0].startswith("error: "):
            raise RuntimeError(f"node tuple buffer: rank 0 could not create its file ({name[0][7:]})")
        try:
            fd = os.open(name[0], os.O_RDWR)
            try:
                self._mm = mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
            finally:
                os.close(fd)
        finally:
            dist.barrier(group=group)  # every rank mapped (or failed) before the name goes
            if rank == 0:
                os.unlink(name[0])
        self.host = torch.frombuffer(self._mm, dtype=torch.uint8)[: self.n * TUPLE_BYTES]
        self._addr = self.host.data_ptr()
        self._size = size
        self._dptr = None
        if device.type == "cuda":
            import ctypes as C

            hip = _hip_runtime()
            err = hip.hipHostRegister(self._addr, size, 0x1 | 0x2)  # portable | mapped
            if err:
                raise RuntimeError(f"hipHostRegister of the node tuple buffer failed ({err})")
            p = C.c_void_p()
            err = hip.hipHostGetDevicePointer(C.byref(p), self._addr, 0)
            if err:
                hip.hipHostUnregister(self._addr)
                raise RuntimeError(f"hipHostGetDevicePointer failed ({err})")
            self._hip, self._dptr = hip, p.value

    def sink_ptr(self) -> int:
        """The device address of this rank's shard within the buffer (the tuple sink)."""
        assert self._dptr is not None, "a GPU rank's buffer"
        return self._dptr + self.plan[self.rank][0] * TUPLE_BYTES

    def put(self, tuples: bytes) -> None:
        """This rank's shard's tuples written by the host (an engine that hands back host tuples)."""
        a, b = self.plan[self.rank]
        assert len(tuples) == (b - a) * TUPLE_BYTES
        self.host[a * TUPLE_BYTES: b * TUPLE_BYTES] = torch_bytes(tuples)

    def close(self) -> None:
        if self._dptr is not None:
            self._hip.hipHostUnregister(self._addr)
            self._dptr = None
        self.host = None
        try:
            self._mm.close()
        except BufferError:  # a caller still holds a view: the mapping goes with the process
            pass


def torch_bytes(b: bytes):
    import torch

    return torch.frombuffer(bytearray(b), dtype=torch.uint8) if b else torch.empty(0, dtype=torch.uint8)


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


def classified_grids(engine, ranges: np.ndarray, domains: np.ndarray):
    """Copies of both grids with every −1 category computed on the engine's device planes (the
    same categories the search uses), so every rank derives the same cost-balanced plan."""
    r, d = ranges, domains
    if (np.asarray(d["category"]) == -1).any():
        d = engine.classify(d, target_plane=False)
    if (np.asarray(r["category"]) == -1).any():
        r = engine.classify(r, target_plane=True)
    return r, d


def encode_sharded(engine, ranges: np.ndarray, domains: np.ndarray, rank: int, world: int, device=None,
                   group=None, use_classifier: bool | None = None) -> np.ndarray:
    """Search this rank's shard of `ranges` on `engine` (frame and `domains` already set), all-gather
    every rank's tuples and return the full encode_item_t array on every rank.  With the
    classifier (engine parameter, or `use_classifier`) the shards are cost-balanced."""
    import torch

    if use_classifier is None:
        use_classifier = bool(getattr(getattr(engine, "_p", None), "use_classifier", 0))
    if use_classifier and world > 1:
        cr, cd = classified_grids(engine, ranges, domains)
        plan = shard_plan(len(ranges), world, range_costs(cr, cd))
    else:
        plan = shard_plan(len(ranges), world)
    start, stop = plan[rank]
    cap = plan_capacity(plan) * TUPLE_BYTES
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
    return records_from_tuples(tuples_from_bytes(gather_tuples(local, plan, group)), ranges, domains)
