"""N>1 path on CPU: world-size-2 `gloo` ranks shard the ranges, search their slice and
all-gather the 32-byte (domain, transform, s, o, rms) tuples (fractencode_amd.distributed).  The per-rank search
here is the oracle behind the engine interface (no GPU in this container); on the
GPU box bench.py runs the same functions over RCCL with the HIP engine."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from fractencode_amd.distributed import shard_bounds, shard_capacity


def test_shard_bounds_cover_all_items_once():
    for n in (0, 1, 7, 64, 1000, 262144):
        for world in (1, 2, 3, 4, 8):
            seen = []
            for r in range(world):
                a, b = shard_bounds(n, world, r)
                assert 0 <= a <= b <= n and b - a <= shard_capacity(n, world)
                seen.extend(range(a, b))
            assert seen == list(range(n))


class OracleEngine:
    """Engine-interface stand-in (CPU): set_ranges / run / fetch_tuples / sync."""

    def __init__(self, plane, doms):
        from oracle import oracle as O
        self.O, self.plane, self.doms = O, plane, doms
        self.index = {(int(d["x"]), int(d["y"])): i for i, d in enumerate(doms)}

    def set_ranges(self, r):
        self.r = r

    def run(self):
        import fractencode_amd as F
        out, _, _ = self.O.estimate(self.plane, self.doms, self.r.astype(self.O.ITEM_DTYPE), threads=2)
        rec = np.zeros(len(out), dtype=F.ENCODE_ITEM)
        rec["x"], rec["y"], rec["w"], rec["h"] = self.r["x"], self.r["y"], self.r["w"], self.r["h"]
        rec["distance"], rec["contrast"], rec["brightness"] = out["dist"], out["s"], out["o"]
        rec["transform"], rec["dx"], rec["dy"], rec["sw"], rec["sh"] = out["t"], out["dx"], out["dy"], out["dw"], out["dh"]
        self.rec = rec

    def fetch_tuples(self):
        import fractencode_amd as F
        t = np.zeros(len(self.rec), dtype=F.TUPLE)
        for k in ("transform", "contrast", "brightness", "distance"):
            t[k] = self.rec[k]
        t["domain"] = [self.index[(int(x), int(y))] if w else F.NO_DOMAIN
                       for x, y, w in zip(self.rec["dx"], self.rec["dy"], self.rec["sw"])]
        return t

    def sync(self):
        pass


def _worker(rank, world, port, path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist

    import fractencode_amd as F
    from fractencode_amd.distributed import encode_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(3)
    plane = rng.integers(0, 256, (64, 96), dtype=np.uint8)
    doms = F.create_uniform_grid(96, 64, 16, 8)
    rngs = F.create_uniform_grid(96, 64, 8, 8)[:93]  # ragged: not a multiple of the world size
    full = encode_sharded(OracleEngine(plane, doms), rngs, doms, rank, world)
    if rank == 0:
        np.save(path, full)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_search_matches_single_rank(tmp_path, oracle, world):
    import fractencode_amd as F
    path = str(tmp_path / "full.npy")
    mp.spawn(_worker, args=(world, _free_port(), path), nprocs=world, join=True)
    full = np.load(path)
    rng = np.random.default_rng(3)
    plane = rng.integers(0, 256, (64, 96), dtype=np.uint8)
    want, _, _ = oracle.estimate(plane, oracle.uniform_grid(96, 64, 16, 8), oracle.uniform_grid(96, 64, 8, 8)[:93])
    assert full.dtype == F.ENCODE_ITEM and len(full) == 93
    np.testing.assert_array_equal(full["dx"], want["dx"])
    np.testing.assert_array_equal(full["dy"], want["dy"])
    np.testing.assert_array_equal(full["transform"], want["t"])
    np.testing.assert_array_equal(full["distance"], want["dist"])
    np.testing.assert_array_equal(full["contrast"], want["s"])
    np.testing.assert_array_equal(full["brightness"], want["o"])


def _gpu_worker(rank, world, port, path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist

    import fractencode_amd as F
    from fractencode_amd.distributed import encode_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    y = np.fromfile(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lenna_y.u8"),
                    dtype=np.uint8).reshape(512, 512)
    doms = F.create_uniform_grid(512, 512, 16, 8)
    with F.Engine(0, 4) as e:  # every rank's engine on GPU 0 (one-GPU box)
        e.set_frame(y)
        e.set_domains(doms)
        full = encode_sharded(e, F.create_uniform_grid(512, 512, 8, 8), doms, rank, world)
    if rank == 0:
        np.save(path, full)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_with_hip_engines_match_reference(tmp_path):
    """world-size-2 ranks, each a real HIP engine, shard Lenna's ranges; the gathered records
    equal the reference golden (lenna_t4)."""
    from golden_util import FIELDS, golden

    path = str(tmp_path / "full.npy")
    mp.spawn(_gpu_worker, args=(2, _free_port(), path), nprocs=2, join=True)
    full = np.load(path)
    rec, _ = golden("lenna_t4")
    got = {"x": full["x"], "y": full["y"], "dx": full["dx"], "dy": full["dy"], "dw": full["sw"], "dh": full["sh"],
           "t": full["transform"], "dist": full["distance"], "s": full["contrast"], "o": full["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(got[k], rec[k], err_msg=k)
