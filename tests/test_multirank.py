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

from fractencode_amd.distributed import plan_capacity, range_costs, shard_bounds, shard_capacity, shard_plan
from oracle_engine import OracleEngine


def test_shard_bounds_cover_all_items_once():
    for n in (0, 1, 7, 64, 1000, 262144):
        for world in (1, 2, 3, 4, 8):
            seen = []
            for r in range(world):
                a, b = shard_bounds(n, world, r)
                assert 0 <= a <= b <= n and b - a <= shard_capacity(n, world)
                seen.extend(range(a, b))
            assert seen == list(range(n))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_cost_plan_balances_classifier_buckets(world):
    # with the classifier a range costs |bucket(category)|; contiguous shards cut on
    # the cost prefix sum stay within one range's cost of the mean, and cover every range once
    rng = np.random.default_rng(11)
    n = 5000
    cost = rng.choice([1, 50, 4000, 20000], size=n, p=[0.2, 0.3, 0.3, 0.2]).astype(np.int64)
    plan = shard_plan(n, world, cost)
    assert plan[0][0] == 0 and plan[-1][1] == n
    assert all(plan[r][1] == plan[r + 1][0] for r in range(world - 1))
    per = [int(cost[a:b].sum()) for a, b in plan]
    assert max(per) - cost.sum() / world <= cost.max()
    eq = [int(cost[a:b].sum()) for a, b in shard_plan(n, world)]
    assert max(per) <= max(eq)
    assert plan_capacity(plan) >= max(b - a for a, b in plan)


def test_range_costs_are_bucket_sizes():
    import fractencode_amd as F
    d = np.zeros(10, dtype=F.GRID_ITEM)
    d["category"] = [-1, 0, 0, 1, 1, 1, 2, 5, 5, 5]
    r = np.zeros(4, dtype=F.GRID_ITEM)
    r["category"] = [0, 1, 3, -1]
    np.testing.assert_array_equal(range_costs(r, d), [3, 4, 1, 2])


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


def _cls_worker(rank, world, port, path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist

    import fractencode_amd as F
    from fractencode_amd.distributed import encode_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(5)
    plane = rng.integers(0, 256, (64, 96), dtype=np.uint8)
    doms = F.preclassify(plane, F.create_uniform_grid(96, 64, 16, 8))
    rngs = F.preclassify(plane, F.create_uniform_grid(96, 64, 8, 8))
    full = encode_sharded(OracleEngine(plane, doms, True), rngs, doms, rank, world, use_classifier=True)
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


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_sharded_search_matches_single_rank(tmp_path, oracle, world):
    # the world sizes the driver's scaling run uses (1/2/4/8 GPUs), with a ragged range count
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


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_cost_balanced_classifier_shards_match_single_rank(tmp_path, oracle, world):
    """Classifier on: cost-balanced (unequal-count) shards, padded all-gather, same records as one
    rank (the oracle), at the driver's world sizes."""
    import fractencode_amd as F
    path = str(tmp_path / "full.npy")
    mp.spawn(_cls_worker, args=(world, _free_port(), path), nprocs=world, join=True)
    full = np.load(path)
    rng = np.random.default_rng(5)
    plane = rng.integers(0, 256, (64, 96), dtype=np.uint8)
    doms = F.preclassify(plane, F.create_uniform_grid(96, 64, 16, 8))
    rngs = F.preclassify(plane, F.create_uniform_grid(96, 64, 8, 8))
    plan = shard_plan(len(rngs), world, range_costs(rngs, doms))
    assert plan != shard_plan(len(rngs), world)  # the plan is not the equal split
    want, _, _ = oracle.estimate(plane, doms.astype(oracle.ITEM_DTYPE), rngs.astype(oracle.ITEM_DTYPE),
                                 use_classifier=True)
    for a, b in (("dx", "dx"), ("dy", "dy"), ("transform", "t"), ("distance", "dist"), ("contrast", "s"),
                 ("brightness", "o")):
        np.testing.assert_array_equal(full[a], want[b], err_msg=a)


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


def _nccl_worker(rank, world, port, path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist

    import fractencode_amd as F
    from fractencode_amd.distributed import encode_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    y = np.fromfile(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lenna_y.u8"),
                    dtype=np.uint8).reshape(512, 512)
    doms = F.create_uniform_grid(512, 512, 16, 8)
    with F.Engine(rank, 4) as e:
        e.set_frame(y)
        e.set_domains(doms)
        # device tuples (frac_copy_tuples_device) through a real RCCL all_gather_into_tensor
        full = encode_sharded(e, F.create_uniform_grid(512, 512, 8, 8), doms, rank, world, device=dev)
    if rank == 0:
        np.save(path, full)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_nccl_device_tuples_world1_match_reference(tmp_path):
    """The nccl path bench.py uses at N > 1 — tuples packed on the device, all-gathered by RCCL —
    run at world size 1 (one GPU per box; the collective still runs), against lenna_t4."""
    from golden_util import FIELDS, golden

    path = str(tmp_path / "full.npy")
    mp.spawn(_nccl_worker, args=(1, _free_port(), path), nprocs=1, join=True)
    full = np.load(path)
    rec, _ = golden("lenna_t4")
    got = {"x": full["x"], "y": full["y"], "dx": full["dx"], "dy": full["dy"], "dw": full["sw"], "dh": full["sh"],
           "t": full["transform"], "dist": full["distance"], "s": full["contrast"], "o": full["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(got[k], rec[k], err_msg=k)


def _stripes_worker(rank, world, port, path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist

    import bench
    import fractencode_amd as F
    from fractencode_amd.distributed import records_from_tuples, shard_plan

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    y = np.fromfile(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lenna_y.u8"),
                    dtype=np.uint8).reshape(512, 512)
    doms = F.create_uniform_grid(512, 512, 16, 8)
    rngs = F.create_uniform_grid(512, 512, 8, 8)
    plan = shard_plan(len(rngs), world)
    a, b = plan[rank]
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    h = torch.from_numpy(y).pin_memory()
    with F.Engine(rank, 4) as e:
        e.set_stream(stream.cuda_stream)
        e.set_frame(np.zeros_like(y))  # the step's stripes and all-gather bring the real frame
        e.set_domains(doms)
        e.set_ranges(rngs[a:b])
        step = bench.FrameStep(e, h, plan, rank, dev, stripes=True)
        step()
        torch.cuda.synchronize(dev)
        full = records_from_tuples(np.frombuffer(step.tuples_bytes(), dtype=F.TUPLE), rngs, doms)
    if rank == 0:
        np.save(path, full)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_nccl_frame_stripes_world1_match_reference(tmp_path):
    """bench.FrameStep with the frame in row stripes assembled by an RCCL all-gather (the N > 1 upload), run at
    world size 1 on the device's nccl group (the collective still runs), against lenna_t4."""
    from golden_util import FIELDS, golden

    path = str(tmp_path / "full.npy")
    mp.spawn(_stripes_worker, args=(1, _free_port(), path), nprocs=1, join=True)
    full = np.load(path)
    rec, _ = golden("lenna_t4")
    got = {"x": full["x"], "y": full["y"], "dx": full["dx"], "dy": full["dy"], "dw": full["sw"], "dh": full["sh"],
           "t": full["transform"], "dist": full["distance"], "s": full["contrast"], "o": full["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(got[k], rec[k], err_msg=k)


def _node_worker(rank, world, port, path, backend):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist

    import bench
    import fractencode_amd as F
    from fractencode_amd.distributed import NodeTuples, records_from_tuples, shard_plan

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)  # one-GPU box: with gloo every rank's engine is on GPU 0
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    y = np.fromfile(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lenna_y.u8"),
                    dtype=np.uint8).reshape(512, 512)
    doms = F.create_uniform_grid(512, 512, 16, 8)
    rngs = F.create_uniform_grid(512, 512, 8, 8)
    plan = shard_plan(len(rngs), world)
    a, b = plan[rank]
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    h = torch.from_numpy(y).pin_memory()
    node = NodeTuples(plan, rank, dev)
    with F.Engine(0, 4) as e:
        e.set_stream(stream.cuda_stream)
        e.set_frame(np.zeros_like(y))  # the step brings the real frame
        e.set_domains(doms)
        e.set_ranges(rngs[a:b])
        step = bench.FrameStep(e, h, plan, rank, dev, stripes=backend == "nccl", node_tuples=node)
        for _ in range(3):  # the buffer is rewritten by every frame
            step()
        torch.cuda.synchronize(dev)
        dist.barrier()
        full = records_from_tuples(np.frombuffer(step.tuples_bytes(), dtype=F.TUPLE), rngs, doms)
        own_ok = step.own_slice_ok(e.fetch_tuples().tobytes())
    if rank == 0:
        np.save(path, full)
    assert own_ok
    dist.barrier()
    del step
    node.close()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("backend,world", [("nccl", 1), ("gloo", 2)])
def test_node_tuple_buffer_match_reference(tmp_path, backend, world):
    """bench.FrameStep at N > 1 on one host: every rank's resolve writes its shard's tuples through the sink
    into the node's one shared, HIP-registered host buffer (distributed.NodeTuples) — at world 1 on the nccl
    group (stripes, the per-frame RCCL token), and at world 2 over gloo with both ranks' engines on GPU 0 (two
    processes writing into one mapping) — against lenna_t4."""
    from golden_util import FIELDS, golden

    path = str(tmp_path / "full.npy")
    mp.spawn(_node_worker, args=(world, _free_port(), path, backend), nprocs=world, join=True)
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("fracenc_tuples_")]
    full = np.load(path)
    rec, _ = golden("lenna_t4")
    got = {"x": full["x"], "y": full["y"], "dx": full["dx"], "dy": full["dy"], "dw": full["sw"], "dh": full["sh"],
           "t": full["transform"], "dist": full["distance"], "s": full["contrast"], "o": full["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(got[k], rec[k], err_msg=k)


def _gpu_cls_worker(rank, world, port, path):
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
    doms = F.create_uniform_grid(512, 512, 16, 8)  # categories −1: classified on the device
    with F.Engine(0, 4, True) as e:
        e.set_frame(y)
        e.set_domains(doms)
        full = encode_sharded(e, F.create_uniform_grid(512, 512, 8, 8), doms, rank, world)
    if rank == 0:
        np.save(path, full)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_cost_balanced_classifier_match_reference(tmp_path):
    """Classifier on (lenna_cls): two ranks cut the ranges at equal bucket cost (unequal counts),
    HIP engines, padded all-gather; records equal the reference golden."""
    from golden_util import FIELDS, golden

    path = str(tmp_path / "full.npy")
    mp.spawn(_gpu_cls_worker, args=(2, _free_port(), path), nprocs=2, join=True)
    full = np.load(path)
    rec, _ = golden("lenna_cls")
    got = {"x": full["x"], "y": full["y"], "dx": full["dx"], "dy": full["dy"], "dw": full["sw"], "dh": full["sh"],
           "t": full["transform"], "dist": full["distance"], "s": full["contrast"], "o": full["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(got[k], rec[k], err_msg=k)
