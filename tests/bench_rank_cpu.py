"""One rank of bench.py's N > 1 orchestration on the CPU (test infrastructure, launched by
tests/test_bench_ranks.py through bench.launch_ranks → torch.distributed.run, or run directly for
world size 1): the oracle stand-in engine behind bench.FrameStep, `gloo` in place of RCCL, the
same timed() bracket and headline_fields() as the GPU headline (the frame in row stripes assembled by
the all-gather when N > 1; the tuples into the node's shared buffer, or with BENCH_TUPLES=gather the
all-gather).  Rank 0 writes the line, every rank's own time and the gathered tuples to OUT.
usage: [BENCH_TUPLES=node|gather] python tests/bench_rank_cpu.py OUT STEPS [FAIL_RANK]"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
import fractencode_amd as F  # noqa: E402
from fractencode_amd.distributed import shard_plan  # noqa: E402
from oracle_engine import OracleEngine  # noqa: E402

out, steps = sys.argv[1], int(sys.argv[2])
fail_rank = int(sys.argv[3]) if len(sys.argv) > 3 else -1
world = int(os.environ.get("WORLD_SIZE", "1"))
rank = int(os.environ.get("RANK", "0"))
if world > 1:
    dist.init_process_group("gloo")
if rank == fail_rank:
    sys.exit(3)  # a failing rank: the launcher must report it
rng = np.random.default_rng(3)
plane = rng.integers(0, 256, (64, 96), dtype=np.uint8)
doms = F.create_uniform_grid(96, 64, 16, 8)
rngs = F.create_uniform_grid(96, 64, 8, 8)[:93]  # ragged: not a multiple of the world size
plan = shard_plan(len(rngs), world)
a, b = plan[rank]
eng = OracleEngine(np.zeros_like(plane), doms)
eng.set_ranges(rngs[a:b])
dev = torch.device("cpu")
node = None
if world > 1 and os.environ.get("BENCH_TUPLES", "node") == "node":
    from fractencode_amd.distributed import NodeTuples

    node = NodeTuples(plan, rank, dev)
step = bench.FrameStep(eng, plane, plan, rank, dev, node_tuples=node)
step()  # warmup
mine, mx = bench.timed(step, steps, world, dev)
line = bench.headline_fields(len(rngs), world, steps, 1, mx)
own = eng.fetch_tuples().tobytes() if b > a else b""
every = [None] * world
if world > 1:
    dist.all_gather_object(every, (rank, mine, step.own_slice_ok(own)))
else:
    every = [(0, mine, step.own_slice_ok(own))]
if rank == 0:
    gathered = step.tuples_bytes()
    json.dump({"line": line, "ranks": every, "digest": bench.digest(gathered), "tuples": gathered.hex(),
               "stripes": step.stripes, "node": node is not None}, open(out, "w"))
if world > 1:
    dist.barrier()
    if node is not None:
        del step
        node.close()
    dist.destroy_process_group()
