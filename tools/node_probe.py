"""The N > 1 tuple paths of bench.FrameStep on one GPU (rank 0 of an nccl group of world size 1, the C3 frame):
`gather` (tuples into the all-gather buffer + RCCL all-gather + the gathered tuples D2H) against `node` (the
resolve writes the tuples into the node's shared, HIP-registered host buffer + a 4-byte RCCL all-reduce per
frame), interleaved, frame stripes on in both.  At world 1 both move the whole frame's 8.4 MB of tuples; at
N ranks the gather path still downloads all of them on every rank while the node path writes 1/N per rank.
usage: python tools/node_probe.py OUT.jsonl [ROUNDS] [STEPS]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
import fractencode_amd as F  # noqa: E402
from fractencode_amd.distributed import NodeTuples, shard_plan  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402


def main():
    out = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    S = 4096
    frame = value_noise(S, S, 1234)
    doms = F.create_uniform_grid(S, S, 16, 8)
    rngs = F.create_uniform_grid(S, S, 8, 8)
    plan = shard_plan(len(rngs), 1)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    h = torch.from_numpy(frame).pin_memory()
    node = NodeTuples(plan, 0, dev)
    with F.Engine(0, 4) as e, open(out, "a") as f:
        e.set_stream(stream.cuda_stream)
        e.set_frame(h.numpy())
        e.set_domains(doms)
        e.set_ranges(rngs)
        legs = {"gather": bench.FrameStep(e, h, plan, 0, dev, stripes=True),
                "node": bench.FrameStep(e, h, plan, 0, dev, stripes=True, node_tuples=node)}
        ref = None
        for r in range(rounds):
            for name, step in legs.items():
                step()
                torch.cuda.synchronize(dev)
                _, sec = bench.timed(step, steps, 1, dev)
                got = step.tuples_bytes()
                ref = ref or got
                rec = {"round": r, "leg": name, "ms_per_step": round(1e3 * sec / steps, 3),
                       "same_tuples": got == ref, "t": time.time()}
                print(json.dumps(rec), flush=True)
                f.write(json.dumps(rec) + "\n")
        del legs, step
    node.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
