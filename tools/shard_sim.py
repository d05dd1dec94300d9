#!/usr/bin/env python3
"""Per-rank step time of bench.py's C3 workload at N-way range sharding, measured on ONE GPU:
each shard k of N (fractencode_amd.distributed.shard_plan) is set as the engine's range batch
and timed the way bench.py times a step for N > 1 (wall clock around K steps, device
synchronised): the search, the 32-byte tuple pack of the shard (frac_copy_tuples_device) and a
world-1 RCCL all_gather_into_tensor of the padded shard on the engine's stream — the collective's
launch and copy on this GPU; the xGMI transfer of the other ranks' shards is not in it.  The
slowest shard bounds the N-GPU step.  Also printed: the search's workgroup count per shard
(prepare()'s build_work rule, fracenc_api.hip), which must stay well above the 256 CUs × 2
workgroups the 8-wave search keeps resident.  The scaling curve itself is the driver's
(SCALE_rNN.json); this is a per-shard prediction, not a claim.
usage: tools/shard_sim.py [N ...]   (default 1 2 4 8)"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fractencode_amd as F  # noqa: E402
from fractencode_amd.distributed import TUPLE_BYTES, plan_capacity, shard_plan  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402


def search_wgs(nranges: int, ndoms: int, bpw: int = 8, target: int = 8192 // 8 * 4) -> int:
    """Workgroups of the 8-wave Fourier search for one bucket (build_work in fracenc_api.hip)."""
    blocks = (nranges + 31) // 32
    tiles = (ndoms + 31) // 32
    groups = (blocks + bpw - 1) // bpw
    splits = max(1, min((target + groups - 1) // groups, max(1, tiles // 4)))
    return groups * splits


def main():
    import torch
    import torch.distributed as dist

    ns = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
    S, K = 4096, 10
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    frame = value_noise(S, S, 1234)
    doms = F.create_uniform_grid(S, S, 16, 8)
    rngs = F.create_uniform_grid(S, S, 8, 8)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    rows = []
    with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_AUTO, timing=True) as e:
        e.set_stream(stream.cuda_stream)
        e.set_frame(torch.from_numpy(frame).cuda())
        e.set_domains(doms)
        base = None
        for n in ns:
            plan = shard_plan(len(rngs), n)
            cap = plan_capacity(plan)
            mine = torch.zeros(cap * TUPLE_BYTES, dtype=torch.uint8, device="cuda")
            out = torch.zeros(cap * TUPLE_BYTES, dtype=torch.uint8, device="cuda")
            worst = None
            for k in sorted({0, n - 1, n // 2}):
                a, b = plan[k]
                e.set_ranges(rngs[a:b])

                def step():
                    e.run()
                    e.copy_tuples_device(mine.data_ptr())
                    dist.all_gather_into_tensor(out, mine)  # world 1: the collective on this GPU only

                step()
                torch.cuda.synchronize()
                e.timing_history()
                t0 = time.perf_counter()
                for _ in range(K):
                    step()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) * 1e3 / K
                h = e.timing_history()
                if worst is None or ms > worst["ms_step"]:
                    worst = {"N": n, "shard": k, "ranges": b - a, "ms_step": round(ms, 3),
                             "ms_search": round(float(np.mean(h["ms_search"])), 3),
                             "ms_prep": round(float(np.mean(h["ms_prep"])), 3),
                             "ms_finish": round(float(np.mean(h["ms_finish"])), 3),
                             "search_workgroups": search_wgs(b - a, len(doms))}
            base = base or worst["ms_step"]
            worst["ideal_ms"] = round(base / n, 3)
            worst["per_shard_efficiency"] = round(base / n / worst["ms_step"], 3)
            rows.append(worst)
            print(json.dumps(worst), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
