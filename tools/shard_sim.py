#!/usr/bin/env python3
"""Per-rank step time of bench.py's C3 workload at N-way range sharding, measured on ONE GPU:
each shard k of N (fractencode_amd.distributed.shard_bounds) is set as the engine's range
batch and timed the way bench.py times a step (wall clock around K runs, device
synchronised), with the library's per-phase HIP events.  The slowest shard bounds the
N-GPU step before the RCCL all-gather is added.
usage: tools/shard_sim.py [N ...]   (default 1 2 4 8)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fractencode_amd as F  # noqa: E402
from fractencode_amd.distributed import shard_bounds  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

ns = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
S, K = 4096, 10
frame = value_noise(S, S, 1234)
doms = F.create_uniform_grid(S, S, 16, 8)
rngs = F.create_uniform_grid(S, S, 8, 8)
with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_AUTO, timing=True) as e:
    e.set_frame(frame)
    e.set_domains(doms)
    base = None
    for n in ns:
        worst = None
        for k in sorted({0, n - 1, n // 2}):
            a, b = shard_bounds(len(rngs), n, k)
            e.set_ranges(rngs[a:b])
            e.run()
            e.sync()
            t0 = time.perf_counter()
            for _ in range(K):
                e.run()
            e.sync()
            ms = (time.perf_counter() - t0) * 1e3 / K
            _, st = e.fetch()
            if worst is None or ms > worst[0]:
                worst = (ms, k, st)
        ms, k, st = worst
        base = base or ms
        print(f"N={n}: slowest shard {k}: {ms:.3f} ms/step (prep {st['ms_prep']:.3f}, search {st['ms_search']:.3f}, "
              f"finish {st['ms_finish']:.3f})  ideal {base / n:.3f}  compute-only efficiency {base / n / ms:.3f}",
              flush=True)
