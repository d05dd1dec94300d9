#!/usr/bin/env python3
"""C2 (Lenna 512², 8×8 ranges, 16×16 domains, T = 4 and 8): frames per second when runs are
enqueued back to back (one sync at the end), with and without the library's timing events, next
to the per-run device time of the event path. Separates the GPU's kernel chain from the host's
launch rate."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fractencode_amd as F  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
p = np.fromfile(os.path.join(ROOT, "tests", "golden", "lenna_y.u8"), np.uint8).reshape(512, 512)
K = int(os.environ.get("C2_FRAMES", "200"))  # the library keeps the last 256 runs' timings
for T in (8, 4):
    for timing in (False, True):
        with F.Engine(0, T, False, 0.0, -1.0, F.ENGINE_AUTO, timing=timing) as e:
            e.set_frame(p)
            e.set_domains(F.create_uniform_grid(512, 512, 16, 8))
            e.set_ranges(F.create_uniform_grid(512, 512, 8, 8))
            for _ in range(20):
                e.run()
            e.sync()
            if timing:
                e.timing_history()  # drain the warm-up runs
            t0 = time.perf_counter()
            for _ in range(K):
                e.run()
            t1 = time.perf_counter()
            e.sync()
            t2 = time.perf_counter()
            us = 1e6 * (t2 - t0) / K
            dev = ""
            if timing:
                h = e.timing_history()
                dev = f", device (events) {np.median(h['ms_device']) * 1e3:.1f} us"
            print(f"T={T} timing={int(timing)}: {us:.1f} us per frame back to back (host enqueue "
                  f"{1e6 * (t1 - t0) / K:.1f} us), {4096 / us:.2f} M range-blocks/s{dev}", flush=True)
