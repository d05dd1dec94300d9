#!/usr/bin/env python3
"""The fp32-regime cost at C3 size (fallback_wave): a 4096² S1 frame scaled into [0, 60] — so no
domain's 2×2 sums come near 1020 — with K isolated white 8×8 ranges, each alone in a black 24×24 patch.  A white
range's best error is then ≥ 48·1020² > 2^24 (the domain holding it covers a quarter of its cells), the
fp32 regime the resolving wave emulates in reference order over every candidate of its bucket.  Prints per K
the per-run device / search / finish ms (library HIP events, median of `reps` runs: the run's kernels, before
the fallback settles), the wall clock per run + sync (the fallback included) and the fallback count.
usage: tools/fallback_probe.py [K ...]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402


def frame(k: int, S: int = 4096) -> np.ndarray:
    p = (value_noise(S, S, 1234).astype(np.float64) * (60.0 / 255.0)).astype(np.uint8)
    rng = np.random.default_rng(17)
    cells = rng.choice((S // 24) ** 2, size=k, replace=False)
    for c in cells:
        y0, x0 = (c // (S // 24)) * 24, (c % (S // 24)) * 24
        y0, x0 = y0 - y0 % 8, x0 - x0 % 8
        p[y0:y0 + 24, x0:x0 + 24] = 0
        p[y0 + 8:y0 + 16, x0 + 8:x0 + 16] = 255
    return p


if __name__ == "__main__":
    ks = [int(a) for a in sys.argv[1:]] or [0, 1, 16]
    S, reps = 4096, 5
    for k in ks:
        with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_AUTO, timing=True) as e:
            e.set_frame(frame(k, S))
            e.set_domains(F.create_uniform_grid(S, S, 16, 8))
            e.set_ranges(F.create_uniform_grid(S, S, 8, 8))
            e.run()
            e.sync()
            e.timing_history()
            t0 = time.perf_counter()
            for _ in range(reps):
                e.run()
                e.sync()  # settles the listed fp32-regime ranges (fallback_grid)
            wall = (time.perf_counter() - t0) / reps
            h = e.timing_history()
            _, st = e.fetch()
        print(json.dumps({"white_ranges": k, "fallback_ranges": st["fallback_ranges"], "wall_ms": round(wall * 1e3, 3),
                          **{k2: round(float(np.median(h["ms_" + k2])), 3) for k2 in ("device", "search", "finish")}}),
              flush=True)
