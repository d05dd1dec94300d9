#!/usr/bin/env python3
"""C4 quadtree encode with FRAC_TRACE=1 (host phase timings on stderr)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

frame = value_noise(4096, 4096, 1234)[:2048, :2048].copy()
split = float(sys.argv[1]) if len(sys.argv) > 1 else 0.05
with F.Engine(0, 4, True, timing=True) as e:
    e.set_frame(frame)
    e.encode_quadtree(16, 4, split)
    os.environ["FRAC_TRACE"] = "1"
    for _ in range(int(os.environ.get("QT_CALLS", "2"))):
        t0 = time.perf_counter()
        items, st = e.encode_quadtree(16, 4, split)
        print(f"call wall {1e3 * (time.perf_counter() - t0):.3f} ms", file=sys.stderr, flush=True)
    print("items", len(items), "ms_search", st["ms_search"], "ms_device", st["ms_device"], file=sys.stderr)
