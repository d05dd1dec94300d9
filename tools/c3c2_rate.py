#!/usr/bin/env python3
"""One JSON line of the two Fourier-path rates an A/B of the search/resolve chain needs, for the library
FRAC_LIB names (or the product): C3 (4096² S1, T = 4) per-run device / search / finish ms (library HIP
events, median of `--c3` runs after 2 warm-ups) and C2 (Lenna 512², T = 8 and 4) µs per frame enqueued back
to back and event-timed (median).  Run it alternately per library for an interleaved A/B
(tools/session.sh paths).  usage: tools/c3c2_rate.py [--c3 K] [--c2 K]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--c3", type=int, default=10)
ap.add_argument("--c2", type=int, default=200)
args = ap.parse_args()
out = {"lib": os.path.basename(os.environ.get("FRAC_LIB", "libfracenc.so")), "build": F.build_info()["build_id"]}
if args.c3:
    S = 4096
    with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_AUTO, timing=True) as e:
        e.set_frame(value_noise(S, S, 1234))
        e.set_domains(F.create_uniform_grid(S, S, 16, 8))
        e.set_ranges(F.create_uniform_grid(S, S, 8, 8))
        for _ in range(2):
            e.run()
        e.sync()
        e.timing_history()
        for _ in range(args.c3):
            e.run()
        h = e.timing_history()
        rec, _ = e.fetch()
    out["c3"] = {k: round(float(np.median(h["ms_" + k])), 4) for k in ("device", "search", "finish")}
    import hashlib
    out["c3"]["records_sha16"] = hashlib.sha256(rec.tobytes()).hexdigest()[:16]
if args.c2:
    p = np.fromfile(os.path.join(ROOT, "tests", "golden", "lenna_y.u8"), np.uint8).reshape(512, 512)
    for T in (8, 4):
        r = {}
        for timing in (False, True):
            with F.Engine(0, T, False, 0.0, -1.0, F.ENGINE_AUTO, timing=timing) as e:
                e.set_frame(p)
                e.set_domains(F.create_uniform_grid(512, 512, 16, 8))
                e.set_ranges(F.create_uniform_grid(512, 512, 8, 8))
                for _ in range(20):
                    e.run()
                e.sync()
                if timing:
                    e.timing_history()
                t0 = time.perf_counter()
                for _ in range(args.c2):
                    e.run()
                e.sync()
                us = 1e6 * (time.perf_counter() - t0) / args.c2
                if timing:
                    r["event_us"] = round(float(np.median(e.timing_history()["ms_device"])) * 1e3, 2)
                else:
                    r["b2b_us"] = round(us, 2)
        out[f"c2_t{T}"] = r
print(json.dumps(out), flush=True)
