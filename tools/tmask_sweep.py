#!/usr/bin/env python3
"""Per frame size the Fourier path's frame time for the library FRAC_LIB names (or the product): value noise
S×S, 8×8 ranges, 16×16 domains stride 8, T = 4 (and Lenna-sized T = 8 at 512), µs per frame enqueued back to
back (median of `rounds` blocks of `reps` runs) plus the library's event split (search / finish, median).
Run alternately per library (search_dft with and without TMASK) to place kDftTmaskTiles.
usage: tools/tmask_sweep.py [reps] [sizes...]"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
sizes = [int(a) for a in sys.argv[2:]] or [512, 1024, 1536, 2048, 2560, 4096]
lib = os.path.basename(os.environ.get("FRAC_LIB", "libfracenc.so"))
for S in sizes:
    for T in ((8, 4) if S == 512 else (4,)):
        n = reps if S <= 2048 else max(5, reps // 10)
        with F.Engine(0, T, False, 0.0, -1.0, F.ENGINE_AUTO, timing=True) as e:
            e.set_frame(value_noise(S, S, 1234))
            e.set_domains(F.create_uniform_grid(S, S, 16, 8))
            e.set_ranges(F.create_uniform_grid(S, S, 8, 8))
            for _ in range(3):
                e.run()
            e.sync()
            e.timing_history()
            blocks = []
            for _ in range(3):
                t0 = time.perf_counter()
                for _ in range(n):
                    e.run()
                e.sync()
                blocks.append((time.perf_counter() - t0) / n)
            h = e.timing_history()
            rec, st = e.fetch()
        print(json.dumps({"lib": lib, "S": S, "T": T, "tiles": (((S - 16) // 8 + 1) ** 2 + 31) // 32,
                          "us_b2b": round(1e6 * float(np.median(blocks)), 2),
                          **{k: round(1e3 * float(np.median(h["ms_" + k])), 2) for k in ("search", "finish")},
                          "digest": hashlib.sha256(np.ascontiguousarray(rec).tobytes()).hexdigest()[:16]}), flush=True)
