#!/usr/bin/env python3
"""One C3 frame (4096² S1 value noise, 8×8 ranges, 16×16 domains stride 8, T = 4) searched
`reps` times on one engine — a short program for rocprofv3 counter passes.
usage: tools/c3_once.py [mfma|sea|valu] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

eng = {"mfma": F.ENGINE_MFMA, "sea": F.ENGINE_SEA, "valu": F.ENGINE_VALU}[sys.argv[1] if len(sys.argv) > 1 else "mfma"]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
S = 4096
p = value_noise(S, S, 1234)
with F.Engine(0, 4, False, 0.0, -1.0, eng) as e:
    e.set_frame(p)
    e.set_domains(F.create_uniform_grid(S, S, 16, 8))
    e.set_ranges(F.create_uniform_grid(S, S, 8, 8))
    for _ in range(reps):
        e.run()
    out, st = e.fetch()
    print(st["search_form"], st["evaluated_mappings"], flush=True)
