#!/usr/bin/env python3
"""SEA engine on several frames: ms per frame (library HIP events, median of 5), fraction of the
candidates evaluated exactly, and identity with the exhaustive MFMA/VALU engine's records.
usage: tools/sea_stats.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import uniform_noise, value_noise  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lenna = np.fromfile(os.path.join(ROOT, "tests", "golden", "lenna_y.u8"), np.uint8).reshape(512, 512)
cases = [("C3 S1 4096^2 T=4", value_noise(4096, 4096, 1234), 4, False),
         ("C4 S1 2048^2 T=4 classifier", value_noise(4096, 4096, 1234)[:2048, :2048].copy(), 4, True),
         ("C2 Lenna 512^2 T=8", lenna, 8, False),
         ("S2 noise 1024^2 T=4", uniform_noise(1024, 1024, 42), 4, False)]
for name, p, T, cls in cases:
    H, W = p.shape
    doms = F.create_uniform_grid(W, H, 16, 8)
    rngs = F.create_uniform_grid(W, H, 8, 8)
    if cls:
        doms = F.preclassify(p, doms)
        rngs = F.preclassify(p, rngs)
    outs, line = [], []
    for eng in (F.ENGINE_AUTO, F.ENGINE_SEA):
        with F.Engine(0, T, cls, 0.0, -1.0, eng, timing=True) as e:
            e.set_frame(p)
            e.set_domains(doms)
            e.set_ranges(rngs)
            ms, srch = [], []
            for _ in range(6):
                e.run()
                out, st = e.fetch()
                ms.append(st["ms_device"])
                srch.append(st["ms_search"])
            outs.append(out)
            line.append(f"{F.FORM_NAMES[st['search_form']]}: {np.median(ms[1:]):.3f} ms (search "
                        f"{np.median(srch[1:]):.3f}), evaluated {st['evaluated_mappings'] / st['total_mappings']:.5f}")
    same = outs[0].tobytes() == outs[1].tobytes()
    print(f"{name}: " + " | ".join(line) + f" | identical={same}", flush=True)
