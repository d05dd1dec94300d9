#!/usr/bin/env python3
"""Interleaved in-process A/B of search_mfma schedule variants (FRAC_MFMA_VARIANT) on the C3
frame; prints per-variant median/min search-kernel ms (library HIP events)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1", "2"])]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
S = int(os.environ.get("AB_SIZE", "4096"))
p = value_noise(S, S, 1234)
ref = None
with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_MFMA, timing=True) as e:
    e.set_frame(p)
    e.set_domains(F.create_uniform_grid(S, S, 16, 8))
    e.set_ranges(F.create_uniform_grid(S, S, 8, 8))
    res = {v: [] for v in variants}
    for r in range(rounds + 1):
        for v in variants:
            os.environ["FRAC_MFMA_VARIANT"] = str(v)
            e.run()
            out, st = e.fetch()
            if ref is None:
                ref = out.tobytes()
            if v < 8:  # 8, 16 are ablations (results intentionally wrong)
                assert out.tobytes() == ref, f"variant {v} differs"
            if r:
                res[v].append(st["ms_search"])
    for v in variants:
        a = np.array(res[v])
        print(f"variant {v}: search median {np.median(a):.3f} ms  min {a.min():.3f} ms  (n={len(a)})", flush=True)
