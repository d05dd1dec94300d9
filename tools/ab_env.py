#!/usr/bin/env python3
"""Interleaved in-process A/B of a prepare-time knob (an environment variable read by
frac_set_ranges) on the C3 frame: search / total device ms (library HIP events), median.
usage: tools/ab_env.py VAR val1,val2,... [rounds]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

var, vals = sys.argv[1], sys.argv[2].split(",")
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
S = 4096
p = value_noise(S, S, 1234)
rngs = F.create_uniform_grid(S, S, 8, 8)
res = {v: [] for v in vals}
tot = {v: [] for v in vals}
ref = None
with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_AUTO, timing=True) as e:
    e.set_frame(p)
    e.set_domains(F.create_uniform_grid(S, S, 16, 8))
    for r in range(rounds + 1):
        for v in vals:
            os.environ[var] = v
            e.set_ranges(rngs)
            e.run()
            e.run()
            out, st = e.fetch()
            if ref is None:
                ref = out.tobytes()
            assert out.tobytes() == ref, f"{var}={v} differs"
            if r:
                res[v].append(st["ms_search"])
                tot[v].append(st["ms_device"])
for v in vals:
    print(f"{var}={v}: search median {np.median(res[v]):.3f} ms  min {min(res[v]):.3f}  device median "
          f"{np.median(tot[v]):.3f} ms (n={len(res[v])})", flush=True)
