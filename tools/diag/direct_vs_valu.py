#!/usr/bin/env python3
"""Diagnostic: the direct MFMA form (FRAC_MFMA_DFT=0, FRAC_MFMA_VARIANT in VARS) against the VALU
engine on an S1 frame, range size N, transforms T; prints the number of differing records."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

S = int(os.environ.get("AB_SIZE", "512"))
N = int(os.environ.get("N", "8"))
T = int(os.environ.get("T", "4"))
p = value_noise(S, S, 1234)
doms = F.create_uniform_grid(S, S, 2 * N, N)
rngs = F.create_uniform_grid(S, S, N, N)
os.environ["FRAC_MFMA_DFT"] = "0"
with F.Engine(0, T, False, 0.0, -1.0, F.ENGINE_VALU) as e:
    e.set_frame(p)
    e.set_domains(doms)
    ref, _ = e.search(rngs)
for v in os.environ.get("VARS", "130").split(","):
    os.environ["FRAC_MFMA_VARIANT"] = v
    with F.Engine(0, T, False, 0.0, -1.0, F.ENGINE_MFMA) as e:
        e.set_frame(p)
        e.set_domains(doms)
        out, st = e.search(rngs)
    bad = (out["dx"] != ref["dx"]) | (out["dy"] != ref["dy"]) | (out["transform"] != ref["transform"]) | \
          (out["distance"] != ref["distance"])
    print(f"S={S} N={N} T={T} variant {v}: form {F.FORM_NAMES.get(st['search_form'])} differing {int(bad.sum())} of {len(out)}",
          flush=True)
