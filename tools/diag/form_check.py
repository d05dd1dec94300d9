#!/usr/bin/env python3
"""Diagnostic: records of a Fourier-form variant (FRAC_MFMA_VARIANT=argv[1]) against the VALU
engine on a uniform-noise frame; prints the first mismatching ranges."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fractencode_amd as F  # noqa: E402

var = sys.argv[1] if len(sys.argv) > 1 else "21"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 128
rng = np.random.default_rng(2000)
p = rng.integers(0, 256, (S, S), dtype=np.uint8)
doms, rngs = F.create_uniform_grid(S, S, 16, 8), F.create_uniform_grid(S, S, 8, 8)
with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_VALU) as e:
    e.set_frame(p)
    e.set_domains(doms)
    want, _ = e.search(rngs)
os.environ["FRAC_MFMA_DFT"] = "1"
os.environ["FRAC_MFMA_VARIANT"] = var
with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_MFMA) as e:
    e.set_frame(p)
    e.set_domains(doms)
    out, _ = e.search(rngs)
bad = np.nonzero(np.any(
    np.stack([out[k] != want[k] for k in ("dx", "dy", "transform", "distance")]), axis=0))[0]
print(f"variant {var}: {len(bad)} of {len(rngs)} ranges differ")
for i in bad[:12]:
    print(i, "got", out[i][["dx", "dy", "transform", "distance"]], "want", want[i][["dx", "dy", "transform", "distance"]],
          "S16 got/want", out["distance"][i] * 256 * 16, want["distance"][i] * 256 * 16)
