#!/usr/bin/env python3
"""Diagnostic: the direct MFMA form (FRAC_MFMA_VARIANT=v, FRAC_MFMA_DFT=0) against the Fourier form
on an S1 frame; prints the differing records with their exact S16 (numpy)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

S = int(os.environ.get("AB_SIZE", "2048"))
p = value_noise(S, S, 1234)
doms = F.create_uniform_grid(S, S, 16, 8)
rngs = F.create_uniform_grid(S, S, 8, 8)
outs = {}
VARS = os.environ.get("VARS", "2,130").split(",")
for name, dft, var in [("fourier", "1", "")] + [("direct" + v, "0", v) for v in VARS]:
    os.environ["FRAC_MFMA_DFT"] = dft
    os.environ["FRAC_MFMA_VARIANT"] = var
    with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_MFMA) as e:
        e.set_frame(p)
        e.set_domains(doms)
        outs[name], _ = e.search(rngs)
fwd = np.array([[F.transform_index(8, t, q) for q in range(64)] for t in range(4)])
pi = p.astype(np.int64)


def s16(r, d, t):
    rr, dd = rngs[r], doms[d]
    R = pi[rr["y"]:rr["y"] + 8, rr["x"]:rr["x"] + 8].reshape(-1)
    D = pi[dd["y"]:dd["y"] + 16, dd["x"]:dd["x"] + 16]
    D4 = (D[0::2, 0::2] + D[1::2, 0::2] + D[0::2, 1::2] + D[1::2, 1::2]).reshape(-1)
    return int(((4 * R - D4[fwd[t]]) ** 2).sum())


didx = {(int(x), int(y)): i for i, (x, y) in enumerate(zip(doms["x"], doms["y"]))}
for name in ["direct" + v for v in VARS]:
    a, b = outs["fourier"], outs[name]
    diff = np.nonzero((a["dx"] != b["dx"]) | (a["dy"] != b["dy"]) | (a["transform"] != b["transform"]))[0]
    print(name, "differing ranges:", len(diff), flush=True)
    for r in diff[:8]:
        for nm, o in (("fourier", a), (name, b)):
            d = didx[(int(o["dx"][r]), int(o["dy"][r]))]
            print(f"  r={r} {nm}: domain {d} t={o['transform'][r]} dist={o['distance'][r]!r} S16={s16(r, d, int(o['transform'][r]))}")
