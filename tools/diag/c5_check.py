#!/usr/bin/env python3
"""Diagnostic: C5 Y/U/V searches vs the reference samples, repeated; prints mismatching records."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from golden_util import FIELDS, c5_rgb, golden, selection  # noqa: E402

import fractencode_amd as F  # noqa: E402
from fractencode_amd.color import ColorEncoder  # noqa: E402


def fields(out):
    return {"x": out["x"], "y": out["y"], "dx": out["dx"], "dy": out["dy"], "dw": out["sw"], "dh": out["sh"],
            "t": out["transform"], "dist": out["distance"], "s": out["contrast"], "o": out["brightness"]}


rgb = c5_rgb()
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    with ColorEncoder(0, 8, 16, 4) as enc:
        enc.load(rgb)
        enc.run()
        enc.sync()
        results = enc.fetch()
        for k, name in enumerate(("c5_y", "c5_u", "c5_v")):
            out, st = results[k]
            rec, meta = golden(name + "_sample")
            sel = selection(meta, len(out))
            g = fields(out[sel])
            bad = np.zeros(len(sel), bool)
            for f in FIELDS:
                bad |= g[f] != rec[f]
            print(rep, name, "mismatches", int(bad.sum()), flush=True)
            for i in np.nonzero(bad)[0][:5]:
                print("   got ", {f: g[f][i] for f in FIELDS})
                print("   want", {f: rec[f][i] for f in FIELDS}, flush=True)
