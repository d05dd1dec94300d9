#!/usr/bin/env python3
"""Interleaved in-process A/B of MFMA search variants on the C3 frame; prints per-variant
median/min search-kernel and finish (resolve + fit) ms (library HIP events).
Variants: "d" = the C4-Fourier search (FRAC_MFMA_DFT=1, default: software-pipelined exact
form), "e" = its unpipelined exact form, "g" = the guarded fast-path form, "d5" = the five-MFMA form (variant 20), "dt" = "d" with the pairwise-tree row maximum (the default uses one v_max3 chain), "p" = pipelined with a forced interleave, "em"/"ev" = MFMA-only / VALU-only ablations of "e", an integer v = the direct
search_mfma with FRAC_MFMA_VARIANT=v (FRAC_MFMA_DFT=0).
Ablation variants need the tuning library: python tools/build_tuning.py, then
FRAC_LIB=fractencode_amd/libfracenc_tuning.so tools/ab_mfma.py ...
usage: tools/ab_mfma.py d,2 [rounds]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

variants = sys.argv[1].split(",") if len(sys.argv) > 1 else ["d", "2"]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
S = int(os.environ.get("AB_SIZE", "4096"))
REPS = int(os.environ.get("AB_REPS", "1"))
p = value_noise(S, S, 1234)
ref = None
with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_MFMA, timing=True) as e:
    e.set_frame(p)
    e.set_domains(F.create_uniform_grid(S, S, 16, 8))
    e.set_ranges(F.create_uniform_grid(S, S, 8, 8))
    res = {v: [] for v in variants}
    fin = {v: [] for v in variants}
    for r in range(rounds + 1):
        for v in variants:
            os.environ["FRAC_MFMA_DFT"] = "1" if not v.isdigit() else "0"
            os.environ["FRAC_MFMA_VARIANT"] = {"d": "2", "e": "1", "g": "3", "p": "4", "d8": "5", "dt": "6", "d2": "12", "d5": "20", "d5s": "22", "d6": "21", "d62": "23", "d6f": "26", "d6w": "27", "d6fw": "28", "fu": "33", "fb": "34", "fub": "35", "fubp": "36", "d4": "24", "dm": "201", "dm0": "202", "dmD": "203", "dmB": "204", "dD": "205", "dB": "206",
                                              "d0": "207", "dfB": "226", "df0": "227", "fM": "240", "fV": "241", "fB": "242", "f0": "243", "em": "9", "ev": "17", "emL": "41", "emB": "73",
                                              "em0": "105", "eB": "65"}.get(v, v)
            for _ in range(REPS):  # back-to-back runs: the last one is timed (the clock settles under load)
                e.run()
            out, st = e.fetch()
            if ref is None:
                ref = out.tobytes()
            if v in ("d", "e", "g", "p", "d8", "dt", "d2", "d5", "d5s", "d6", "d62", "d6f", "d6w", "d6fw", "fu", "fb", "fub", "fubp", "d4") or (v.isdigit() and (int(v) < 8 or int(v) in (32, 64, 96, 98, 128, 130))):  # 8, 16 are ablations (results intentionally wrong)
                assert out.tobytes() == ref, f"variant {v} differs"
            if r:
                res[v].append(st["ms_search"])
                fin[v].append(st["ms_finish"])
    for v in variants:
        a = np.array(res[v])
        print(f"variant {v}: search median {np.median(a):.3f} ms  min {a.min():.3f} ms  finish median "
              f"{np.median(fin[v]):.3f} ms  (n={len(a)})", flush=True)
