#!/usr/bin/env python3
"""Times the oracle restatement (oracle/fracoracle.c) against the reference build (oracle/_ref) on the
same sample of the C3 frame, same threads: the speed ratio DESIGN §6 quotes for the cpu_baseline.
usage: tools/oracle_vs_ref.py [ranges] [threads]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fractencode_amd.synth import value_noise  # noqa: E402
from oracle import oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
S = 4096
frame = value_noise(S, S, 1234)
sel = np.arange(0, (S // 8) ** 2, (S // 8) ** 2 // n, dtype=np.uint32)[:n]
doms, rngs = O.uniform_grid(S, S, 16, 8), O.uniform_grid(S, S, 8, 8)[sel]
res = {}
for rep in range(2):
    t0 = time.perf_counter()
    O.estimate(frame, doms, rngs, T=4, threads=threads)
    res.setdefault("oracle", []).append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    O.ref_estimate(frame, 16, 8, 4, sel=sel, threads=threads)
    res.setdefault("reference", []).append(time.perf_counter() - t0)
o, r = min(res["oracle"]), min(res["reference"])
print(f"{n} ranges of the C3 frame, {threads} threads: oracle {o:.2f} s, reference {r:.2f} s, "
      f"oracle/reference time {o / r:.3f}", flush=True)
