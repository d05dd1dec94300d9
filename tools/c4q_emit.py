#!/usr/bin/env python3
"""C4 quadtree frames (2048² S1 crop, classifier, 16/8/4, split 0.05) into a pinned caller buffer, as 64-byte
records or as 32-byte leaves — a short program for a rocprofv3 kernel trace of qt_split_emit.
usage: tools/c4q_emit.py records|leaves [frames]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "records"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dt = F.QT_LEAF if mode == "leaves" else F.ENCODE_ITEM
frame = value_noise(4096, 4096, 1234)[:2048, :2048].copy()
cap = (2048 // 4) ** 2
buf = torch.empty(cap * dt.itemsize, dtype=torch.uint8).pin_memory().numpy().view(dt)
with F.Engine(0, 4, True) as e:
    e.set_frame(frame)
    for _ in range(frames + 2):
        items, _ = e.encode_quadtree(16, 4, 0.05, out=buf, leaves=mode == "leaves")
print(mode, len(items), flush=True)
