#!/usr/bin/env python3
"""One C3 frame (4096² S1 value noise, 8×8 ranges, 16×16 domains stride 8, T = 4) searched
`reps` times on one engine — a short program for rocprofv3 counter passes and kernel traces.
Mode "e2e" runs bench.py's headline step instead: per rep the frame H2D from pinned memory, the
search and the 32-byte tuples D2H into pinned memory (bench.FrameStep at N = 1), so a kernel trace
of it times search_dft under the headline's own conditions (roofline.kernel_ms).
usage: tools/c3_once.py [mfma|sea|valu] [reps] [e2e]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

eng = {"mfma": F.ENGINE_MFMA, "sea": F.ENGINE_SEA, "valu": F.ENGINE_VALU}[sys.argv[1] if len(sys.argv) > 1 else "mfma"]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
e2e = len(sys.argv) > 3 and sys.argv[3] == "e2e"
S = 4096
p = value_noise(S, S, 1234)
rngs = F.create_uniform_grid(S, S, 8, 8)
with F.Engine(0, 4, False, 0.0, -1.0, eng) as e:
    e.set_domains(F.create_uniform_grid(S, S, 16, 8))
    e.set_ranges(rngs)
    if e2e:
        import torch

        import bench
        from fractencode_amd.distributed import shard_plan

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(0)
        stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        e.set_stream(stream.cuda_stream)
        h = torch.from_numpy(p).pin_memory()
        e.set_frame(h.numpy())
        step = bench.FrameStep(e, h.numpy(), shard_plan(len(rngs), 1), 0, dev)
        for _ in range(reps):
            step()
        torch.cuda.synchronize(dev)
    else:
        e.set_frame(p)
        for _ in range(reps):
            e.run()
    out, st = e.fetch()
    print(st["search_form"], st["evaluated_mappings"], flush=True)
