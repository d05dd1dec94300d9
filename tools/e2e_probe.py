#!/usr/bin/env python3
"""Where the headline's end-to-end step (bench.FrameStep: frame H2D, search, tuples D2H) spends its time
beside the device-resident step: per leg the step ms (host clock) and the library's per-run event times
(device / prep / search / finish, median), alternated `rounds` times so drift shows as a pattern.  Two more
legs separate why the search runs slower in the end-to-end step: the device-resident step with the GPU idle
0.5 ms between steps (clock / power), and with a device-to-device re-copy of the frame instead of the H2D.
Leg e2e_zc packs the tuples straight into the pinned host buffer (the pack kernel's stores cross PCIe) instead
of packing on the device and copying.  Run it with HSA_ENABLE_SDMA=0 to see the copies done by blit kernels.
Legs idle_<µs>: the device-resident step after that many µs of GPU idle (how the slowdown grows with the idle).
Leg e2e_nosink: the end-to-end step without the tuple sink (pack + D2H after the run).
usage: tools/e2e_probe.py [steps] [rounds] [legs,...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import fractencode_amd as F  # noqa: E402
from fractencode_amd.distributed import shard_plan  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
only = sys.argv[3].split(",") if len(sys.argv) > 3 else None
S = 4096
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
frame = value_noise(S, S, 1234)
rngs = F.create_uniform_grid(S, S, 8, 8)
plan = shard_plan(len(rngs), 1)
h_frame = torch.from_numpy(frame).pin_memory()
d_frame = torch.from_numpy(frame).to(dev)
with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_AUTO, timing=True) as e:
    e.set_stream(stream.cuda_stream)
    e.set_frame(h_frame.numpy())
    e.set_domains(F.create_uniform_grid(S, S, 16, 8))
    e.set_ranges(rngs)
    dstep = bench.FrameStep(e, None, plan, 0, dev, device_resident=True)
    d_frame2 = d_frame.clone()

    def idle_step():  # the device-resident step with the GPU idle 0.5 ms between steps (no copy)
        torch.cuda.synchronize(dev)
        time.sleep(0.0005)
        dstep()

    def d2d_step():  # a device-to-device re-copy of the frame each step instead of the H2D
        e.set_frame(d_frame2)
        dstep()

    zstep = bench.FrameStep(e, h_frame.numpy(), plan, 0, dev)

    def zc_step():  # H2D, search, tuples packed by the kernel directly into pinned host memory
        e.set_frame(h_frame.numpy())
        e.run()
        e.copy_tuples_device(zstep.h_out.data_ptr())

    nosink = bench.FrameStep(e, h_frame.numpy(), plan, 0, dev)
    nosink.sink = False  # the pack kernel and the D2H copy after the run (the step before frac_set_tuple_sink)
    legs = {"e2e": bench.FrameStep(e, h_frame.numpy(), plan, 0, dev), "device": dstep, "device_idle": idle_step,
            "device_d2d": d2d_step, "e2e_zc": zc_step, "e2e_nosink": nosink}
    for us in (50, 100, 200, 500, 1000, 2000):  # idle_<µs>: the device-resident step after that much GPU idle
        legs[f"idle_{us}"] = (lambda sec: (lambda: (torch.cuda.synchronize(dev), time.sleep(sec), dstep())))(us * 1e-6)
    if only:
        legs = {k: v for k, v in legs.items() if k in only}
    ref = None
    for r in range(rounds):
        for name, step in legs.items():
            if name.startswith(("device", "idle")):
                e.set_frame(d_frame)
            for _ in range(3):
                step()
            torch.cuda.synchronize(dev)
            e.timing_history()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize(dev)
            sec = (time.perf_counter() - t0) / steps
            h = e.timing_history()
            if name == "e2e_zc":  # the zero-copy tuples equal the device-packed ones
                dstep()
                torch.cuda.synchronize(dev)
                zc_step()
                torch.cuda.synchronize(dev)
                assert zstep.h_out.numpy().tobytes() == dstep.gathered.cpu().numpy().tobytes()
            print(json.dumps({"round": r, "leg": name, "ms_per_step": round(sec * 1e3, 3),
                              **{k: round(float(np.median(h["ms_" + k])), 3) for k in ("device", "prep", "search", "finish")}}),
                  flush=True)
