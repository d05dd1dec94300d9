#!/usr/bin/env python3
"""In-kernel shader clock of the C3 Fourier search (MI355X_MICROARCH.md "DVFS
give-back" item 6): needs the diagnostic library (python tools/build_tuning.py --stamps), whose
search_dft stamps s_memtime and s_memrealtime around its loop per workgroup.  For each variant,
runs the C3 frame back to back for --seconds (≥ 2 s: the clock settles under load), then reads the
last launch's stamps: per workgroup clock = Δs_memtime ÷ Δs_memrealtime × 100 MHz; prints the
median / p10 / p90 over workgroups and the launch's span (first start to last end, in µs) as
one JSON line per variant.  --dump DIR: each variant's last-launch stamps (with the workgroup's XCC, HW_ID
and tile range) to DIR/stamps_<variant>.npy for tools/l2_model.py.
usage: FRAC_LIB=fractencode_amd/libfracenc_stamps.so tools/clock_stamp.py 35,240 [--seconds 2.5] [--dump DIR]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fractencode_amd as F  # noqa: E402
from fractencode_amd.synth import value_noise  # noqa: E402

variants = (sys.argv[1] if len(sys.argv) > 1 else "35,240").split(",")
seconds = float(sys.argv[sys.argv.index("--seconds") + 1]) if "--seconds" in sys.argv else 2.5
dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
WORDS = 6  # fracenc_dft.hip kClockStampWords
lib = ctypes.CDLL(F.LIB_PATH)
if not hasattr(lib, "frac_clock_stamps"):
    sys.exit(f"{F.LIB_PATH} is not the diagnostic clock build (tools/build_tuning.py --stamps)")
lib.frac_clock_stamps.restype = ctypes.c_int
lib.frac_clock_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_size_t]
REALTIME_HZ = 100e6  # s_memrealtime: the constant 100 MHz reference

# --c2: BASELINE configs[1] instead (Lenna 512², T = 8) — where the search is latency-bound
c2 = "--c2" in sys.argv
if c2:
    S, T = 512, 8
    plane = np.fromfile(os.path.join(ROOT, "tests", "golden", "lenna_y.u8"), np.uint8).reshape(S, S)
else:
    S, T = 4096, 4
    plane = value_noise(S, S, 1234)
os.environ["FRAC_MFMA_DFT"] = "1"
with F.Engine(0, T, False, 0.0, -1.0, F.ENGINE_MFMA, timing=True) as e:
    e.set_frame(plane)
    e.set_domains(F.create_uniform_grid(S, S, 16, 8))
    e.set_ranges(F.create_uniform_grid(S, S, 8, 8))
    for v in variants:
        os.environ["FRAC_MFMA_VARIANT"] = v
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            e.run()
            n += 1
            if n % 16 == 0:  # bound the queue: the loop's clock is the device's
                e.fetch()
        _, st = e.fetch()
        cap = 1 << 16
        buf = (ctypes.c_ulonglong * (cap * WORDS))()
        got = lib.frac_clock_stamps(buf, cap)
        if got <= 0:
            sys.exit(f"variant {v}: no stamps ({got})")
        raw = np.frombuffer(buf, dtype=np.uint64, count=got * WORDS).reshape(got, WORDS).copy()
        if dump:
            os.makedirs(dump, exist_ok=True)
            np.save(os.path.join(dump, f"stamps_{v}.npy"), raw)
        s = raw[:, :4].astype(np.float64)
        dck, drt = s[:, 1] - s[:, 0], s[:, 3] - s[:, 2]
        ok = drt > 0
        mhz = dck[ok] / drt[ok] * REALTIME_HZ / 1e6
        span_us = (s[:, 3].max() - s[:, 2].min()) / REALTIME_HZ * 1e6
        print(json.dumps({"variant": int(v), "launches": n, "seconds": round(time.perf_counter() - t0, 2),
                          "workgroups": int(got), "clock_mhz_median": round(float(np.median(mhz)), 1),
                          "clock_mhz_p10": round(float(np.percentile(mhz, 10)), 1),
                          "clock_mhz_p90": round(float(np.percentile(mhz, 90)), 1),
                          "wg_loop_us_median": round(float(np.median(drt[ok])) / REALTIME_HZ * 1e6, 2),
                          "wg_loop_us_max": round(float(drt[ok].max()) / REALTIME_HZ * 1e6, 2),
                          "wg_start_spread_us": round(float(s[:, 2].max() - s[:, 2].min()) / REALTIME_HZ * 1e6, 2),
                          "launch_span_us": round(float(span_us), 2),
                          "ms_search_event": round(float(st["ms_search"]), 4)}), flush=True)
