#!/usr/bin/env python3
"""C2 (Lenna 512², 8×8 ranges, 16×16 domains, all 8 transforms): per-run device ms
(library HIP events) for the MFMA engine; run under rocprofv3 for the kernel breakdown."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fractencode_amd as F  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
p = np.fromfile(os.path.join(ROOT, "tests", "golden", "lenna_y.u8"), np.uint8).reshape(512, 512)
for T in (8, 4):
    with F.Engine(0, T, False, 0.0, -1.0, F.ENGINE_AUTO, timing=True) as e:
        e.set_frame(p)
        e.set_domains(F.create_uniform_grid(512, 512, 16, 8))
        e.set_ranges(F.create_uniform_grid(512, 512, 8, 8))
        ms = []
        for _ in range(20):
            e.run()
            _, st = e.fetch()
            ms.append((st["ms_device"], st["ms_prep"], st["ms_search"], st["ms_finish"]))
        a = np.median(np.array(ms[2:]), axis=0)
        print(f"T={T}: device {a[0]:.3f} ms (prep {a[1]:.3f}, search {a[2]:.3f}, finish {a[3]:.3f}), "
              f"{4096 / a[0] * 1e3 / 1e6:.2f} M range-blocks/s", flush=True)

if len(sys.argv) > 1 and sys.argv[1] == "c3t8":
    # the C3 frame with all 8 transforms (BASELINE configs[1]'s transform set at configs[2]'s size)
    from fractencode_amd.synth import value_noise  # noqa: E402

    S = 4096
    q = value_noise(S, S, 1234)
    with F.Engine(0, 8, False, 0.0, -1.0, F.ENGINE_AUTO, timing=True) as e:
        e.set_frame(q)
        e.set_domains(F.create_uniform_grid(S, S, 16, 8))
        e.set_ranges(F.create_uniform_grid(S, S, 8, 8))
        ms = []
        for _ in range(4):
            e.run()
            _, st = e.fetch()
            ms.append((st["ms_device"], st["ms_prep"], st["ms_search"], st["ms_finish"]))
        a = np.median(np.array(ms[1:]), axis=0)
        print(f"C3 T=8: device {a[0]:.3f} ms (prep {a[1]:.3f}, search {a[2]:.3f}, finish {a[3]:.3f}), "
              f"{262144 / a[0] * 1e3 / 1e6:.2f} M range-blocks/s, form {st['search_form']}", flush=True)

if len(sys.argv) > 1 and sys.argv[1] == "cli4096":
    # the reference CLI's default geometry (16×16 domains at offset 8, 4×4 ranges: match_16to4) at C3 size
    from fractencode_amd.synth import value_noise  # noqa: E402

    S = 4096
    q = value_noise(S, S, 1234)
    for cls in (False, True):
        with F.Engine(0, 4, cls, 0.0, -1.0, F.ENGINE_AUTO, timing=True) as e:
            e.set_frame(q)
            e.set_domains(F.create_uniform_grid(S, S, 16, 8))
            e.set_ranges(F.create_uniform_grid(S, S, 4, 4))
            ms = []
            for _ in range(3):
                e.run()
                _, st = e.fetch()
                ms.append((st["ms_device"], st["ms_prep"], st["ms_search"], st["ms_finish"]))
            a = np.median(np.array(ms[1:]), axis=0)
            nr = (S // 4) ** 2
            print(f"16->4 at {S}², classifier {cls}: device {a[0]:.3f} ms (prep {a[1]:.3f}, search {a[2]:.3f}, "
                  f"finish {a[3]:.3f}), {nr / a[0] * 1e3 / 1e6:.2f} M range-blocks/s, form {st['search_form']}, "
                  f"engine {st['engine']}", flush=True)
