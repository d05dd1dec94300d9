#!/usr/bin/env python3
"""Does replaying a captured HIP graph of frac_run beat launching it (C2: Lenna 512², T = 8 and 4; C3)?
One context per case on a torch stream; frac_run captured once with torch.cuda.graph (the library enqueues on
the stream it was given), then K back-to-back launches vs K graph replays, interleaved rounds; the records after
the replays must equal the launched run's.  usage: tools/graph_probe.py [K] [rounds]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch

    import fractencode_amd as F
    from fractencode_amd.synth import value_noise
    from golden_util import plane

    K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    cases = [("c2_t8", plane("lenna_y"), 8, K), ("c2_t4", plane("lenna_y"), 4, K),
             ("c3", value_noise(4096, 4096, 1234), 4, max(4, K // 100))]
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    for name, p, T, k in cases:
        H, W = p.shape
        e = F.Engine(0, T)
        e.set_stream(s.cuda_stream)
        e.set_frame(p)
        e.set_domains(F.create_uniform_grid(W, H, 16, 8))
        e.set_ranges(F.create_uniform_grid(W, H, 8, 8))
        e.run()
        want, _ = e.fetch()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            e.run()
        g.replay()
        torch.cuda.synchronize()
        got, _ = e.fetch()
        same = got.tobytes() == want.tobytes()
        res = {"launch": [], "graph": []}
        for _ in range(rounds):
            for mode in ("launch", "graph"):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(k):
                    if mode == "graph":
                        g.replay()
                    else:
                        e.run()
                torch.cuda.synchronize()
                res[mode].append((time.perf_counter() - t0) / k * 1e6)
        print(json.dumps({"case": name, "frames": k, "records_equal": same,
                          "launch_us": [round(x, 2) for x in res["launch"]],
                          "graph_us": [round(x, 2) for x in res["graph"]]}), flush=True)
        del g
        e.close()


if __name__ == "__main__":
    main()
