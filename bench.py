#!/usr/bin/env python3
"""Headline bench: range-blocks/s of the exhaustive range×domain search (BASELINE.json).

Workload (BASELINE.json configs[2]): one 4096×4096 grayscale frame
(synthetic S1 value noise, seed 1234), 8×8 ranges (262,144), 16×16 domains at stride 8
(261,121), the reference's 4 transforms, exhaustive (no classifier), rms threshold 0.
A step = one full search of the frame's ranges already resident in HBM: domain-pool
build, search, winner fit, fp32 fallback and — for N > 1 — the RCCL all-gather of the
32-byte (domain, transform, s, o, rms) winner tuples.  Ranges are sharded contiguously over ranks (fixed total work:
strong scaling).

Run:  python bench.py [--gpus N] [--steps K] [--warmup W] [--engine valu|mfma|auto]
N > 1 is launched by torch.distributed.run (one process per GPU, RCCL over xGMI).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "range-blocks/s (1/2/4/8 GPU) + achieved HBM GB/s vs roofline, 8×8 ranges"
VALU_PEAK_TOPS = 157.3  # MI355X vector peak (MI355X_MICROARCH.md: 256 CU x 2.4 GHz x 256 op/clk)
MFMA_F16_PEAK_TFLOPS = 2500.0  # dense f16 MFMA peak (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--engine", default="auto", choices=["auto", "valu", "mfma"])
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--transforms", type=int, default=4)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline sampling (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--alt-steps", type=int, default=2,
                    help="steps of the VALU engine (north_star's no-MFMA formulation) reported beside (0 = skip)")
    return ap.parse_args()


def cpu_baseline(frame: np.ndarray, budget: float, threads: int):
    """Reference CPU path (oracle/_ref, the unmodified reference built by oracle/ref/Makefile)
    timed on this host on a bounded strided sample of the same workload; the oracle
    restatement ("port") when the reference build is absent."""
    from oracle import oracle as O

    H, W = frame.shape
    n_ranges = (W // 8) * (H // 8)
    sel = np.arange(0, n_ranges, max(1, n_ranges // 4096), dtype=np.uint32)
    t0 = time.perf_counter()
    if O.ref_lib() is not None:
        _, _, done = O.ref_estimate(frame, 16, 8, 4, sel=sel, threads=threads, budget_s=budget)
        kind = "reference"
    else:
        doms = O.uniform_grid(W, H, 16, 8)
        rngs = O.uniform_grid(W, H, 8, 8)[sel]
        _, _, done = O.estimate(frame, doms, rngs, T=4, threads=threads, budget_s=budget)
        kind = "port"
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "range-blocks/s", "cores": threads, "kind": kind,
            "sample": f"{done} ranges of the same {W}x{H} S1 frame (strided over all {n_ranges}), "
                      f"{threads} threads, {dt:.1f} s"}


def load_traffic(engine_name: str):
    """HBM bytes per search launch from the committed rocprofv3 PMC summary (profiles/),
    corrected as MI355X_MICROARCH.md §HBM prescribes; None when absent."""
    path = os.path.join(ROOT, "profiles", "pmc_search.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    e = d.get(engine_name)
    return None if e is None else e.get("hbm_bytes_per_launch")


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import fractencode_amd as F
    from fractencode_amd.distributed import TUPLE_BYTES, gather_tuples, shard_bounds, shard_capacity
    from fractencode_amd.synth import value_noise

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    S = args.size
    frame = value_noise(S, S, 1234)
    doms = F.create_uniform_grid(S, S, 16, 8)
    rngs = F.create_uniform_grid(S, S, 8, 8)
    nr_total = len(rngs)
    per = shard_capacity(nr_total, world)
    start, stop = shard_bounds(nr_total, world, rank)
    mine = rngs[start:stop]
    engine_id = {"auto": F.ENGINE_AUTO, "valu": F.ENGINE_VALU, "mfma": F.ENGINE_MFMA}[args.engine]

    # one dedicated stream for the engine and the RCCL gather, so the all-gather is ordered after
    # the record copy (the legacy null stream cannot be handed to the library: NULL = its own stream)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng = F.Engine(dev.index, args.transforms, False, 0.0, -1.0, engine_id, timing=True)
    eng.set_stream(stream.cuda_stream)
    d_frame = torch.from_numpy(frame).to(dev)  # the frame is resident in HBM before timing
    eng.set_frame(d_frame)
    eng.set_domains(doms)
    eng.set_ranges(mine)
    mine_bytes = torch.zeros(per * TUPLE_BYTES, dtype=torch.uint8, device=dev)

    def step():
        eng.run()
        if world > 1:  # RCCL all-gather of the 32-byte (domain, t, s, o, rms) tuples (same stream)
            eng.copy_tuples_device(mine_bytes.data_ptr())
            gather_tuples(mine_bytes, nr_total, world)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    search_ms = []
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    # per-kernel device times of the last step (library HIP events on this stream)
    _, st = eng.fetch()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # separate timed pass for the dominant kernel's average duration (HIP events around
    # the search kernel on the stream it is launched on, recorded by the library)
    for _ in range(max(3, min(args.steps, 10))):
        eng.run()
        _, st_i = eng.fetch()
        search_ms.append(st_i["ms_search"])
    avg_search_ms = float(np.mean(search_ms))

    ms_per_step = 1000.0 * elapsed / args.steps
    value = nr_total / (elapsed / args.steps)
    engine_name = {1: "valu", 2: "mfma"}.get(st["engine"], "valu")
    n_d = len(doms)
    ops_per_rb = 2 * 64 * args.transforms * n_d  # one MAC per pixel per candidate
    ops_per_launch = ops_per_rb * len(mine)
    achieved = ops_per_launch / (avg_search_ms * 1e-3) / 1e12
    if engine_name == "mfma":
        bound, peak, unit = "mfma", MFMA_F16_PEAK_TFLOPS, "TFLOP/s"
    else:
        bound, peak, unit = "valu", VALU_PEAK_TOPS, "TOP/s"
    traffic = load_traffic(F.FORM_NAMES.get(st["search_form"], engine_name))
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "range-blocks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u16" if engine_name == "valu" else "f16",
        "data": "synthetic",
        "config": {"workload": f"C3: {S}x{S} S1 value-noise frame (seed 1234), 8x8 ranges ({nr_total}), "
                               f"16x16 domains stride 8 ({n_d}), T={args.transforms}, exhaustive, rms 0",
                   "engine": engine_name, "ranges_per_gpu": len(mine), "parallelism": f"ranges/{world}"},
        "roofline": {"bound": bound, "achieved": round(achieved, 2), "peak": peak, "unit": unit,
                     "frac": round(achieved / peak, 4), "traffic": traffic,
                     "kernel": "search", "kernel_ms": round(avg_search_ms, 3),
                     "ops_per_launch": ops_per_launch},
        "search_form": F.FORM_NAMES.get(st["search_form"], "?"),
        "phases_ms": {"prep": round(st["ms_prep"], 3), "search": round(st["ms_search"], 3),
                      "finish": round(st["ms_finish"], 3)},
        "fallback_ranges": st["fallback_ranges"],
    }
    if st["matrix_flops"]:
        # the matrix-core work the search actually issued (the Fourier form needs 3/8 of the
        # §8(d) direct-form count): the hardware utilisation beside the algorithmic figure
        issued = st["matrix_flops"] / (avg_search_ms * 1e-3) / 1e12
        line["roofline"]["issued"] = {"flops_per_launch": st["matrix_flops"], "achieved": round(issued, 2),
                                      "frac": round(issued / MFMA_F16_PEAK_TFLOPS, 4)}
    if traffic:
        line["roofline"]["hbm_gbs"] = round(traffic / (avg_search_ms * 1e-3) / 1e9, 3)
        line["roofline"]["hbm_frac"] = round(line["roofline"]["hbm_gbs"] / HBM_PEAK_GBS, 6)
    if world == 1 and engine_name == "mfma" and args.alt_steps > 0:
        # the same workload on the other engines, measured the same way: the VALU engine (packed-u16
        # v_dot2, north_star's no-MFMA formulation, exhaustive) and the SEA engine (successive
        # elimination: identical records, most candidates skipped by an exact bound, data-dependent)
        line["alt_engines"] = {}
        for alt_name, alt_id in (("valu", F.ENGINE_VALU), ("sea", F.ENGINE_SEA)):
            with F.Engine(dev.index, args.transforms, False, 0.0, -1.0, alt_id, timing=True) as alt:
                alt.set_stream(stream.cuda_stream)
                alt.set_frame(d_frame)
                alt.set_domains(doms)
                alt.set_ranges(mine)
                alt.run()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(args.alt_steps):
                    alt.run()
                torch.cuda.synchronize(dev)
                alt_sec = (time.perf_counter() - t0) / args.alt_steps
                alt_out, ast = alt.fetch()
            entry = {"value": round(nr_total / alt_sec, 1), "ms_per_step": round(alt_sec * 1e3, 3),
                     "steps": args.alt_steps, "dtype": "u16",
                     "phases_ms": {"prep": round(ast["ms_prep"], 3), "search": round(ast["ms_search"], 3),
                                   "finish": round(ast["ms_finish"], 3)}}
            if alt_name == "valu":
                alt_ach = ops_per_launch / (ast["ms_search"] * 1e-3) / 1e12
                entry["roofline"] = {"bound": "valu", "achieved": round(alt_ach, 2), "peak": VALU_PEAK_TOPS,
                                     "unit": "TOP/s", "frac": round(alt_ach / VALU_PEAK_TOPS, 4),
                                     "kernel_ms": round(ast["ms_search"], 3)}
            else:
                main_out, _ = eng.fetch()
                entry["records_identical_to_exhaustive"] = bool(alt_out.tobytes() == main_out.tobytes())
                entry["evaluated_frac"] = round(ast["evaluated_mappings"] / (len(mine) * n_d), 6)
            line["alt_engines"][alt_name] = entry
    if rank == 0 and world == 1 and args.cpu_budget > 0:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        line["cpu_baseline"] = cpu_baseline(frame, args.cpu_budget, threads)
    eng.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
