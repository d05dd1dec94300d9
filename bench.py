#!/usr/bin/env python3
"""Headline bench: range-blocks/s of the exhaustive range×domain search (BASELINE.json).

Workload (BASELINE.json configs[2]): one 4096×4096 grayscale frame
(synthetic S1 value noise, seed 1234), 8×8 ranges (262,144), 16×16 domains at stride 8
(261,121), the reference's 4 transforms, exhaustive (no classifier), rms threshold 0.
Ranges are sharded contiguously over ranks (fixed total work: strong scaling).

`value` is BASELINE.md's / SURVEY §8(d)'s end-to-end step, the span the reference's own timer
wraps (main.cpp:164-168, the whole Encoder2): per step the frame H2D from pinned host memory
(N > 1: each rank uploads its 1/N stripe of the rows and an RCCL all-gather assembles the frame
on every rank over xGMI), domain-pool build, search, winner fit and fp32 fallback of this
rank's shard, its 32-byte (domain, transform, s, o, rms) tuples written by the resolve — at N = 1 straight
into pinned host memory; at N > 1 (ranks on one host) each rank's resolve writes its shard's tuples into one node-shared pinned host
buffer, one 4-byte RCCL all-reduce per frame marks it complete (with ranks on several hosts: the RCCL
all-gather of the tuples + rank 0's D2H) — serial, one frame after another.  Beside it the line carries:
  phases_ms     per phase (frame H2D, frame all-gather, run = prep + search + finish, tuple exchange)
                the mean over the timed steps, MAX over ranks (phases_ms_by_rank: every rank's)
  rank_ms_per_step  every rank's own step time (ms_per_step / value are the slowest rank's)
  gather_value  N > 1: the same step with north_star's RCCL all-gather of the tuples + rank 0's D2H in place
                of the headline's node-shared host buffer (every rank's resolve writing its shard's tuples
                into one pinned buffer mapped by all; --tuples gather swaps the two: `node_value`); the
                records check `gather_equals_headline` verifies the node buffer against it in the same run
  device_value  the same search with the frame already resident in HBM and the tuples left there
                (the all-gather still runs for N > 1): the device-only rate
  stream_value  a frame stream: frame k+1's H2D on the context's copy stream overlaps frame k's search
                (one context, two plane buffers; frac_set_frame_async), tuples into pinned memory
  c5            BASELINE configs[4]: the S1 RGB 4096² frame H2D (N > 1: row stripes + all-gather),
                rgb2yuv on the device, every plane's shard searched, one all-gather of the three
                planes' tuples, D2H — range-blocks/s over Y + U + V
  roofline      the search kernel against the dense f16 MFMA peak: `achieved` = the matrix flops
                the search issues per launch (its algorithm's count) ÷ the kernel's mean duration
                over exactly the headline's timed steps (library HIP events on the kernel's stream,
                frac_timing_history); `frac_device` the same over the device-resident leg's steps;
                `direct_form` = the §8(d) direct-form op count over the same time (an
                algorithmic-equivalent rate, not a hardware fraction); `traffic` = HBM bytes per launch
                from the committed rocprofv3 PMC passes of THIS library build (null when
                profiles/pmc_search.json was taken from another build)
  arith         what `dtype` "f16" means here: exact integer arithmetic in f16 containers
  records       a digest of the gathered tuples (equal across N = 1/2/4/8 iff the shards' gathered
                records equal the single-rank run's), and the checks that each rank's slice of the
                gathered tuples is its own shard and that the legs agree
  cpu_baseline  the unmodified reference (oracle/_ref) on a bounded sample, all the host cores this
                process may use (affinity, capped by the cgroup CPU quota), CPU model recorded
  drop_in       (N = 1) the same C3 frame through the reference's own EncodingEngineCore2 with the HIP
                engine registered (oracle/ref/core_driver): the rate a reference user gets through
                its API, alone and beside its CPU engines, and with the batch-claim patch

Run:  python bench.py [--gpus N] [--steps K] [--warmup W] [--engine valu|mfma|auto]
--gpus N > 1 without WORLD_SIZE in the environment: this process launches N ranks itself
(torch.distributed.run as a child process, before anything touches the GPU) and exits with its
status; under torch.distributed.run (WORLD_SIZE set) it runs one rank per GPU over RCCL.
main() takes an engine factory, a process-group backend and the device kind: tests/bench_main_cpu.py
runs this same main() on `gloo` ranks with the oracle stand-in engine.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "range-blocks/s (1/2/4/8 GPU) + achieved HBM GB/s vs roofline, 8×8 ranges"
VALU_PEAK_TOPS = 157.3  # MI355X vector peak (MI355X_MICROARCH.md: 256 CU x 2.4 GHz x 256 op/clk)
MFMA_F16_PEAK_TFLOPS = 2500.0  # dense f16 MFMA peak (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
ARITH = ("exact integer: f16 operands are integers |x| <= 2048 (exact in f16), fp32 accumulation with every "
         "partial sum < 2^24 (guarded per tile pair), winners re-resolved in integer arithmetic, fit in fp64")
TUPLE_BYTES = 32
PHASES = ("frame_h2d", "frame_allgather", "run", "tuples")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--engine", default="auto", choices=["auto", "valu", "mfma"])
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--transforms", type=int, default=4)
    ap.add_argument("--cpu-budget", type=float, default=45.0,
                    help="cap in seconds on the CPU-baseline sample (1,024 ranges, ≈28 s at 16 threads; 0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may use")
    ap.add_argument("--alt-steps", type=int, default=2,
                    help="steps of the VALU engine (north_star's no-MFMA formulation) reported beside (0 = skip)")
    ap.add_argument("--side-steps", type=int, default=-1,
                    help="steps of the device-resident, stream, other-tuples and C5 legs (-1 = --steps, 0 = skip)")
    ap.add_argument("--tuples", default="node", choices=["node", "gather"],
                    help="N > 1: the headline's tuple exchange — ranks on one host: one node-shared host buffer every "
                         "rank's resolve writes its shard into (node); the RCCL all-gather + rank 0's download (gather, "
                         "north_star's design; always with ranks on several hosts); the other is a side leg, and the "
                         "line checks that both give the same tuples")
    ap.add_argument("--drop-in", type=int, default=1,
                    help="N = 1: time the frame through the reference's own core (oracle/_ref/core_driver; 0 = skip)")
    ap.add_argument("--out", default=None, help="also write the line to this file (rank 0)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: the process group's backend (nccl = RCCL; gloo only for tests)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="test only: every rank on GPU 0 (a one-GPU box; with --backend gloo)")
    ap.add_argument("--group", action="store_true",
                    help="test only: initialise the process group at N = 1 too and take every N > 1 path (frame "
                         "stripes, tuple exchange, node buffer, C5 all-gathers): an RCCL rehearsal on one GPU")
    ap.add_argument("--ab", action="store_true",
                    help="allow FRAC_LIB / A/B knobs in the environment (the line is then marked, not a headline)")
    return ap.parse_args(argv)


# environment knobs the library (or the package) reads that change which code runs: the headline
# refuses them (an A/B run passes --ab and is marked as such); every FRAC_* variable in effect is
# echoed into the line's config
AB_KNOBS = ("FRAC_LIB", "FRAC_MFMA_VARIANT", "FRAC_MFMA_DFT", "FRAC_DFT_WGS", "FRAC_XCD_ORDER", "FRAC_SEA_TILED",
            "FRAC_DECODE_UNFUSED")


def frac_env() -> dict:
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("FRAC_")}


def check_headline_env(args) -> list:
    knobs = [k for k in AB_KNOBS if k in os.environ]
    if knobs and not args.ab:
        raise SystemExit(f"bench.py: {', '.join(knobs)} set: the headline runs the product library with no A/B "
                         "knob (pass --ab for an A/B run)")
    return knobs


def launch_ranks(nproc: int, script: str | None = None, argv: list | None = None, env: dict | None = None) -> int:
    """`nproc` ranks on this node via torch.distributed.run (a child process; this parent never
    initialises the GPU, so no exec happens after GPU init).  Returns the launcher's exit status,
    which is non-zero when any rank failed."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ if env is None else env)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), script or os.path.abspath(__file__),
           *(sys.argv[1:] if argv is None else argv)]
    return subprocess.call(cmd, env=env)


def host_cores() -> tuple[int, dict]:
    """Threads for the CPU baseline: the CPUs this process may run on (sched_getaffinity), capped by
    the cgroup CPU quota when one is set; plus the host description recorded in the line."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except (OSError, ValueError):
            pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return threads, {"cpu_model": model, "affinity_cpus": aff, "cgroup_cpu_quota": quota}


def cpu_baseline(frame: np.ndarray, budget: float, threads: int, host: dict):
    """Reference CPU path (oracle/_ref, the unmodified reference built by oracle/ref/Makefile)
    timed on this host on SURVEY §8(d)'s sample of the same workload: the 1,024 ranges i·256 of the
    C3 frame (every ⌈n/1024⌉-th range of another frame), capped at `budget` seconds; the oracle
    restatement ("port") when the reference build is absent."""
    from oracle import oracle as O

    H, W = frame.shape
    n_ranges = (W // 8) * (H // 8)
    sel = np.arange(0, n_ranges, max(1, -(-n_ranges // 1024)), dtype=np.uint32)
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
    return {"value": done / dt, "unit": "range-blocks/s", "cores": threads, "kind": kind, **host,
            "sample": f"{done} ranges of the same {W}x{H} S1 frame (strided over all {n_ranges}), "
                      f"{threads} threads, {dt:.1f} s"}


CORE_DRIVER = os.path.join(ROOT, "oracle", "_ref", "core_driver")
# (name, CPU engines beside the HIP engine, core mode): the reference's core as compiled, and the batch-claim
# patch INTEGRATION.md §Drop-in rate proposes (HIP engines claim 4,096 ranges per lock, CPU engines one)
DROP_IN_RUNS = (("hip_only", 0, "ref"), ("cpu2_and_hip", 2, "ref"), ("cpu16_and_hip", 16, "ref"),
                ("batched_hip_only", 0, "batch:4096"), ("batched_cpu16_and_hip", 16, "batch:4096"))


def drop_in(frame: np.ndarray, timeout_s: float = 240.0) -> dict:
    """The C3 frame through the reference's own EncodingEngineCore2 (compiled unmodified, oracle/ref/Makefile)
    with one HipEncodingEngine2 registered (integration/, oracle/ref/core_driver.cpp): core.encode()'s time,
    which is what a reference user times (main.cpp:164-167), alone (--nocpu) and beside k of the reference's
    CPU engines on the one claim queue (EncodingEngine2.hpp:126-152, EncodingEngine2.cpp:12-20), and with
    the batch-claim patch.  After the timed region, in child processes (the reference never runs in this one)."""
    if not os.path.exists(CORE_DRIVER):
        return {"skipped": "oracle/_ref/core_driver not built"}
    H, W = frame.shape
    out = {"workload": f"C3 {W}x{H} S1 frame, 16x16 domains stride 8, 8x8 ranges, T=4, exhaustive, through "
                       "EncodingEngineCore2::encode with HipEncodingEngine2 on device 0",
           "timer": "value: core.encode() minus the lost-wakeup guard's hold (core_driver's tail engine); "
                    "encoder2_value: with the construction of the core and its engines (HIP runtime start, frame "
                    "and domain upload) added, the span of the reference's own timer around Encoder2 "
                    "(main.cpp:164-167)", "runs": {}}
    with tempfile.TemporaryDirectory() as td:
        plane = os.path.join(td, "c3.u8")
        frame.tofile(plane)
        for name, ncpu, mode in DROP_IN_RUNS:
            res = os.path.join(td, f"{name}.bin")
            cmd = [CORE_DRIVER, plane, str(W), str(H), "16", "8", "0", "0", "-1", res, str(ncpu), "0", mode]
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
            except subprocess.TimeoutExpired:
                out["runs"][name] = {"error": f"timeout {timeout_s} s"}
                continue
            rec = next((json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")), None)
            if r.returncode != 0 or rec is None:
                out["runs"][name] = {"error": f"exit {r.returncode}: {r.stderr[-300:]}"}
                continue
            try:
                out["runs"][name] = _drop_in_run(rec, res, ncpu, mode)
            except (KeyError, ValueError, OSError, IndexError) as exc:  # a driver of another build: recorded
                out["runs"][name] = {"error": f"unreadable result: {exc!r}"}
    return out


def _drop_in_run(rec: dict, res: str, ncpu: int, mode: str) -> dict:
    """One core_driver run's entry: its timing line `rec` and its output file `res` (records, then the trailer
    rejected, HIP ranges, one count per HIP engine, the number of HIP engines)."""
    n = rec["ranges"]
    raw = open(res, "rb").read()
    n_hip = int(np.frombuffer(raw[-8:], dtype=np.uint64)[0])
    hip_ranges = int(np.frombuffer(raw[-8 * (2 + n_hip): -8 * (1 + n_hip)], dtype=np.uint64)[0])
    return {"value": round(n / rec["drop_in_s"], 1), "unit": "range-blocks/s",
            "drop_in_s": rec["drop_in_s"], "encode_s": rec["encode_s"], "tail_hold_s": rec["tail_hold_s"],
            "records_s": rec["records_s"], "hip_search_s": rec["hip_search_s"],
            "hip_handback_s": rec["hip_handback_s"], "construct_s": rec["construct_s"],
            "hip_search_parts_s": {part: rec[f"hip_{part}_s"] for part in ("prepare", "device", "fetch")},
            "encoder2_value": round(n / (rec["drop_in_s"] + rec["construct_s"]), 1),
            "cpu_engines": ncpu, "mode": mode, "hip_ranges": hip_ranges,
            "records": int((len(raw) - 8 * (3 + n_hip)) // 64)}


def lib_sha16() -> str:
    import fractencode_amd as F

    return F.source_id()


def load_traffic(form: str):
    """HBM bytes per search launch from the committed rocprofv3 PMC summary (profiles/), corrected as
    MI355X_MICROARCH.md §HBM prescribes — only when it was measured on this library build."""
    path = os.path.join(ROOT, "profiles", "pmc_search.json")
    if not os.path.exists(path):
        return None, "no PMC summary"
    with open(path) as f:
        d = json.load(f)
    e = d.get(form)
    if e is None:
        return None, f"no PMC entry for form {form}"
    import fractencode_amd as F

    if e.get("source_id") != F.build_info()["build_id"]:
        return None, f"PMC entry is from build {e.get('source_id')}, not this library's"
    return e.get("hbm_bytes_per_launch"), e.get("source")


# ---------------------------------------------------------------------------------------------
# the step, its timing and the line's core fields: any engine object (set_frame / run /
# copy_tuples_device or fetch_tuples), any process-group backend (nccl on the GPU, gloo on the CPU)
# ---------------------------------------------------------------------------------------------

def _sync(dev) -> None:
    import torch

    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def max_over_ranks(x: float, world: int, dev) -> float:
    """The largest of every rank's `x` (the slowest rank's time)."""
    return max_vector([x], world, dev)[0]


def max_vector(xs: list, world: int, dev) -> list:
    """Element-wise maximum over ranks of a list of floats."""
    if world == 1:
        return list(xs)
    import torch
    import torch.distributed as dist

    t = torch.tensor(xs, dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def gather_floats(xs: list, world: int, dev) -> list:
    """Every rank's list of floats (rank order)."""
    if world == 1:
        return [list(xs)]
    import torch
    import torch.distributed as dist

    t = torch.tensor(xs, dtype=torch.float64, device=dev)
    out = torch.empty(world * len(xs), dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(out, t)
    return out.cpu().view(world, len(xs)).tolist()


def timed(fn, steps: int, world: int, dev) -> tuple[float, float]:
    """`steps` calls of fn bracketed by a barrier + device synchronisation on both sides; returns
    (this rank's seconds, the maximum over ranks)."""
    import torch.distributed as dist

    _sync(dev)
    if world > 1:
        dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    _sync(dev)
    if world > 1:
        dist.barrier()
    _sync(dev)
    mine = time.perf_counter() - t0
    return mine, max_over_ranks(mine, world, dev)


class PhaseClock:
    """Per-step phase marks: HIP events on torch's current stream (the engine's) on the GPU, the host clock
    on the CPU (where every step's operations are synchronous).  A phase's time is the span from the
    previous mark to its own; `means()` averages over the recorded steps (after a synchronisation)."""

    def __init__(self, dev):
        self.cuda = dev.type == "cuda"
        self.rows = []
        self._cur = None

    def _now(self):
        if self.cuda:
            import torch

            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def begin(self) -> None:
        self._cur = [("", self._now())]

    def mark(self, name: str) -> None:
        if self._cur is not None:
            self._cur.append((name, self._now()))

    def end(self) -> None:
        if self._cur is not None:
            self.rows.append(self._cur)
        self._cur = None

    def means(self) -> dict:
        acc = {k: 0.0 for k in PHASES}
        for row in self.rows:
            for (_, a), (name, b) in zip(row, row[1:]):
                acc[name] += a.elapsed_time(b) if self.cuda else (b - a) * 1e3
        n = max(1, len(self.rows))
        return {k: v / n for k, v in acc.items()}


class FrameStep:
    """The headline step (BASELINE.md "Metric"): the frame H2D from the caller's
    pinned host plane, the search of this rank's shard (frame-dependent preparation included), the
    shard's 32-byte tuples into the all-gather buffer, the all-gather (whenever a process group is
    up), and the gathered tuples D2H into rank 0's pinned host memory (the frame's result reaches the host once;
    the other ranks keep the gathered tuples on the device).  `device_resident=True`: the frame is
    not uploaded and the gathered tuples stay on the device (the device-only leg).
    `stripes` (default: with more than one rank): each rank uploads only its 1/N stripe of the frame's
    rows across its own PCIe link and one all-gather assembles the frame on every rank over xGMI,
    instead of N full 16.8 MB uploads; the frame the engine gets is the same plane.
    On the GPU the run writes its tuples itself (frac_set_tuple_sink): without a process group straight
    into the pinned output (they cross PCIe while the resolve writes them: no pack kernel and no D2H
    copy after it), with one into the all-gather buffer.
    `node_tuples` (a distributed.NodeTuples, ranks on one host): every rank's run writes its shard's tuples
    into the node's one shared host buffer (each PCIe link carries only its own shard's tuples, no tuple
    all-gather, no download of every rank's tuples by every rank), then one completion token per frame.
    `clock` (a PhaseClock): marks frame_h2d / frame_allgather / run / tuples per step."""

    def __init__(self, eng, frame, plan, rank: int, dev, device_resident: bool = False, stripes=None,
                 node_tuples=None, clock=None):
        import torch

        world = len(plan)
        self.node = None if device_resident else node_tuples
        self.stripes = (world > 1 and not device_resident) if stripes is None else bool(stripes)
        if self.stripes:
            from fractencode_amd.distributed import FrameStripes

            self.frame_stripes = FrameStripes(frame, world, rank, dev)
        if isinstance(frame, torch.Tensor):
            frame = frame.numpy()
        self.eng, self.frame, self.plan, self.rank, self.dev = eng, frame, plan, rank, dev
        self.device_resident = device_resident
        self.clock = clock
        self.sink = hasattr(eng, "set_tuple_sink") and dev.type == "cuda"
        # the assembled frame goes to the engine without a host synchronisation when the engine enqueues on
        # torch's current stream (where the all-gather leaves it): frac_set_frame_device_async (ABI 9)
        self.async_frame = False
        if self.stripes and dev.type == "cuda" and hasattr(eng, "set_frame_device_async"):
            self.async_frame = eng.stream_handle() == torch.cuda.current_stream(dev).cuda_stream
        a, b = plan[rank]
        self.n_mine = b - a
        cap = max((q - p for p, q in plan), default=0)
        self.local = torch.zeros(cap * TUPLE_BYTES, dtype=torch.uint8, device=dev)
        self.h_out = torch.empty(plan[-1][1] * TUPLE_BYTES, dtype=torch.uint8, pin_memory=dev.type == "cuda")
        self.gathered = None
        if self.node is not None:
            import torch.distributed as dist

            self.h_out = self.node.host
            self.nccl = dist.get_backend() == "nccl"
            self.token = torch.zeros(1, dtype=torch.int32, device=dev if self.nccl else "cpu")

    def _mark(self, name: str) -> None:
        if self.clock is not None:
            self.clock.mark(name)

    def __call__(self) -> None:
        if self.clock is not None:
            self.clock.begin()
        self._step()
        if self.clock is not None:
            self.clock.end()

    def _step(self) -> None:
        import torch.distributed as dist

        from fractencode_amd.distributed import gather_tuples

        if self.stripes:  # this rank's rows H2D + the all-gather (on the engine's = torch's current stream)
            full = self.frame_stripes(self._mark)
            if self.async_frame:  # the device-to-device copy ordered after the all-gather: no host wait
                self.eng.set_frame_device_async(full)
            else:
                self.eng.set_frame(full if full.is_cuda else full.numpy())
        elif not self.device_resident:
            self.eng.set_frame(self.frame)  # H2D (returns once the plane is on the device)
            self._mark("frame_h2d")
        if self.node is not None:
            self._node_step()
            return
        direct = self.sink and not self.device_resident and not dist.is_initialized() and self.n_mine > 0
        if self.sink and self.n_mine:  # the run writes the tuples: into the pinned output, or the gather buffer
            self.eng.set_tuple_sink(self.h_out.data_ptr() if direct else self.local.data_ptr())
        self.eng.run()
        self._mark("run")
        if self.sink and self.n_mine:
            self.eng.set_tuple_sink(None)
        if direct:  # one rank, no group: the tuples are already on their way into h_out
            self.gathered = None
            self._mark("tuples")
            return
        if self.local.is_cuda:  # packed on the device, on the engine's (= torch's current) stream
            if self.n_mine and not self.sink:
                self.eng.copy_tuples_device(self.local.data_ptr())
        elif self.n_mine:  # CPU backend: the engine hands back host tuples
            import torch

            t = np.ascontiguousarray(self.eng.fetch_tuples())
            self.local[: self.n_mine * TUPLE_BYTES] = torch.from_numpy(t.view(np.uint8))
        self.gathered = gather_tuples(self.local, self.plan)
        if not self.device_resident and self.rank == 0:  # the frame's tuples reach the host once: rank 0's D2H
            self.h_out.copy_(self.gathered, non_blocking=True)  # into pinned memory
        self._mark("tuples")

    def _node_step(self) -> None:
        """The run writes its shard's tuples into the node's shared host buffer (NodeTuples): on the GPU
        through the tuple sink, else copied in from the engine's host tuples; then one completion token
        per frame — a 4-byte RCCL all-reduce on the stream after the run (nccl), or a synchronisation and
        a barrier (gloo)."""
        import torch.distributed as dist

        if self.n_mine and self.sink:
            self.eng.set_tuple_sink(self.node.sink_ptr())
            self.eng.run()
            self._mark("run")
            self.eng.set_tuple_sink(None)
        else:
            self.eng.run()
            self._mark("run")
            if self.n_mine:
                self.node.put(np.ascontiguousarray(self.eng.fetch_tuples()).tobytes())
        if self.nccl:
            dist.all_reduce(self.token)
        else:
            _sync(self.dev)
            dist.barrier()
        self._mark("tuples")

    def tuples_bytes(self) -> bytes:
        """The last step's gathered tuples (after a synchronisation)."""
        src = self.gathered if self.device_resident or (self.node is None and self.rank != 0) else self.h_out
        return src.cpu().numpy().tobytes()

    def own_slice_ok(self, own: bytes) -> bool:
        """This rank's slice of the gathered tuples is its own shard's."""
        a, b = self.plan[self.rank]
        return self.tuples_bytes()[a * TUPLE_BYTES: b * TUPLE_BYTES] == own


class ColorStep:
    """C5 (BASELINE configs[4]): one RGB frame per step — its H2D from pinned host
    memory (N > 1: this rank's stripe of rows + one all-gather), ImageIO::rgb2yuv on the device
    (image/ImageIO.cpp:43-58), every plane's shard of its ranges searched on the three engines (one stream;
    the resolvers write the tuples into one buffer, plane after plane), one all-gather of the three planes'
    tuples (N > 1) and the D2H into pinned memory.  CPU engines take the host frame and hand back host tuples."""

    def __init__(self, engines, rgb, plans, rank: int, dev, stripes=None):
        import torch

        self.engines, self.plans, self.rank, self.dev = engines, plans, rank, dev
        self.world = len(plans[0])
        self.use_stripes = self.world > 1 if stripes is None else bool(stripes)
        self.cuda = dev.type == "cuda"
        H, W = rgb.shape[:2]
        self.H, self.W = H, W
        self.rgb_np = rgb if isinstance(rgb, np.ndarray) else None
        if self.cuda:
            self.rgb = rgb  # pinned host tensor [H, W, 3]
            if self.use_stripes:
                from fractencode_amd.distributed import FrameStripes

                self.stripes = FrameStripes(rgb.view(H, W * 3), self.world, rank, dev)
            else:
                self.d_rgb = torch.empty((H, W, 3), dtype=torch.uint8, device=dev)
        self.caps = [max(b - a for a, b in p) for p in plans]
        self.offs = np.concatenate([[0], np.cumsum(self.caps)]).astype(int)
        cap = int(self.offs[-1])
        self.local = torch.zeros(cap * TUPLE_BYTES, dtype=torch.uint8, device=dev)
        self.h_out = torch.empty(self.world * cap * TUPLE_BYTES, dtype=torch.uint8, pin_memory=self.cuda)
        self.out = None

    def __call__(self) -> None:
        import torch
        import torch.distributed as dist

        if self.cuda:
            if self.use_stripes:
                d_rgb = self.stripes().view(self.H, self.W, 3)
            else:
                self.d_rgb.copy_(self.rgb, non_blocking=True)
                d_rgb = self.d_rgb
            planes = self.engines[0].rgb_to_yuv(d_rgb)
        else:
            planes = self.engines[0].rgb_to_yuv(self.rgb_np)
        for e, p in zip(self.engines, planes):
            e.set_frame(p)
        for k, (e, plan) in enumerate(zip(self.engines, self.plans)):
            a, b = plan[self.rank]
            off = int(self.offs[k]) * TUPLE_BYTES
            if self.cuda and b > a:
                e.set_tuple_sink(self.local.data_ptr() + off)
            e.run()
            if self.cuda and b > a:
                e.set_tuple_sink(None)
            elif b > a:
                t = np.ascontiguousarray(e.fetch_tuples())
                self.local[off: off + (b - a) * TUPLE_BYTES] = torch.from_numpy(t.view(np.uint8))
        if dist.is_initialized():
            out = torch.empty(self.world * self.local.numel(), dtype=torch.uint8, device=self.dev)
            dist.all_gather_into_tensor(out, self.local)
        else:
            out = self.local
        self.h_out[: out.numel()].copy_(out, non_blocking=True)
        self.out = out

    def tuples_bytes(self) -> bytes:
        """The last step's tuples in plane order (Y's ranges, then U's, then V's), rank shards concatenated."""
        raw = self.h_out.numpy().tobytes() if not self.cuda else self.h_out.cpu().numpy().tobytes()
        cap = int(self.offs[-1]) * TUPLE_BYTES
        parts = []
        for k, plan in enumerate(self.plans):
            for r, (a, b) in enumerate(plan):
                base = r * cap + int(self.offs[k]) * TUPLE_BYTES
                parts.append(raw[base: base + (b - a) * TUPLE_BYTES])
        return b"".join(parts)


def headline_fields(nr_total: int, world: int, steps: int, warmup: int, elapsed_max: float) -> dict:
    """The contract's core fields from the slowest rank's time over the timed steps."""
    return {"metric": METRIC, "value": round(nr_total / (elapsed_max / steps), 1), "unit": "range-blocks/s",
            "n_gpus": world, "steps": steps, "warmup": warmup, "ms_per_step": round(1e3 * elapsed_max / steps, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None}


def digest(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()[:16]


def hip_engine(dev, transforms: int, engine_id: int, timing: bool = False):
    """The product engine factory: one fracenc context on `dev` (exhaustive, no classifier, rms 0, sMax −1)."""
    import fractencode_amd as F

    return F.Engine(dev.index, transforms, False, 0.0, -1.0, engine_id, timing=timing)


def _setup(args, backend: str, cuda: bool):
    """The process group (N > 1) and this rank's device: (world, rank, dev, ranks on one host)."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    one_host = True
    share = cuda and getattr(args, "share_gpu", False)
    if share and backend == "nccl" and world > 1:
        raise SystemExit("bench.py: --share-gpu needs --backend gloo (RCCL takes one rank per GPU)")
    if cuda:
        dev = torch.device("cuda", local if world > 1 and not share else 0)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if world > 1 or getattr(args, "group", False):
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if "MASTER_ADDR" not in os.environ:  # --group without a launcher: a one-rank group on this host
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]), RANK="0",
                              WORLD_SIZE="1")
            s.close()
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        where = [None] * world
        name = torch.cuda.get_device_name(dev) if cuda else "cpu"
        dist.all_gather_object(where, (socket.gethostname(), local, name))
        if cuda and not share and len({(h, d) for h, d, _ in where}) != world:
            raise SystemExit(f"bench.py: ranks share a GPU: {where}")
        one_host = len({h for h, _, _ in where}) == 1
    return world, rank, dev, one_host


def _node_buffer(plan, rank, dev, world):
    """A NodeTuples on every rank, or None on every rank when any rank could not map or register it (a
    Python error on one rank must not leave the others waiting in a collective)."""
    import torch
    import torch.distributed as dist

    from fractencode_amd.distributed import NodeTuples

    node, err = None, ""
    try:
        node = NodeTuples(plan, rank, dev)
    except (OSError, RuntimeError) as exc:
        err = str(exc)
    ok = torch.tensor([0 if node is None else 1], dtype=torch.int32, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 0:
        if node is not None:
            node.close()
        return None, err or "another rank could not map the node buffer"
    return node, ""


def _run_leg(step, steps: int, warmup: int, world: int, dev):
    for _ in range(warmup):
        step()
    return timed(step, steps, world, dev)


class Bench:
    """One rank's bench: the process group, the C3 grids and this rank's shard, the engine on its dedicated
    stream, and the line that the headline and each side leg (methods below) add to."""

    def __init__(self, args, engine_factory=None, backend: str | None = None, cuda: bool = True):
        import torch

        import fractencode_amd as F
        from fractencode_amd.distributed import shard_plan
        from fractencode_amd.synth import value_noise

        self.args, self.cuda, self.F = args, cuda, F
        self.product = engine_factory is None
        self.engine_factory = engine_factory or hip_engine
        self.knobs = check_headline_env(args)
        self.build = F.build_info()
        if self.product and not self.build["matches_sources"] and not args.ab:
            raise SystemExit(f"bench.py: the library was built from sources {self.build['build_id']}, these are "
                             f"{F.source_id()}: rebuild (__graft_entry__.build())")
        self.world, self.rank, self.dev, self.one_host = _setup(args, backend or args.backend, cuda)
        self.ranked = self.world > 1 or bool(getattr(args, "group", False))  # the N > 1 paths (a group exists)
        S = self.S = args.size
        self.frame = value_noise(S, S, 1234)
        self.doms = F.create_uniform_grid(S, S, 16, 8)
        rngs = F.create_uniform_grid(S, S, 8, 8)
        self.nr_total = len(rngs)
        self.plan = shard_plan(self.nr_total, self.world)
        start, stop = self.plan[self.rank]
        self.mine = rngs[start:stop]
        self.engine_id = {"auto": F.ENGINE_AUTO, "valu": F.ENGINE_VALU, "mfma": F.ENGINE_MFMA}[args.engine]
        self.side_steps = args.steps if args.side_steps < 0 else args.side_steps
        # one dedicated stream for the engine, the tuple copies and the RCCL collectives, so every copy and the
        # all-gathers are ordered after the kernels (the legacy null stream cannot be handed to the library:
        # NULL = its own stream)
        self.stream = None
        if cuda:
            self.stream = torch.cuda.Stream(self.dev)
            torch.cuda.set_stream(self.stream)
        self.eng = self.new_engine(timing=True)
        self.h_frame = torch.from_numpy(self.frame)
        if cuda:
            self.h_frame = self.h_frame.pin_memory()  # the caller's plane, in pinned host memory
        self.eng.set_frame(self.h_frame.numpy())
        self.eng.set_domains(self.doms)
        self.eng.set_ranges(self.mine)
        self.checks = {}
        self.line = {}

    def new_engine(self, timing: bool = False):
        e = self.engine_factory(self.dev, self.args.transforms, self.engine_id, timing)
        if self.stream is not None:
            e.set_stream(self.stream.cuda_stream)
        return e

    def per_step(self, seconds: float, steps: int, n: int | None = None) -> dict:
        n = self.nr_total if n is None else n
        return {"value": round(n / (seconds / steps), 1), "ms_per_step": round(1e3 * seconds / steps, 3),
                "steps": steps}

    # ---- the headline: the end-to-end step ----
    def headline(self) -> None:
        args, world, rank, dev, eng = self.args, self.world, self.rank, self.dev, self.eng
        use_node = self.ranked and self.one_host and args.tuples == "node"
        node, node_err = (_node_buffer(self.plan, rank, dev, world) if use_node else (None, ""))
        clock = PhaseClock(dev)
        step = FrameStep(eng, self.h_frame, self.plan, rank, dev, stripes=self.ranked, node_tuples=node, clock=clock)
        for _ in range(args.warmup):
            step()
        _sync(dev)
        clock.rows = []
        eng.timing_history()  # drop the warmup runs: the history now covers exactly the timed steps
        mine_s, elapsed = timed(step, args.steps, world, dev)
        hist = eng.timing_history()  # per-run HIP events of the K timed steps (on the kernel's stream)
        # the library keeps the last 256 runs: with more steps the mean is over the last 256 of them
        assert len(hist) == min(args.steps, 256), (len(hist), args.steps)
        self.main_out, st = eng.fetch()  # the timed steps' records (the SEA engine is checked against them)
        self.gathered = step.tuples_bytes()
        self.own = eng.fetch_tuples().tobytes() if len(self.mine) else b""
        self.checks["own_slice_in_gather"] = step.own_slice_ok(self.own)
        phases = clock.means()
        phases.update({k: float(np.mean(hist["ms_" + k])) if len(hist) else 0.0 for k in ("prep", "search", "finish")})
        keys = list(PHASES) + ["prep", "search", "finish"]
        by_rank = gather_floats([phases[k] for k in keys], world, dev)
        rank_s = [r[0] for r in gather_floats([mine_s], world, dev)]
        if node is not None:
            del step
            node.close()
        self.engine_name = {1: "valu", 2: "mfma"}.get(st["engine"], "valu")
        self.form = self.F.FORM_NAMES.get(st["search_form"], self.engine_name)
        self.tuples_out = "node" if use_node and not node_err else ("gather" if self.ranked else "sink")
        S, nr_total, n_d = self.S, self.nr_total, len(self.doms)
        line = self.line
        line.update(headline_fields(nr_total, world, args.steps, args.warmup, elapsed))
        line.update({
            "dtype": "u16" if self.engine_name == "valu" else "f16",
            "arith": ARITH if self.engine_name == "mfma" else "exact integer (u16 x u16 -> u32 dot products), fit in "
                                                             "fp64",
            "data": "synthetic",
            "config": {"workload": f"C3: {S}x{S} S1 value-noise frame (seed 1234), 8x8 ranges ({nr_total}), "
                                   f"16x16 domains stride 8 ({n_d}), T={args.transforms}, exhaustive, rms 0",
                       "engine": self.engine_name, "ranges_per_gpu": len(self.mine), "parallelism": f"ranges/{world}",
                       "env": frac_env(), "ab_run": bool(self.knobs)},
            "step": ("frame H2D (pinned, 16 MiB) + pool build + search + fit + 32-byte tuples written by the resolve "
                     "into pinned host memory" if not self.ranked else
                     "frame H2D of the rank's 1/N stripe of rows (pinned) + RCCL all-gather of the frame + pool build "
                     "+ search + fit of the rank's shard + " +
                     ("its 32-byte tuples written by the resolve into the node's shared pinned tuple buffer + a "
                      "4-byte RCCL all-reduce per frame" if self.tuples_out == "node" else
                      "32-byte tuples written by the resolve into the all-gather buffer + RCCL all-gather + the "
                      "gathered tuples D2H into rank 0's pinned memory")) +
                    "; serial, barrier + synchronisation around the timed steps, slowest rank",
            "tuples_out": self.tuples_out,
            "rank_ms_per_step": [round(1e3 * s / args.steps, 3) for s in rank_s],
            "roofline": self.roofline(hist, st),
            "search_form": self.form,
            "phases_ms": {k: round(v, 3) for k, v in zip(keys, max_vector([phases[k] for k in keys], world, dev))},
            "phases_ms_by_rank": [{k: round(v, 3) for k, v in zip(keys, row)} for row in by_rank],
            "phases_note": "frame_h2d / frame_allgather / run / tuples: spans between marks on the engine's stream "
                           "(the tuple exchange includes the D2H); prep / search / finish: the library's events "
                           "inside run; each the mean over the timed steps, phases_ms the maximum over ranks",
            "fallback_ranges": st["fallback_ranges"],
            "source_id": lib_sha16(),
            "build": self.build,  # the loaded library's compiled-in id (frac_build_id): the binary that ran
        })
        if node_err:
            line["node_error"] = node_err
        if self.tuples_out == "node":
            line["tuples_note"] = ("the node-shared buffer had run only on one GPU before this line (ADVICE r05): "
                                   "records.gather_equals_headline checks it here against the RCCL all-gather leg")

    def roofline(self, hist, st) -> dict:
        """The search kernel against its roofline: the work one launch issues ÷ its mean duration over the
        timed steps (library HIP events on the kernel's stream)."""
        kernel_ms = float(np.mean(hist["ms_search"]))
        self.direct_ops = 2 * 64 * self.args.transforms * len(self.doms) * len(self.mine)
        traffic, traffic_src = load_traffic(self.form) if self.product else (None, "stand-in engine")
        if self.engine_name == "mfma":
            # the matrix flops the search issues: the Fourier form's own count (6 MFMA 32x32x16 per
            # 32-range × 32-domain tile pair), fewer than the direct form's §8(d) count for the same result
            self.work = st["matrix_flops"]
            bound, self.peak, unit = "mfma", MFMA_F16_PEAK_TFLOPS, "TFLOP/s"
        else:
            self.work = self.direct_ops
            bound, self.peak, unit = "valu", VALU_PEAK_TOPS, "TOP/s"
        achieved = self.work / (kernel_ms * 1e-3) / 1e12 if kernel_ms > 0 else 0.0
        roof = {"bound": bound, "achieved": round(achieved, 2), "peak": self.peak, "unit": unit,
                "frac": round(achieved / self.peak, 4), "traffic": traffic,
                "kernel": {"fourier": "search_dft", "direct": "search_mfma"}.get(self.form, "search_valu"),
                "kernel_ms": round(kernel_ms, 3),
                "kernel_ms_timed_steps": [round(float(x), 3) for x in hist["ms_search"]],
                "flops_per_launch": int(self.work),
                "direct_form": {"ops_per_launch": self.direct_ops,
                                "rate": round(self.direct_ops / (kernel_ms * 1e-3) / 1e12, 2) if kernel_ms > 0 else 0.0,
                                "note": "SURVEY §8(d) direct-form count over the same kernel time: an "
                                        "algorithmic-equivalent rate, not a hardware fraction"}}
        if traffic:
            roof["hbm_gbs"] = round(traffic / (kernel_ms * 1e-3) / 1e9, 3)
            roof["hbm_frac"] = round(roof["hbm_gbs"] / HBM_PEAK_GBS, 6)
            roof["traffic_source"] = traffic_src
        else:
            roof["traffic_note"] = traffic_src
        return roof

    # ---- side legs ----
    def other_tuples_leg(self) -> None:
        """N > 1: the other tuple exchange, timed the same way (north_star's all-gather beside the node buffer)."""
        world, rank, dev = self.world, self.rank, self.dev
        other = "gather" if self.tuples_out == "node" else "node"
        onode, oerr = (None, "")
        if other == "node":
            onode, oerr = (_node_buffer(self.plan, rank, dev, world) if self.one_host else
                           (None, "ranks on several hosts"))
        if other == "gather" or onode is not None:
            ostep = FrameStep(self.eng, self.h_frame, self.plan, rank, dev, stripes=True, node_tuples=onode)
            _, osec = _run_leg(ostep, self.side_steps, 1, world, dev)
            self.checks[f"{other}_equals_headline"] = ostep.tuples_bytes() == self.gathered
            self.line[f"{other}_value"] = {**self.per_step(osec, self.side_steps), "tuples_out": other}
            del ostep
            if onode is not None:
                onode.close()
        else:
            self.line[f"{other}_value"] = {"skipped": oerr}

    def device_leg(self) -> None:
        """The device-only rate: the frame resident in HBM, the gathered tuples left on the device."""
        import torch

        eng, ss = self.eng, self.side_steps
        self.d_frame = torch.from_numpy(self.frame).to(self.dev)
        eng.set_frame(self.d_frame if self.cuda else self.frame)
        dstep = FrameStep(eng, None, self.plan, self.rank, self.dev, device_resident=True)
        dstep()
        eng.timing_history()
        _, dsec = timed(dstep, ss, self.world, self.dev)
        dhist = eng.timing_history()
        self.checks["device_leg_equals_e2e"] = dstep.tuples_bytes() == self.gathered
        self.line["device_value"] = {**self.per_step(dsec, ss),
                                     "step": "the same with the frame resident in HBM before timing and the gathered "
                                             "tuples left on the device"}
        if len(dhist):
            dk = float(np.mean(dhist["ms_search"]))
            if dk > 0:
                roof = self.line["roofline"]
                roof["kernel_ms_device"] = round(dk, 3)
                roof["frac_device"] = round(self.work / (dk * 1e-3) / 1e12 / self.peak, 4)

    def stream_leg(self) -> None:
        """A frame stream on one context: each frame's H2D runs on the context's own copy stream into its second
        plane buffer while the previous frame searches (frac_set_frame_async, ABI 9); the context's stream waits
        for the upload and runs, the resolve writing the frame's tuples into one of two pinned buffers (per rank,
        no gather).  CPU stand-in engines: the same frames in turn."""
        import torch

        eng, ss, mine = self.eng, self.side_steps, self.mine
        pin = self.cuda
        h_tup = [torch.zeros(max(1, len(mine)) * TUPLE_BYTES, dtype=torch.uint8) for _ in range(2)]
        if pin:
            h_tup = [t.pin_memory() for t in h_tup]
            h_frame = self.h_frame.numpy()  # pinned: the upload is asynchronous

            def stream_steps():
                for k in range(ss):
                    eng.set_frame_async(h_frame)
                    if len(mine):
                        eng.set_tuple_sink(h_tup[k & 1].data_ptr())
                    eng.run()
                eng.set_tuple_sink(None)
        else:
            def stream_steps():
                for k in range(ss):
                    eng.set_frame(self.frame)
                    eng.run()
                    if len(mine):
                        eng.fetch_tuples(h_tup[k & 1].numpy().view(self.F.TUPLE))

        stream_steps()
        eng.timing_history()
        _, ssec = timed(stream_steps, 1, self.world, self.dev)
        shist = eng.timing_history()
        self.checks["stream_leg_equals_e2e"] = h_tup[(ss - 1) & 1].numpy().tobytes()[: len(self.own)] == self.own
        self.line["stream_value"] = {
            **self.per_step(ssec, ss),
            "step": "per frame: H2D on the context's copy stream into its second plane buffer, overlapped with the "
                    "previous frame's kernels + search + tuples written by the resolve into pinned memory" +
                    (" (per rank, no gather)" if self.ranked else ""),
            "phases_ms": {k: round(float(np.mean(shist["ms_" + k])), 3) if len(shist) else 0.0
                          for k in ("prep", "search", "finish")}}
        eng.set_frame(self.d_frame if self.cuda else self.frame)
        eng.run()

    def c5_leg(self) -> None:
        """C5 (BASELINE configs[4]): three planes of an S1 RGB frame, each plane's ranges sharded the same way."""
        import torch

        from fractencode_amd.distributed import shard_plan
        from fractencode_amd.synth import value_noise

        F, S, ss, rank = self.F, self.S, self.side_steps, self.rank
        rgb = np.stack([value_noise(S, S, 1234 + k) for k in range(3)], -1)
        h_rgb = torch.from_numpy(rgb)
        if self.cuda:
            h_rgb = h_rgb.pin_memory()
        sizes = [(S, S), (S // 2, S // 2), (S // 2, S // 2)]
        c5_rngs = [F.create_uniform_grid(w, h, 8, 8) for w, h in sizes]
        c5_plans = [shard_plan(len(r), self.world) for r in c5_rngs]
        c5_eng = [self.new_engine() for _ in range(3)]
        for e, (w, h), r, p in zip(c5_eng, sizes, c5_rngs, c5_plans):
            a, b = p[rank]
            e.set_frame(np.zeros((h, w), np.uint8))
            e.set_domains(F.create_uniform_grid(w, h, 16, 8))
            e.set_ranges(r[a:b])
        cstep = ColorStep(c5_eng, h_rgb if self.cuda else rgb, c5_plans, rank, self.dev, stripes=self.ranked)
        _, csec = _run_leg(cstep, ss, 1, self.world, self.dev)
        n5 = sum(len(r) for r in c5_rngs)
        self.line["c5"] = {
            **self.per_step(csec, ss, n5), "unit": "range-blocks/s",
            "workload": f"C5: S1 RGB {S}x{S} (seeds 1234/1235/1236) -> Y {S}x{S}, U/V {S // 2}x{S // 2}, 8x8 ranges "
                        f"({n5}), 16x16 domains stride 8, T={self.args.transforms}, exhaustive",
            "step": "RGB H2D (N > 1: row stripes + RCCL all-gather) + rgb2yuv on the device + the three planes' shards "
                    "searched on one stream + one all-gather of their tuples + D2H",
            "records": {"tuples_sha16": digest(cstep.tuples_bytes()), "n": n5}}
        for e in c5_eng:
            e.close()

    def alt_engines(self) -> None:
        """The same workload on the other engines, frame resident, measured the same way: the VALU engine
        (packed-u16 v_dot2, north_star's no-MFMA formulation, exhaustive) and the SEA engine (successive
        elimination: identical records, most candidates skipped by an exact bound, data-dependent)."""
        import torch

        F, dev, args = self.F, self.dev, self.args
        d_frame = torch.from_numpy(self.frame).to(dev)
        out = self.line["alt_engines"] = {}
        for alt_name, alt_id in (("valu", F.ENGINE_VALU), ("sea", F.ENGINE_SEA)):
            with F.Engine(dev.index, args.transforms, False, 0.0, -1.0, alt_id, timing=True) as alt:
                alt.set_stream(self.stream.cuda_stream)
                alt.set_frame(d_frame)
                alt.set_domains(self.doms)
                alt.set_ranges(self.mine)
                alt.run()
                torch.cuda.synchronize(dev)
                alt.timing_history()
                t0 = time.perf_counter()
                for _ in range(args.alt_steps):
                    alt.run()
                torch.cuda.synchronize(dev)
                alt_sec = (time.perf_counter() - t0) / args.alt_steps
                ah = alt.timing_history()
                alt_out, ast = alt.fetch()
            a_ms = float(np.mean(ah["ms_search"]))
            entry = {"value": round(self.nr_total / alt_sec, 1), "ms_per_step": round(alt_sec * 1e3, 3),
                     "steps": args.alt_steps, "dtype": "u16", "step": "device-resident (as device_value)",
                     "phases_ms": {k: round(float(np.mean(ah["ms_" + k])), 3) for k in ("prep", "search", "finish")}}
            if alt_name == "valu":
                alt_ach = self.direct_ops / (a_ms * 1e-3) / 1e12
                entry["roofline"] = {"bound": "valu", "achieved": round(alt_ach, 2), "peak": VALU_PEAK_TOPS,
                                     "unit": "TOP/s", "frac": round(alt_ach / VALU_PEAK_TOPS, 4),
                                     "kernel_ms": round(a_ms, 3)}
            else:
                entry["records_identical_to_exhaustive"] = bool(alt_out.tobytes() == self.main_out.tobytes())
                entry["evaluated_frac"] = round(ast["evaluated_mappings"] / (len(self.mine) * len(self.doms)), 6)
            out[alt_name] = entry

    def run(self) -> dict:
        import torch.distributed as dist

        args, world, rank = self.args, self.world, self.rank
        self.headline()
        if self.side_steps > 0:
            if self.ranked:
                self.other_tuples_leg()
            self.device_leg()
            self.stream_leg()
            self.c5_leg()
        self.line["records"] = {"tuples_sha16": digest(self.gathered), "n": self.nr_total, **self.checks}
        if world == 1 and self.engine_name == "mfma" and args.alt_steps > 0 and self.product:
            self.alt_engines()
        if rank == 0 and world == 1 and args.cpu_budget > 0:
            threads, host = host_cores()
            self.line["cpu_baseline"] = cpu_baseline(self.frame, args.cpu_budget, args.cpu_threads or threads, host)
        if rank == 0 and world == 1 and self.cuda and self.product and args.drop_in:
            self.line["drop_in"] = drop_in(self.frame)
        self.eng.close()
        if rank == 0:
            print(json.dumps(self.line), flush=True)
            if args.out:
                with open(args.out, "w") as f:
                    json.dump(self.line, f)
        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
        return self.line


def main(args, engine_factory=None, backend: str | None = None, cuda: bool = True) -> dict:
    """The bench on this rank.  `engine_factory(dev, transforms, engine_id, timing)` builds an engine (default:
    the HIP library's), `backend` the process group's (default --backend: nccl = RCCL), `cuda` whether ranks own a
    GPU; the CPU tests pass the oracle stand-in, gloo and False.  Rank 0 prints the line and returns it."""
    return Bench(args, engine_factory, backend, cuda).run()


if __name__ == "__main__":
    _args = parse()
    if _args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(_args.gpus))
    main(_args)
