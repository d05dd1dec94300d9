"""The reference-side binding (integration/HipEncodingEngine2.hpp) as a compiled fact.

CPU: the binding compiles against the reference's own headers (/root/reference), its
static_asserts pinning frac_* to UniformGridItem / transform_score_t / item_match_t /
encode_item_t (sizes and field offsets), and the driver that runs it exists.
GPU: the reference's EncodingEngineCore2 (encode/EncodingEngine2.cpp, compiled unmodified by
oracle/ref/Makefile into oracle/_ref/core_driver) runs with the HIP engine in the engine slot of
EncodingEngine2.cpp:21-29 — alone (--nocpu) and beside the reference's CPU engines sharing the one
claim queue (the CLI default) — and the records it returns equal the reference goldens,
rejected-mapping counts included, for the classic 16→8, the classifier and the CLI's default 16→4.
A geometry the engine refuses fails its finalize(); the failure comes back on the caller's thread
(rethrowIfFailed), not as std::terminate on the core's worker.  Without a device the engine's
constructor throws where EncodingEngine2.cpp:27-29 catches ("failed to create engine").
"""
import json
import os
import subprocess

import numpy as np
import pytest

import fractencode_amd as F
from golden_util import FIELDS, GOLD, golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
DRIVER = os.path.join(ROOT, "oracle", "_ref", "core_driver")


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference sources exist only in the build container")
def test_binding_compiles_against_reference_headers(tmp_path):
    src = tmp_path / "tu.cpp"
    src.write_text('#include "HipEncodingEngine2.hpp"\n'
                   "static_assert(sizeof(Frac2::HipEncodingEngine2) > sizeof(Frac2::AbstractEncodingEngine2));\n"
                   "int main() { return 0; }\n")
    subprocess.check_call(["g++", "-std=gnu++20", "-fsyntax-only", "-Wall", "-Wno-deprecated-declarations",
                           "-include", "mutex", "-include", "condition_variable", "-include", "sstream",
                           f"-I{REF}", f"-I{REF}/thirdparty/gsl/include", f"-I{ROOT}/include",
                           f"-I{ROOT}/integration", str(src)])
    assert os.path.exists(DRIVER), "oracle/_ref/core_driver not built (__graft_entry__.build)"


def _run_core(tmp_path, plane_name, W, H, src, tgt, cls, cpu=False, check=True, devices=None, per_engine=False,
              mode=None):
    out = tmp_path / f"core_{src}_{tgt}_{cls}_{int(cpu)}.bin"
    plane_path = plane_name if os.path.isabs(plane_name) else os.path.join(GOLD, plane_name + ".u8")
    # cpu: 2 of the reference's CPU engines beside the HIP engine(s) on the core's queue (core_driver's usage note)
    r = subprocess.run([DRIVER, plane_path, str(W), str(H), str(src), str(tgt), str(int(cls)), "0", "-1", str(out),
                        str(2 if cpu else 0)] + ([devices or "0"] if devices or mode else []) + ([mode] if mode else []),
                       timeout=300, capture_output=True, text=True)
    if not check:
        return r
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    # the timing line (bench.py's drop_in reads it): core.encode()'s time, and the tail engine's hold that
    # closes the reference core's lost-wakeup window (0 in the batch-claim mode, which has no tail)
    timing = next(json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{"))
    assert timing["mode"] == (mode or "ref").split(":")[0]
    assert 0 < timing["records_s"] <= timing["encode_s"] and timing["drop_in_s"] > 0
    assert (timing["tail_hold_s"] >= 0.02) if timing["mode"] == "ref" else timing["tail_hold_s"] == 0
    raw = out.read_bytes()
    # trailer: rejected, HIP ranges, one count per HIP engine, the number of HIP engines (u64 each)
    k = int(np.frombuffer(raw[-8:], dtype=np.uint64)[0])
    n = (len(raw) - 8 * (3 + k)) // 64
    rec = np.frombuffer(raw[: n * 64], dtype=F.ENCODE_ITEM)
    tail = [int(v) for v in np.frombuffer(raw[n * 64:], dtype=np.uint64)]
    rejected, hip_ranges, each = tail[0], tail[1], tail[2:2 + k]
    assert sum(each) == hip_ranges
    rec = rec[np.lexsort((rec["x"], rec["y"]))]
    return (rec, rejected, hip_ranges, each) if per_engine else (rec, rejected, hip_ranges)


@pytest.mark.skipif(not os.path.exists(DRIVER), reason="oracle/_ref/core_driver not built")
def test_engine_creation_failure_is_caught_by_the_reference_core(tmp_path):
    # no device here: HipEncodingEngine2's constructor throws inside EncodingEngine2.cpp:21-29's try
    # block, the reference logs "failed to create engine" and the driver reports it (exit 4)
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    r = _run_core(tmp_path, "lenna_y", 512, 512, 16, 8, False, check=False)
    assert r.returncode == 4, (r.returncode, r.stdout, r.stderr)
    assert "failed to create engine" in r.stdout and "frac_create" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("cpu", [False, True], ids=["hip_only", "cpu_and_hip"])
@pytest.mark.parametrize("name,src,tgt,cls", [("lenna_t4", 16, 8, False), ("lenna_cls", 16, 8, True),
                                              ("lenna_16to4", 16, 4, False)])
def test_reference_core_with_hip_engine_matches_goldens(tmp_path, name, src, tgt, cls, cpu):
    assert os.path.exists(DRIVER), "oracle/_ref/core_driver must be built in the build container"
    if cpu and name == "lenna_16to4":
        pytest.skip("the CPU engines' share of 16,384 4×4 ranges is slow on the box's CPUs; 16→8 covers the queue")
    rec, meta = golden(name)
    got, rejected, hip_ranges = _run_core(tmp_path, "lenna_y", 512, 512, src, tgt, cls, cpu=cpu)
    assert len(got) == len(rec["x"])
    if cpu:  # both kinds of engine claimed ranges from the one queue (EncodingEngine2.hpp:131-140)
        assert 0 < hip_ranges < len(got), hip_ranges
    else:
        assert hip_ranges == len(got)
    fields = {"x": got["x"], "y": got["y"], "dx": got["dx"], "dy": got["dy"], "dw": got["sw"], "dh": got["sh"],
              "t": got["transform"], "dist": got["distance"], "s": got["contrast"], "o": got["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(fields[k], rec[k], err_msg=f"{name}: {k}")
    assert rejected == meta["rejected"]


@pytest.mark.gpu
def test_hip_engine_failure_comes_back_on_the_callers_thread(tmp_path):
    # 16×16 ranges against 8×8 domains (the CLI refuses them, main.cpp:99; the driver does not check): the
    # engine's constructor accepts the domain grid, frac_search fails inside finalize() on the core's worker
    # thread ("domains must be wider than the ranges", metrics.h:39's FRAC_ASSERT); the binding keeps the error
    # and the driver's rethrowIfFailed() reports it after the workers joined (exit 6), where a throw on the
    # worker would have been std::terminate (SIGABRT)
    r = _run_core(tmp_path, "lenna_y", 512, 512, 8, 16, False, check=False)
    assert r.returncode == 6, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "HIP engine failed" in r.stderr and "domains must be wider than the ranges" in r.stderr
    assert "1024 ranges without a record" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("cpu", [False, True], ids=["hips_only", "cpu_and_hips"])
@pytest.mark.parametrize("name,cls", [("lenna_t4", False), ("lenna_cls", True)])
def test_reference_core_with_two_hip_engines_on_one_queue(tmp_path, name, cls, cpu):
    """Two HipEncodingEngine2 registered in the reference's core (two contexts on device 0 — the one-GPU
    box's stand-in for one engine per device) claim ranges from the core's
    one queue (EncodingEngine2.hpp:126-168), with and without the CPU engines beside them: each HIP
    engine searched ranges, and the records and reject count equal the reference goldens."""
    assert os.path.exists(DRIVER), "oracle/_ref/core_driver must be built in the build container"
    rec, meta = golden(name)
    got, rejected, hip_ranges, each = _run_core(tmp_path, "lenna_y", 512, 512, 16, 8, cls, cpu=cpu, devices="0,0",
                                                per_engine=True)
    assert len(each) == 2 and all(c > 0 for c in each), each
    assert len(got) == len(rec["x"])
    assert (hip_ranges < len(got)) if cpu else (hip_ranges == len(got))
    fields = {"x": got["x"], "y": got["y"], "dx": got["dx"], "dy": got["dy"], "dw": got["sw"], "dh": got["sh"],
              "t": got["transform"], "dist": got["distance"], "s": got["contrast"], "o": got["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(fields[k], rec[k], err_msg=f"{name}: {k}")
    assert rejected == meta["rejected"]


@pytest.mark.gpu
@pytest.mark.parametrize("cpu", [False, True], ids=["hip_only", "cpu_and_hip"])
def test_batch_claim_core_matches_goldens(tmp_path, cpu):
    """The maintainer patch INTEGRATION.md §Drop-in rate proposes (core_driver MODE batch:K: HIP engines claim
    K ranges per lock, CPU engines one, a join instead of the predicate-less wait), over the same engines:
    the records and reject counts are the reference goldens', like the reference's own core."""
    rec, meta = golden("lenna_t4")
    got, rejected, hip_ranges = _run_core(tmp_path, "lenna_y", 512, 512, 16, 8, False, cpu=cpu, mode="batch:256")
    assert len(got) == len(rec["x"])
    assert (0 < hip_ranges < len(got)) if cpu else (hip_ranges == len(got))
    fields = {"x": got["x"], "y": got["y"], "dx": got["dx"], "dy": got["dy"], "dw": got["sw"], "dh": got["sh"],
              "t": got["transform"], "dist": got["distance"], "s": got["contrast"], "o": got["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(fields[k], rec[k], err_msg=k)
    assert rejected == meta["rejected"]
