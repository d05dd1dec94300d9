"""The reference-side binding (integration/HipEncodingEngine2.hpp) as a compiled fact.

CPU: the binding compiles against the reference's own headers (/root/reference), its
static_asserts pinning frac_* to UniformGridItem / transform_score_t / item_match_t /
encode_item_t (sizes and field offsets), and the driver that runs it exists.
GPU: the reference's EncodingEngineCore2 (encode/EncodingEngine2.cpp, compiled unmodified by
oracle/ref/Makefile into oracle/_ref/core_driver) runs with --nocpu and the HIP engine in the
engine slot of EncodingEngine2.cpp:21-29; the records it returns equal the reference goldens,
rejected-mapping counts included — for the classic 16→8, the classifier, and the CLI's default 16→4.
"""
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


def _run_core(tmp_path, plane_name, W, H, src, tgt, cls):
    out = tmp_path / f"core_{src}_{tgt}_{cls}.bin"
    subprocess.run([DRIVER, os.path.join(GOLD, plane_name + ".u8"), str(W), str(H), str(src), str(tgt), str(int(cls)),
                    "0", "-1", str(out)], check=True, timeout=300)
    raw = out.read_bytes()
    n = (len(raw) - 8) // 64
    rec = np.frombuffer(raw[: n * 64], dtype=F.ENCODE_ITEM)
    rejected = int(np.frombuffer(raw[n * 64:], dtype=np.uint64)[0])
    return rec[np.lexsort((rec["x"], rec["y"]))], rejected


@pytest.mark.gpu
@pytest.mark.parametrize("name,src,tgt,cls", [("lenna_t4", 16, 8, False), ("lenna_cls", 16, 8, True),
                                              ("lenna_16to4", 16, 4, False)])
def test_reference_core_with_hip_engine_matches_goldens(tmp_path, name, src, tgt, cls):
    assert os.path.exists(DRIVER), "oracle/_ref/core_driver must be built in the build container"
    rec, meta = golden(name)
    got, rejected = _run_core(tmp_path, "lenna_y", 512, 512, src, tgt, cls)
    assert len(got) == len(rec["x"])
    fields = {"x": got["x"], "y": got["y"], "dx": got["dx"], "dy": got["dy"], "dw": got["sw"], "dh": got["sh"],
              "t": got["transform"], "dist": got["distance"], "s": got["contrast"], "o": got["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(fields[k], rec[k], err_msg=f"{name}: {k}")
    assert rejected == meta["rejected"]
