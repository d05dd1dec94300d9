"""The C++ host layer (include/fracenc.hpp): tests/cpp/host_test drives EncodingEngineCore
(two engines claiming 1,000-range batches), the device classifier, Quantizer<double>, the
decoder, frame streaming (setFrameAsync) with 32-byte tuples, per-run timings and the quadtree's
32-byte leaves from C++ with no Python in the loop; its output is compared here with the reference
goldens and with the Python layer's results on the same library."""
import json
import os
import subprocess

import numpy as np
import pytest

import fractencode_amd as F
from golden_util import FIELDS, GOLD, golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "host_test")


def _build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])
    return BIN


def test_cpp_host_layer_builds_and_links():
    b = _build()
    r = subprocess.run([b], capture_output=True, text=True)  # usage: no device call
    assert r.returncode == 2 and "usage" in r.stderr


def _chunks(path):
    raw = open(path, "rb").read()
    out, i = [], 0
    while i < len(raw):
        n = int(np.frombuffer(raw[i:i + 8], np.uint64)[0])
        out.append(raw[i + 8:i + 8 + n])
        i += 8 + n
    return out


def _fields(items):
    return {"x": items["x"], "y": items["y"], "dx": items["dx"], "dy": items["dy"], "dw": items["sw"],
            "dh": items["sh"], "t": items["transform"], "dist": items["distance"], "s": items["contrast"],
            "o": items["brightness"]}


@pytest.mark.gpu
def test_cpp_host_layer_matches_reference(tmp_path):
    out = tmp_path / "host.bin"
    r = subprocess.run([_build(), ROOT, str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    c = _chunks(out)
    t4 = np.frombuffer(c[0], dtype=F.ENCODE_ITEM)
    rej = int(np.frombuffer(c[1], np.uint64)[0])
    rec, meta = golden("lenna_t4")
    for k, v in _fields(t4).items():
        np.testing.assert_array_equal(v, rec[k], err_msg=k)
    assert rej == meta["rejected"]
    cls = np.frombuffer(c[2], dtype=F.ENCODE_ITEM)
    rej_c = int(np.frombuffer(c[3], np.uint64)[0])
    rec, meta = golden("lenna_cls")
    for k, v in _fields(cls).items():
        np.testing.assert_array_equal(v, rec[k], err_msg="cls " + k)
    assert rej_c == meta["rejected"]
    q = np.load(os.path.join(GOLD, "lenna_t4_quant.npz"))
    codes = np.frombuffer(c[4], np.uint64)
    values = np.frombuffer(c[5], np.float64)
    n = len(t4)
    np.testing.assert_array_equal(codes[:n], q["q_s"])
    np.testing.assert_array_equal(codes[n:], q["q_o"])
    np.testing.assert_array_equal(values[:n], q["v_s"])
    np.testing.assert_array_equal(values[n:], q["v_o"])
    d = np.load(os.path.join(GOLD, "lenna_t4_decode.npz"))
    dmeta = json.loads(bytes(d["meta"]).decode())
    np.testing.assert_array_equal(np.frombuffer(c[6], np.uint8).reshape(512, 512), d["plane"])
    assert int(np.frombuffer(c[7], np.int32)[0]) == dmeta["iterations"]
    assert float(np.frombuffer(c[8], np.float64)[0]) == dmeta["rms"]
    # 5. frame streaming: every streamed frame's tuples equal its synchronous search's, and frame 0's equal the
    # Python layer's tuples for the golden frame
    nr = len(t4)
    sync_t = np.frombuffer(c[9], dtype=F.TUPLE)
    async_t = np.frombuffer(c[10], dtype=F.TUPLE)
    assert len(sync_t) == len(async_t) == 3 * nr
    assert sync_t.tobytes() == async_t.tobytes()
    y = np.fromfile(os.path.join(GOLD, "lenna_y.u8"), np.uint8).reshape(512, 512)
    with F.Engine(0, 4) as e:
        e.set_frame(y)
        e.set_domains(F.create_uniform_grid(512, 512, 16, 8))
        e.search(F.create_uniform_grid(512, 512, 8, 8))
        assert e.fetch_tuples().tobytes() == sync_t[:nr].tobytes()
    assert not np.array_equal(sync_t[:nr], sync_t[nr:2 * nr])  # the frames differ
    # 6. one timing entry per streamed run
    assert int(np.frombuffer(c[11], np.uint64)[0]) == 3
    # 7. the quadtree leaves equal the Python layer's
    with F.Engine(0, 4, True) as e:
        e.set_frame(y)
        want, _ = e.encode_quadtree(16, 4, 4.0, leaves=True)
    assert np.frombuffer(c[12], dtype=F.QT_LEAF).tobytes() == want.tobytes()
