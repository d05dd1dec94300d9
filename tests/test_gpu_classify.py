"""Classifier pre-pass on the device (fracenc_classify.hip) against the oracle and the
reference's ClassifierTest known answers; the engine's internal −1 recomputation gives
the same search results as host-preclassified grids; and the reference's own GPU
classifier test (tests/OpenCLTest.cpp:65-111) re-expressed against the device kernel."""
import json
import os

import numpy as np
import pytest

import fractencode_amd as F
from golden_util import FIELDS, GOLD, golden, plane

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("size,off", [(2, 2), (4, 2), (8, 8), (16, 8), (32, 16), (64, 32), (7, 3), (5, 5)])
def test_device_classify_matches_oracle(oracle, size, off):
    y = plane("lenna_y")
    items = F.create_uniform_grid(512, 512, size, off)
    with F.Engine(0) as e:
        e.set_frame(y)
        got = e.classify(items)
    want = oracle.classify(y, items)
    np.testing.assert_array_equal(got["category"], want["category"])


def test_device_classify_reference_kat():
    # reference tests/ClassifierTest.cpp:24-50 on the Lenna Y plane
    y = plane("lenna_y")
    cases = [(204, 78, 2, 0), (242, 242, 2, 1), (6, 6, 2, 2), (82, 226, 2, 3), (418, 486, 2, 4), (384, 250, 2, 5),
             (136, 40, 2, -1), (184, 96, 8, 0), (472, 96, 8, -1), (320, 224, 16, 4), (416, 256, 16, -1),
             (384, 224, 32, -1), (64, 320, 32, 5), (64, 0, 64, 0), (128, 320, 64, 5)]
    items = np.zeros(len(cases), dtype=F.GRID_ITEM)
    for i, (x, yy, s, _) in enumerate(cases):
        items[i] = (x, yy, s, s, -1)
    with F.Engine(0) as e:
        e.set_frame(y)
        got = e.classify(items)
    assert list(got["category"]) == [c for *_, c in cases]


@pytest.mark.parametrize("engine", [F.ENGINE_VALU, F.ENGINE_MFMA, F.ENGINE_SEA])
def test_engine_classifies_unlabelled_items_on_device(engine):
    # categories −1 + use_classifier: the engine's device pre-pass reproduces the
    # reference goldens made with host-preclassified grids (main.cpp:155-162)
    rec, meta = golden("lenna_cls")
    p = plane("lenna_y")
    with F.Engine(0, 4, True, 0.0, -1.0, engine) as e:
        e.set_frame(p)
        e.set_domains(F.create_uniform_grid(512, 512, 16, 8))
        out, st = e.search(F.create_uniform_grid(512, 512, 8, 8))
    got = {"x": out["x"], "y": out["y"], "dx": out["dx"], "dy": out["dy"], "dw": out["sw"], "dh": out["sh"],
           "t": out["transform"], "dist": out["distance"], "s": out["contrast"], "o": out["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(got[k], rec[k], err_msg=k)
    assert st["rejected_mappings"] == meta["rejected"]


def test_device_frame_classifier_without_host_copy():
    # a CUDA-tensor frame never comes back to the host; the classifier still runs
    import torch

    rec, meta = golden("lenna_cls")
    p = plane("lenna_y")
    with F.Engine(0, 4, True) as e:
        e.set_frame(torch.from_numpy(p).cuda())
        e.set_domains(F.create_uniform_grid(512, 512, 16, 8))
        out, st = e.search(F.create_uniform_grid(512, 512, 8, 8))
    np.testing.assert_array_equal(out["dx"], rec["dx"])
    np.testing.assert_array_equal(out["transform"], rec["t"])
    assert st["rejected_mappings"] == meta["rejected"]


def opencl_test_plane():
    """tests/OpenCLTest.cpp:67-75: value (11w + 43h + 124) mod 256 on a 512² plane."""
    hh, ww = np.mgrid[0:512, 0:512]
    return ((ww * 11 + hh * 43 + 124) % 256).astype(np.uint8)


def test_reference_opencl_classify_test_on_device(oracle):
    # OpenCLTest.cpp:65-111: 4×4 items at the anisotropic offset (4, 2) (createUniformGrid with Size32u
    # size and offset), the GPU classifier's categories equal the CPU preclassify's item for item.
    # Here: the device kernel vs the reference's preclassify (tests/golden/opencl_classify.npz, made by
    # tools/make_golden.py from the unmodified reference), the host helper and the oracle.
    z = np.load(os.path.join(GOLD, "opencl_classify.npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    ref = z["items"]
    p = opencl_test_plane()
    from fractencode_amd.synth import sha256
    assert sha256(p) == meta["plane_sha256"]
    grid = F.create_uniform_grid(512, 512, (4, 4), (4, 2))
    for k in ("x", "y", "w", "h"):
        np.testing.assert_array_equal(grid[k], ref[k], err_msg=f"createUniformGrid {k}")
    assert not (ref["category"] == 0).all()  # OpenCLTest.cpp:85-87
    with F.Engine(0) as e:
        e.set_frame(p)
        dev = e.classify(grid)
    np.testing.assert_array_equal(dev["category"], ref["category"])
    np.testing.assert_array_equal(F.preclassify(p, grid)["category"], ref["category"])
    np.testing.assert_array_equal(oracle.classify(p, grid)["category"], ref["category"])


def test_classifier_pool_beyond_the_one_pass_sort(oracle):
    """A classified pool of 1,042,441 domains (8×8 at stride 2 over 2048²): 1,018 sort tiles, above
    kBkSelfTiles, so the bucket sort runs its three-launch form (count, per-bucket scan, scatter).  A strided
    sample of the ranges equals the oracle's classified search, and every winner is in its range's bucket."""
    from fractencode_amd.synth import value_noise

    W = H = 2048
    p = value_noise(W, H, 77)
    doms = F.create_uniform_grid(W, H, 8, 2)
    assert len(doms) > 512 * 1024
    rngs = F.create_uniform_grid(W, H, 4, 4)[:16384]
    with F.Engine(0, 4, True, 0.0, -1.0) as e:
        e.set_frame(p)
        e.set_domains(doms)
        e.set_ranges(rngs)
        e.run()
        out, st = e.fetch()
    assert st["rejected_mappings"] > 0
    pick = np.arange(0, len(rngs), 1024)
    rg = np.zeros(len(pick), dtype=oracle.ITEM_DTYPE)
    for k in ("x", "y", "w", "h"):
        rg[k] = rngs[k][pick]
    rg = oracle.classify(p, rg)
    want, _, _ = oracle.estimate(p, oracle.classify(p, oracle.uniform_grid(W, H, 8, 2)), rg, T=4,
                                 use_classifier=True, threads=16)
    got = out[pick]
    g = {"x": got["x"], "y": got["y"], "dx": got["dx"], "dy": got["dy"], "dw": got["sw"], "dh": got["sh"],
         "t": got["transform"], "dist": got["distance"], "s": got["contrast"], "o": got["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(g[k], want[k], err_msg=k)
