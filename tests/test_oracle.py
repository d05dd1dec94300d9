"""Pins the CPU oracle (oracle/fracoracle.c) before it is trusted as the checker:
  * bit-exact against every golden vector generated from the unmodified reference
    (tests/golden/, tools/make_golden.py), including rejected-mapping counts;
  * the reference's own known-answer tests re-expressed
    (tests/TransformMatcherTest.cpp, TransformEstimatorTest.cpp, ImageSamplerTest.cpp,
    ImageStatisticsTest.cpp, ClassifierTest.cpp, PartitionTests.cpp of the reference).
"""
import os

import numpy as np
import pytest

from golden_util import FIELDS, GOLDEN_NAMES, golden, make_grids, plane, selection


def _grids(O, p, meta):
    # main.cpp:155-162: preclassify on the (source) plane for both grids
    return make_grids(O.uniform_grid, O.classify, p, meta)


# Large fixtures are checked on a strided subset here (the full check is `slow`).
_SUBSET = {"s1_4096_sample": 16, "s1_2048_cls_sample": 8, "lenna_n4": 4, "lenna_16to4": 4, "lenna_16to4_t8": 8,
           "lenna_16to4_cls": 4, "lenna_16to4_thr": 4, "c5_y_sample": 16, "c5_u_sample": 8, "c5_v_sample": 8,
           "s1_2048_cls_n16_sample": 8, "s1_2048_cls_n4_sample": 8}


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_oracle_matches_reference_goldens(oracle, name):
    rec, meta = golden(name)
    p = plane(meta["plane"])
    doms, rngs = _grids(oracle, p, meta)
    sel = selection(meta, len(rngs))
    idx = np.arange(len(rngs)) if sel is None else sel
    step = _SUBSET.get(name, 1)
    pick = np.arange(0, len(idx), step)
    out, rej, _ = oracle.estimate(p, doms, rngs[idx[pick]], T=meta["T"], thr=meta["thr"], smax=meta["smax"],
                                  use_classifier=meta["cls"])
    for k in FIELDS:
        np.testing.assert_array_equal(out[k], rec[k][pick], err_msg=f"{name}:{k}")
    if step == 1 and sel is None:
        assert rej == meta["rejected"]


@pytest.mark.slow
@pytest.mark.skipif(not os.environ.get("FRAC_SLOW"), reason="full large-fixture oracle check: set FRAC_SLOW=1")
@pytest.mark.parametrize("name", [n for n in GOLDEN_NAMES if n in _SUBSET])
def test_oracle_matches_reference_goldens_full(oracle, name):
    rec, meta = golden(name)
    p = plane(meta["plane"])
    doms, rngs = _grids(oracle, p, meta)
    sel = selection(meta, len(rngs))
    idx = np.arange(len(rngs)) if sel is None else sel
    out, rej, _ = oracle.estimate(p, doms, rngs[idx], T=meta["T"], thr=meta["thr"], smax=meta["smax"],
                                  use_classifier=meta["cls"])
    for k in FIELDS:
        np.testing.assert_array_equal(out[k], rec[k], err_msg=f"{name}:{k}")
    if sel is None:
        assert rej == meta["rejected"]


def test_decode_matches_reference(oracle):
    rec, meta = golden("lenna_t4")
    z = np.load("tests/golden/lenna_t4_decode.npz")
    import json
    dmeta = json.loads(bytes(z["meta"]).decode())
    r = np.zeros(len(rec["x"]), dtype=oracle.RESULT_DTYPE)
    for k in FIELDS:
        r[k] = rec[k]
    dec, it, rms = oracle.decode(r, 8, 512, 512)
    assert it == dmeta["iterations"] and rms == dmeta["rms"]
    np.testing.assert_array_equal(dec, z["plane"])


# --- the reference's own known-answer tests ------------------------------------

def _item(x, y, w, h=None, cat=-1):
    from oracle.oracle import ITEM_DTYPE
    return np.array([(x, y, w, w if h is None else h, cat)], dtype=ITEM_DTYPE)


def test_kat_transform_matcher(oracle):
    # reference tests/TransformMatcherTest.cpp:13-35
    src = np.array([[1, 1, 2, 2, 40, 41, 50, 51], [1, 1, 2, 2, 40, 41, 50, 51], [3, 3, 4, 4, 70, 71, 80, 81],
                    [3, 3, 4, 4, 70, 71, 80, 81], [0] * 8, [1] * 8, [0] * 8, [1] * 8], np.uint8)
    tgt = np.array([[2, 4, 40, 50], [1, 3, 70, 80], [0, 0, 0, 0], [1, 1, 1, 1]], np.uint8)
    out, _, _ = oracle.estimate(src, _item(0, 0, 4), _item(0, 0, 2), T=4, thr=0.0, smax=100.0, tgt=tgt)
    assert out["dist"][0] == 0.0
    assert out["t"][0] == 3  # Rotate_270
    assert out["s"][0] < 1.0 and out["o"][0] < 1.0


def test_kat_transform_estimator(oracle):
    # reference tests/TransformEstimatorTest.cpp:14-47
    src = np.array([[1, 1, 2, 2, 40, 41, 50, 51], [1, 1, 2, 2, 40, 41, 50, 51], [3, 3, 4, 4, 70, 71, 80, 81],
                    [3, 3, 4, 4, 70, 71, 80, 81], [10, 10, 10, 10, 0, 0, 0, 0], [11, 11, 11, 11, 1, 1, 1, 1],
                    [10, 10, 10, 10, 0, 0, 0, 0], [11, 11, 11, 11, 1, 1, 1, 1]], np.uint8)
    tgt = np.array([[40, 50, 2, 4], [70, 80, 1, 3], [0, 0, 10, 10], [1, 1, 11, 11]], np.uint8)
    doms = oracle.uniform_grid(8, 8, 4, 2)
    rngs = oracle.uniform_grid(4, 4, 2, 2)
    out, _, _ = oracle.estimate(src, doms, rngs, T=4, thr=0.0, smax=100.0, tgt=tgt)
    expected = {(0, 0): (4, 0), (2, 0): (0, 0), (0, 2): (4, 4), (2, 2): (0, 4)}
    got = {(int(r["x"]), int(r["y"])): (int(r["dx"]), int(r["dy"])) for r in out}
    assert got == expected


def test_kat_image_sampler_via_estimate(oracle):
    # reference tests/ImageSamplerTest.cpp:13-45: SamplerBilinear on 2×2 / 4×4 patches.
    # The oracle's sampler is exercised through a 1-pixel-range match whose
    # distance is (r − sample)²/(domain area); choose r = 0 so dist·area = sample².
    img = np.array([[1, 1, 2, 2, 3, 3, 4, 4], [5, 5, 6, 6, 7, 7, 8, 8], [9, 9, 10, 10, 11, 11, 12, 12],
                    [13, 13, 14, 14, 15, 15, 16, 16], [17, 17, 18, 18, 19, 19, 20, 20],
                    [21, 21, 22, 22, 23, 23, 24, 24], [25, 25, 26, 26, 27, 27, 28, 28],
                    [29, 29, 30, 30, 31, 31, 32, 32]], np.uint8)
    zero = np.zeros((1, 1), np.uint8)

    def sample(x, y, size, t):
        # domain size×size, range 1×1: ratio = size; sample at (0,0) of the domain
        out, _, _ = oracle.estimate(img, _item(x, y, size), _item(0, 0, 1), T=8, thr=-1.0, tgt=zero)
        # T=8 chain keeps the LAST minimum; read the sample of one transform by
        # running the chain with a single domain and checking the min — instead
        # compute through the distance of each transform individually:
        return out

    # Per-transform samples: compute distance for each transform by making the
    # chain see only one transform value — use T=4/8 and compare with the closed form.
    def expect(x, y, size, t):
        # transform.h:96-109 offsets for local (0,0)
        from oracle.oracle import lib  # noqa: F401
        a = [(1, 0, 0, 0, 0, 1, 0, 0), (0, 1, 0, 0, -1, 0, 1, 0), (-1, 0, 1, 0, 0, -1, 0, 1), (0, -1, 0, 1, 1, 0, 0, 0),
             (1, 0, 0, 0, 0, -1, 0, 1), (0, 1, 0, 0, 1, 0, 0, 0), (-1, 0, 1, 0, 0, 1, 0, 0),
             (0, -1, 0, 1, -1, 0, 1, 0)][t]
        px = x + a[2] * (size - 1) + a[3] * (size - 1)
        py = y + a[6] * (size - 1) + a[7] * (size - 1)
        pts = [(px, py), (px + a[0], py + a[4]), (px + a[1], py + a[5]), (px + a[0] + a[1], py + a[4] + a[5])]
        return sum(int(img[v, u]) for u, v in pts) / 4.0

    # the reference's expected values (ImageSamplerTest.cpp:29-45)
    assert expect(0, 0, 2, 0) == (1 + 1 + 5 + 5) / 4.0
    assert expect(1, 0, 2, 0) == (1 + 2 + 5 + 6) / 4.0
    assert expect(3, 3, 2, 0) == (14 + 15 + 18 + 19) / 4.0
    assert expect(3, 6, 2, 0) == (26 + 27 + 30 + 31) / 4.0
    assert expect(0, 0, 4, 0) == (1 + 1 + 5 + 5) / 4.0
    assert expect(0, 0, 4, 3) == (2 + 2 + 6 + 6) / 4.0
    assert expect(0, 0, 4, 4) == (9 + 9 + 13 + 13) / 4.0
    assert expect(3, 4, 4, 0) == (18 + 19 + 22 + 23) / 4.0
    assert expect(3, 4, 4, 1) == (26 + 27 + 30 + 31) / 4.0
    assert expect(3, 4, 4, 2) == (27 + 28 + 31 + 32) / 4.0
    assert expect(3, 4, 4, 3) == (19 + 20 + 23 + 24) / 4.0
    assert expect(3, 4, 4, 4) == (26 + 27 + 30 + 31) / 4.0
    # and the oracle's sampler agrees: min over the 8 transforms of sample² / area
    for (x, y, size) in [(0, 0, 2), (1, 0, 2), (3, 3, 2), (0, 0, 4), (3, 4, 4)]:
        out = sample(x, y, size, 0)
        vals = [expect(x, y, size, t) for t in range(8)]
        best = min(v * v for v in vals)
        assert out["dist"][0] == best / (size * size)
        # chain keeps the later transform on ties
        assert out["t"][0] == max(t for t in range(8) if vals[t] ** 2 == best)


def test_kat_image_statistics_and_classifier(oracle):
    # reference tests/ClassifierTest.cpp:24-50 on the Lenna Y plane
    y = plane("lenna_y")
    expected = {
        2: [(204, 78, 0), (242, 242, 1), (6, 6, 2), (82, 226, 3), (418, 486, 4), (384, 250, 5), (136, 40, -1)],
        4: [(416, 336, 5), (440, 336, 0), (448, 336, 1), (504, 336, 2), (316, 340, 3), (336, 340, 4), (400, 340, -1)],
        8: [(184, 96, 0), (192, 96, 1), (264, 96, 2), (368, 96, 3), (400, 96, 4), (440, 96, 5), (472, 96, -1)],
        16: [(320, 224, 4), (80, 240, 5), (416, 256, -1), (464, 256, 0), (0, 272, 1), (96, 272, 2), (112, 272, 3)],
        32: [(384, 224, -1), (448, 224, 0), (0, 256, 1), (96, 256, 2), (160, 256, 3), (288, 256, 4), (64, 320, 5)],
        64: [(64, 0, 0), (192, 64, 1), (448, 128, 2), (256, 192, 3), (256, 256, 4), (128, 320, 5)],
    }
    for size, items in expected.items():
        for x, yy, cat in items:
            assert oracle.category(y, x, yy, size) == cat, (size, x, yy)


def test_kat_partition(oracle):
    # reference tests/PartitionTests.cpp:13-31
    assert len(oracle.uniform_grid(512, 512, 32, 32)) == (512 // 32) ** 2
    g = oracle.uniform_grid(64, 64, 16, 8)
    assert len(g) == 49
    assert list(g["x"][:8]) == [0, 8, 16, 24, 32, 40, 48, 0]
    assert list(g["y"][:8]) == [0] * 7 + [8]
