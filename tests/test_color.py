"""Colour conversion oracle (fracoracle.c or_rgb2yuv ← image/ImageIO.cpp:43-58), CPU only.

Pinned against the reference build three ways: the Lenna planes its loader produced
(tests/golden/lenna_{y,u,v}.u8 from ImageIO::loadImage), a seeded odd-sized RGB frame
(rgb_synth_yuv.npz) and digests of its output on all 2^24 colours (rgb_all_colours.json).
"""
import json

import numpy as np
import pytest

from color_util import all_colours_rgb
from fractencode_amd.synth import sha256
from golden_util import GOLD, plane


def test_oracle_rgb2yuv_lenna(oracle):
    y, u, v = oracle.rgb2yuv(plane("lenna_rgb"))
    np.testing.assert_array_equal(y, plane("lenna_y"))
    np.testing.assert_array_equal(u, plane("lenna_u"))
    np.testing.assert_array_equal(v, plane("lenna_v"))


def test_oracle_rgb2yuv_odd_sizes(oracle):
    z = np.load(f"{GOLD}/rgb_synth_yuv.npz")
    y, u, v = oracle.rgb2yuv(z["rgb"])
    assert z["rgb"].shape[:2] == (67, 101)
    for got, k in ((y, "y"), (u, "u"), (v, "v")):
        np.testing.assert_array_equal(got, z[k], err_msg=k)


@pytest.mark.parametrize("chunk", range(4))
def test_oracle_rgb2yuv_all_colours(oracle, chunk):
    want = json.load(open(f"{GOLD}/rgb_all_colours.json"))["chunks"][chunk]
    y, u, v = oracle.rgb2yuv(all_colours_rgb(chunk))
    assert sha256(np.ascontiguousarray(y[::2, ::2])) == want["y"]
    assert sha256(u) == want["u"] and sha256(v) == want["v"]


def test_fma_contraction_matters(oracle):
    # the unfused form differs from the reference on some grey levels:
    # the oracle must not be the unfused one
    g = np.arange(256, dtype=np.float64)
    unfused = np.floor(0.299 * g + 0.587 * g + 0.114 * g).astype(np.uint8)
    rgb = np.repeat(np.arange(256, dtype=np.uint8), 3).reshape(1, 256, 3)
    y, _, _ = oracle.rgb2yuv(np.repeat(rgb, 2, 0))
    assert (y[0] != unfused).any()
    assert (y[0] <= np.arange(256)).all()
