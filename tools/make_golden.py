#!/usr/bin/env python3
"""Generate the committed golden vectors under tests/golden/ from the REFERENCE.

Runs only in the build container (needs /root/reference): builds
oracle/_ref/libfracref.so from the unmodified reference sources
(oracle/ref/Makefile) and records, per fixture, the reference's per-range
winners.  Only data is written (raw planes and result arrays); no reference
source travels.  Re-run with:  python tools/make_golden.py [--only NAME ...]
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fractencode_amd.synth import value_noise, sha256  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
REF_PNG = "/root/reference/tests/input/lenna512x512.png"


class FrResult(C.Structure):
    _fields_ = [("x", C.c_uint32), ("y", C.c_uint32), ("dx", C.c_uint32), ("dy", C.c_uint32),
                ("dw", C.c_uint32), ("dh", C.c_uint32), ("transform", C.c_int32), ("pad", C.c_int32),
                ("distance", C.c_double), ("contrast", C.c_double), ("brightness", C.c_double)]


def load_ref():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle", "ref")])
    lib = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfracref.so"))
    lib.fr_estimate.restype = C.c_int
    lib.fr_estimate.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                C.c_int, C.c_double, C.c_double, C.c_int, C.c_int, C.c_void_p, C.c_size_t,
                                C.c_void_p, C.POINTER(C.c_uint64), C.c_double, C.POINTER(C.c_size_t)]
    lib.fr_decode.restype = C.c_int
    lib.fr_decode.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_double,
                              C.c_void_p, C.POINTER(C.c_double)]
    lib.fr_quantize.restype = C.c_int
    lib.fr_quantize.argtypes = [C.c_double, C.c_double, C.c_int, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
    lib.fr_rgb2yuv.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p,
                               C.c_uint32, C.c_void_p, C.c_uint32]
    lib.fr_load_yuv.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint32),
                                C.POINTER(C.c_uint32)]
    return lib


def ref_estimate(lib, plane, src_size, tgt_size, T, thr=0.0, smax=-1.0, cls=False, sel=None, threads=8):
    plane = np.ascontiguousarray(plane, dtype=np.uint8)
    H, W = plane.shape
    n_ranges = (W // tgt_size) * (H // tgt_size)
    count = n_ranges if sel is None else len(sel)
    out = (FrResult * count)()
    rej = C.c_uint64(0)
    done = C.c_size_t(0)
    sel_arr = None if sel is None else np.ascontiguousarray(sel, dtype=np.uint32)
    lib.fr_estimate(plane.ctypes.data, plane.ctypes.data, W, H, W, src_size, tgt_size, T, thr, smax, int(cls),
                    threads, None if sel_arr is None else sel_arr.ctypes.data, count, out, C.byref(rej), 0.0,
                    C.byref(done))
    a = np.frombuffer(out, dtype=np.dtype([("x", "<u4"), ("y", "<u4"), ("dx", "<u4"), ("dy", "<u4"), ("dw", "<u4"),
                                           ("dh", "<u4"), ("t", "<i4"), ("pad", "<i4"), ("dist", "<f8"),
                                           ("s", "<f8"), ("o", "<f8")])).copy()
    return a, int(rej.value)


ITEM = np.dtype([("x", "<u4"), ("y", "<u4"), ("w", "<u4"), ("h", "<u4"), ("category", "<i4")])
RESULT = np.dtype([("x", "<u4"), ("y", "<u4"), ("dx", "<u4"), ("dy", "<u4"), ("dw", "<u4"), ("dh", "<u4"),
                   ("t", "<i4"), ("pad", "<i4"), ("dist", "<f8"), ("s", "<f8"), ("o", "<f8")])


def ref_grid(lib, spec):
    """The reference's createUniformGrid(Size32u(W, H), Size32u(sw, sh), Size32u(ox, oy))."""
    lib.fr_uniform_grid.restype = C.c_size_t
    lib.fr_uniform_grid.argtypes = [C.c_uint32] * 6 + [C.c_void_p, C.c_size_t]
    n = lib.fr_uniform_grid(*spec, None, 0)
    out = np.zeros(n, ITEM)
    lib.fr_uniform_grid(*spec, out.ctypes.data, n)
    return out


def ref_estimate_items(lib, plane, dom_spec, rng_spec, T, thr=0.0, smax=-1.0, cls=False):
    """TransformEstimator2::estimate over the reference's grids of the two specs (Size32u items: any
    rectangle), categories preclassified as main.cpp:155-161 does."""
    plane = np.ascontiguousarray(plane, dtype=np.uint8)
    H, W = plane.shape
    doms, rngs = ref_grid(lib, dom_spec), ref_grid(lib, rng_spec)
    lib.fr_estimate_items.restype = C.c_int
    lib.fr_estimate_items.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                      C.c_size_t, C.c_void_p, C.c_size_t, C.c_int, C.c_double, C.c_double, C.c_int,
                                      C.c_void_p, C.POINTER(C.c_uint64)]
    out = np.zeros(len(rngs), RESULT)
    rej = C.c_uint64(0)
    lib.fr_estimate_items(plane.ctypes.data, plane.ctypes.data, W, H, W, doms.ctypes.data, len(doms),
                          rngs.ctypes.data, len(rngs), T, thr, smax, int(cls), out.ctypes.data, C.byref(rej))
    return out, int(rej.value)


def opencl_test_plane():
    """tests/OpenCLTest.cpp:67-75's synthetic plane: (11w + 43h + 124) mod 256, 512²."""
    hh, ww = np.mgrid[0:512, 0:512]
    return ((ww * 11 + hh * 43 + 124) % 256).astype(np.uint8)


def ref_rgb2yuv(lib, rgb):
    """ImageIO::rgb2yuv of the reference build → (Y [H,W], U, V [H/2, W/2])."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W = rgb.shape[:2]
    y = np.zeros((H, W), np.uint8)
    cs = W // 2 + 1  # the reference writes the odd trailing column / row's chroma past the plane
    u = np.zeros(((H + 1) // 2, cs), np.uint8)
    v = np.zeros_like(u)
    lib.fr_rgb2yuv(rgb.ctypes.data, W, H, 3 * W, y.ctypes.data, W, u.ctypes.data, cs, v.ctypes.data, cs)
    return y, np.ascontiguousarray(u[:H // 2, :W // 2]), np.ascontiguousarray(v[:H // 2, :W // 2])


def all_colours_rgb(chunk: int) -> np.ndarray:
    """Chunk k (of 4) of the 2^24 colours, colour c on the 2×2 block at ((c%2048)·2, (c//2048)·2)."""
    c = np.arange(chunk << 22, (chunk + 1) << 22, dtype=np.uint32).reshape(2048, 2048)
    rgb = np.stack([(c >> 16) & 255, (c >> 8) & 255, c & 255], -1).astype(np.uint8)
    return np.repeat(np.repeat(rgb, 2, 0), 2, 1)


def save(name, plane_ref, rec, rejected, params, extra=None):
    d = {k: rec[k] for k in ("x", "y", "dx", "dy", "dw", "dh", "t", "dist", "s", "o")}
    meta = dict(params, rejected=rejected, plane=plane_ref)
    if extra:
        meta.update(extra)
    d["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(GOLD, name + ".npz"), **d)
    print(f"  {name}: {len(rec)} ranges, rejected={rejected}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    os.makedirs(GOLD, exist_ok=True)
    lib = load_ref()
    want = (lambda n: True) if not args.only else (lambda n: n in args.only)

    # -- input planes (data only) --------------------------------------------
    y = np.zeros((512, 512), np.uint8)
    u = np.zeros((256, 256), np.uint8)
    v = np.zeros((256, 256), np.uint8)
    w = C.c_uint32()
    h = C.c_uint32()
    lib.fr_load_yuv(REF_PNG.encode(), y.ctypes.data, u.ctypes.data, v.ctypes.data, C.byref(w), C.byref(h))
    assert (w.value, h.value) == (512, 512)
    planes = {"lenna_y": y, "lenna_u": u, "lenna_v": v, "crop64": np.ascontiguousarray(y[256:320, 256:320])}
    rng = np.random.default_rng(7)
    inexact = rng.integers(0, 41, size=(64, 64), dtype=np.uint8)
    inexact[0:8, 0:8] = 255
    inexact[40:48, 24:32] = 250
    planes["inexact64"] = inexact
    yy, xx = np.mgrid[0:64, 0:64]
    planes["checker64"] = np.where(((yy // 8) + (xx // 8)) % 2 == 0, 0, 255).astype(np.uint8)
    planes["crop48"] = np.ascontiguousarray(y[256:304, 256:304])
    planes["crop60"] = np.ascontiguousarray(y[256:316, 256:316])
    planes["inexact48"] = np.ascontiguousarray(inexact[:48, :48])
    # range sides above 32 (round 4): frames that are multiples of the item sizes (partition2.hpp:119)
    planes["crop480"] = np.ascontiguousarray(y[16:496, 16:496])
    planes["crop360"] = np.ascontiguousarray(y[100:460, 60:420])
    planes["crop400"] = np.ascontiguousarray(y[56:456, 56:456])
    # Lenna RGB (the reference's own test input, decoded losslessly; checked against the
    # reference loader's planes below) and a seeded synthetic RGB frame with odd sizes
    from PIL import Image
    lrgb = np.asarray(Image.open(REF_PNG).convert("RGB"), dtype=np.uint8)
    ly, lu, lv = ref_rgb2yuv(lib, lrgb)
    assert (ly == y).all() and (lu == u).all() and (lv == v).all(), "PIL decode differs from stb_image"
    planes["lenna_rgb"] = lrgb
    if want("color"):
        srgb = np.random.default_rng(11).integers(0, 256, size=(67, 101, 3), dtype=np.uint8)
        sy, su, sv = ref_rgb2yuv(lib, srgb)
        np.savez_compressed(os.path.join(GOLD, "rgb_synth_yuv.npz"), rgb=srgb, y=sy, u=su, v=sv)
        # all 2^24 colours: digest of the reference's Y/U/V per chunk (the data itself is 48 MB)
        digests = []
        for k in range(4):
            cy, cu, cv = ref_rgb2yuv(lib, all_colours_rgb(k))
            digests.append({"y": sha256(np.ascontiguousarray(cy[::2, ::2])), "u": sha256(cu), "v": sha256(cv)})
        with open(os.path.join(GOLD, "rgb_all_colours.json"), "w") as f:
            json.dump({"layout": "tools/make_golden.py:all_colours_rgb", "chunks": digests}, f, indent=1)
        print("  colour goldens written")
    for k, p in planes.items():
        p.tofile(os.path.join(GOLD, k + ".u8"))
    manifest = {k: {"shape": list(p.shape), "sha256": sha256(p)} for k, p in planes.items()}

    # -- reference runs -------------------------------------------------------
    jobs = [
        ("crop64_t4", "crop64", dict(src=16, tgt=8, T=4)),
        ("lenna_t4", "lenna_y", dict(src=16, tgt=8, T=4)),
        ("lenna_t8", "lenna_y", dict(src=16, tgt=8, T=8)),
        ("lenna_cls", "lenna_y", dict(src=16, tgt=8, T=4, cls=True)),
        ("lenna_cls_t8", "lenna_y", dict(src=16, tgt=8, T=8, cls=True)),
        ("lenna_thr10", "lenna_y", dict(src=16, tgt=8, T=4, thr=10.0)),
        ("lenna_smax", "lenna_y", dict(src=16, tgt=8, T=4, smax=0.9)),
        ("lenna_n4", "lenna_y", dict(src=8, tgt=4, T=4)),
        ("lenna_n16", "lenna_y", dict(src=32, tgt=16, T=4)),
        ("lenna_16to4", "lenna_y", dict(src=16, tgt=4, T=4)),
        ("lenna_u_t4", "lenna_u", dict(src=16, tgt=8, T=4)),
        ("lenna_v_t4", "lenna_v", dict(src=16, tgt=8, T=4)),
        ("crop64_n2", "crop64", dict(src=4, tgt=2, T=4)),
        ("crop64_n2_t8", "crop64", dict(src=4, tgt=2, T=8)),
        ("crop64_cls", "crop64", dict(src=16, tgt=8, T=4, cls=True)),
        ("inexact64_t8", "inexact64", dict(src=16, tgt=8, T=8)),
        ("inexact64_t4", "inexact64", dict(src=16, tgt=8, T=4)),
        ("checker64_t8", "checker64", dict(src=16, tgt=8, T=8)),
        ("checker64_thr", "checker64", dict(src=16, tgt=8, T=4, thr=8200.0)),
        # geometry other than domain = 2 × range (RootMeanSquare's sampler at ratio S/n, the fit at
        # (x·S)/n: image/metrics.h:40-45, encode/transformmatcher.h:94-95,113-144)
        ("lenna_32to8", "lenna_y", dict(src=32, tgt=8, T=4)),
        ("lenna_16to4_t8", "lenna_y", dict(src=16, tgt=4, T=8)),
        ("lenna_16to4_cls", "lenna_y", dict(src=16, tgt=4, T=4, cls=True)),
        ("lenna_16to4_thr", "lenna_y", dict(src=16, tgt=4, T=4, thr=2.0)),
        ("lenna_64to16", "lenna_y", dict(src=64, tgt=16, T=4)),
        ("lenna_64to32", "lenna_y", dict(src=64, tgt=32, T=4)),
        # createUniformGrid asserts the frame is a multiple of the item size (image/partition2.hpp:119)
        ("crop48_12to8", "crop48", dict(src=12, tgt=8, T=4)),
        ("crop48_24to8_t8", "crop48", dict(src=24, tgt=8, T=8)),
        ("crop48_12to6", "crop48", dict(src=12, tgt=6, T=4)),
        ("crop48_8to3_t8", "crop48", dict(src=8, tgt=3, T=8)),
        ("crop60_20to6_cls", "crop60", dict(src=20, tgt=6, T=4, cls=True)),
        ("crop60_5to4", "crop60", dict(src=5, tgt=4, T=4)),
        ("inexact64_32to8_t8", "inexact64", dict(src=32, tgt=8, T=8)),
        ("inexact48_12to6", "inexact48", dict(src=12, tgt=6, T=4)),
        # range sides above 32 (match_generic at any size, transformmatcher.h:80-111; ΣA as u32 above
        # 16 wide, ImageStatistics.cpp:4-11): ratio 2 at 64, 48, 40 and 36, with T = 8, the classifier, a threshold
        ("lenna_128to64", "lenna_y", dict(src=128, tgt=64, T=4)),
        ("lenna_128to64_t8", "lenna_y", dict(src=128, tgt=64, T=8)),
        ("crop480_96to48_cls", "crop480", dict(src=96, tgt=48, T=4, cls=True)),
        ("crop400_80to40_thr", "crop400", dict(src=80, tgt=40, T=4, thr=110.0)),
        ("crop360_72to36_t8", "crop360", dict(src=72, tgt=36, T=8)),
    ]
    for name, pk, p in jobs:
        if not want(name):
            continue
        t0 = time.time()
        rec, rej = ref_estimate(lib, planes[pk], p["src"], p["tgt"], p["T"], p.get("thr", 0.0), p.get("smax", -1.0),
                                p.get("cls", False))
        params = dict(src=p["src"], tgt=p["tgt"], T=p["T"], thr=p.get("thr", 0.0), smax=p.get("smax", -1.0),
                      cls=p.get("cls", False), sel=None)
        save(name, pk, rec, rej, params, {"seconds": round(time.time() - t0, 2)})
        if name == "lenna_t4":
            # Frac::Quantizer on (s, o) with main.cpp:120-121's bit depths (5 / 7)
            qd = {}
            for key, bits in (("s", 5), ("o", 7)):
                v = np.ascontiguousarray(rec[key], dtype=np.float64)
                q = np.zeros(len(v), np.uint64)
                back = np.zeros(len(v), np.float64)
                lib.fr_quantize(float(v.min()), float(v.max()), bits, v.ctypes.data, len(v), q.ctypes.data,
                                back.ctypes.data)
                qd["q_" + key], qd["v_" + key] = q, back
            np.savez_compressed(os.path.join(GOLD, "lenna_t4_quant.npz"), **qd)
            print("  quantizer golden written")
            dec = np.zeros((512, 512), np.uint8)
            rms = C.c_double()
            it = lib.fr_decode(rec.ctypes.data, len(rec), 8, 512, 512, -1, 1e-5, dec.ctypes.data, C.byref(rms))
            np.savez_compressed(os.path.join(GOLD, "lenna_t4_decode.npz"), plane=dec,
                                meta=np.frombuffer(json.dumps({"iterations": it, "rms": rms.value}).encode(),
                                                   dtype=np.uint8))
            print(f"  decode: {it} iterations rms={rms.value}")

    # -- rectangular items (Size32u grids, image/partition2.hpp:13-31, 109-135) -------------------------
    # RootMeanSquare samples at (x·⌊Sw/nw⌋, y·⌊Sh/nh⌋) (metrics.h:40-45) and the fit at ((x·Sw)/nw,
    # (y·Sh)/nh) (transformmatcher.h:94-95).  A rotation of a rectangular domain samples outside its patch
    # (transform.h:96-109), up to max(Sw, Sh) from its origin in both directions: the domain grids are
    # cut to the part of the plane where those reads stay inside it (out of bounds in the reference
    # otherwise).  (grid W, H, item w, h, offset x, y)
    def cut(W, H, sw, sh, ox, oy):
        import math
        M = max(sw, sh)
        W2, H2 = W - (M - sw), H - (M - sh)
        # createUniformGrid asserts the area is a multiple of the item size and offset (partition2.hpp:119-120)
        W2 -= W2 % math.lcm(sw, ox)
        H2 -= H2 % math.lcm(sh, oy)
        return (W2, H2, sw, sh, ox, oy)

    rect_jobs = [
        ("rect64_8x4_16x16", "crop64", cut(64, 64, 16, 16, 8, 8), (64, 64, 8, 4, 8, 4), 4, False),
        ("rect64_8x4_16x8", "crop64", cut(64, 64, 16, 8, 8, 4), (64, 64, 8, 4, 8, 4), 4, False),
        ("rect64_4x8_8x16_t8", "crop64", cut(64, 64, 8, 16, 4, 8), (64, 64, 4, 8, 4, 8), 8, False),
        ("rect64_8x4_16x8_cls", "crop64", cut(64, 64, 16, 8, 8, 4), (64, 64, 8, 4, 8, 4), 4, True),
        ("rect64_8x8_16x12", "crop64", cut(64, 64, 16, 12, 8, 4), (64, 64, 8, 8, 8, 8), 4, False),
        ("rect48_6x4_12x8_thr", "crop48", cut(48, 48, 12, 8, 6, 4), (48, 48, 6, 4, 6, 4), 4, False),
        # a 16-wide, 32-tall range: ImageStatistics2::sum's u16 sum wraps (up to 130,560)
        ("rect512_16x32_32x64", "lenna_y", cut(512, 512, 32, 64, 16, 32), (512, 512, 16, 32, 16, 32), 4, False),
    ]
    for name, pk, dspec, rspec, T, cls in rect_jobs:
        if not want(name):
            continue
        t0 = time.time()
        thr = 2.0 if name.endswith("_thr") else 0.0
        rec, rej = ref_estimate_items(lib, planes[pk], dspec, rspec, T, thr=thr, cls=cls)
        save(name, pk, rec, rej, dict(src=list(dspec), tgt=list(rspec), T=T, thr=thr, smax=-1.0, cls=cls, sel=None,
                                      grids="createUniformGrid specs (W, H, w, h, ox, oy)"),
             {"seconds": round(time.time() - t0, 2)})
    # -- tests/OpenCLTest.cpp:65-111: classifier categories of 4×4 items at offset (4, 2) on its
    # synthetic plane, by the reference's preclassify (the GPU kernel there is compared with these)
    if want("opencl_classify"):
        pl = opencl_test_plane()
        items = ref_grid(lib, (512, 512, 4, 4, 4, 2))
        lib.fr_classify_items.restype = C.c_int
        lib.fr_classify_items.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_size_t]
        lib.fr_classify_items(pl.ctypes.data, 512, 512, 512, items.ctypes.data, len(items))
        assert not (items["category"] == 0).all()  # OpenCLTest.cpp:85-87
        np.savez_compressed(os.path.join(GOLD, "opencl_classify.npz"), items=items,
                            meta=np.frombuffer(json.dumps({"plane": "(11w + 43h + 124) % 256, 512x512",
                                                           "plane_sha256": sha256(pl),
                                                           "grid": [512, 512, 4, 4, 4, 2]}).encode(), dtype=np.uint8))
        print(f"  opencl_classify: {len(items)} items, categories {np.bincount(items['category'] + 1)}")

    # -- S1 4096^2 strided sample (C3 parity on a sample) ----------------------
    if want("s1_4096_sample"):
        t0 = time.time()
        s1 = value_noise(4096, 4096, 1234)
        manifest["s1_4096"] = {"shape": [4096, 4096], "sha256": sha256(s1), "generator": "value_noise(4096,4096,1234)"}
        sel = np.arange(0, 262144, 256, dtype=np.uint32)  # 1,024 ranges, range index i*256
        rec, rej = ref_estimate(lib, s1, 16, 8, 4, sel=sel)
        save("s1_4096_sample", "s1_4096", rec, rej, dict(src=16, tgt=8, T=4, thr=0.0, smax=-1.0, cls=False,
                                                         sel="arange(0,262144,256)"),
             {"seconds": round(time.time() - t0, 2)})
    if want("s1_2048_cls_sample"):
        t0 = time.time()
        s1 = value_noise(4096, 4096, 1234)[:2048, :2048].copy()
        manifest["s1_2048"] = {"shape": [2048, 2048], "sha256": sha256(s1),
                               "generator": "value_noise(4096,4096,1234)[:2048,:2048]"}
        sel = np.arange(0, 65536, 64, dtype=np.uint32)
        rec, rej = ref_estimate(lib, s1, 16, 8, 4, cls=True, sel=sel)
        save("s1_2048_cls_sample", "s1_2048", rec, rej, dict(src=16, tgt=8, T=4, thr=0.0, smax=-1.0, cls=True,
                                                             sel="arange(0,65536,64)"),
             {"seconds": round(time.time() - t0, 2)})
    # C4 levels: the quadtree's 16/8/4 level searches at 2048² with the classifier (n = 8 above)
    for name, src, tgt, nr, step in (("s1_2048_cls_n16_sample", 32, 16, 16384, 16),
                                     ("s1_2048_cls_n4_sample", 8, 4, 262144, 256)):
        if not want(name):
            continue
        t0 = time.time()
        s1 = value_noise(4096, 4096, 1234)[:2048, :2048].copy()
        sel = np.arange(0, nr, step, dtype=np.uint32)
        rec, rej = ref_estimate(lib, s1, src, tgt, 4, cls=True, sel=sel)
        save(name, "s1_2048", rec, rej, dict(src=src, tgt=tgt, T=4, thr=0.0, smax=-1.0, cls=True,
                                             sel=f"arange(0,{nr},{step})"), {"seconds": round(time.time() - t0, 2)})
    # C5: the S1 RGB frame (value_noise seeds 1234/1235/1236 as R, G, B) through the reference's
    # rgb2yuv; digests of its Y/U/V planes and reference samples of each plane's search
    if want("c5"):
        t0 = time.time()
        rgb = np.stack([value_noise(4096, 4096, 1234 + k) for k in range(3)], -1)
        cy, cu, cv = ref_rgb2yuv(lib, rgb)
        for pk, pl in (("c5_y", cy), ("c5_u", cu), ("c5_v", cv)):
            manifest[pk] = {"shape": list(pl.shape), "sha256": sha256(pl),
                            "generator": "reference rgb2yuv of stack(value_noise(4096,4096,1234+k), k<3)"}
        for pk, pl, nr, step in (("c5_y", cy, 262144, 256), ("c5_u", cu, 65536, 128), ("c5_v", cv, 65536, 128)):
            sel = np.arange(0, nr, step, dtype=np.uint32)
            rec, rej = ref_estimate(lib, pl, 16, 8, 4, sel=sel)
            save(pk + "_sample", pk, rec, rej, dict(src=16, tgt=8, T=4, thr=0.0, smax=-1.0, cls=False,
                                                    sel=f"arange(0,{nr},{step})"))
        print(f"  c5 goldens: {time.time() - t0:.1f} s")
    path = os.path.join(GOLD, "manifest.json")
    old = json.load(open(path)) if os.path.exists(path) else {}
    old.update(manifest)
    json.dump(old, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
