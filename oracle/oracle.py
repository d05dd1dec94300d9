"""ctypes binding of the CPU oracle (fracoracle.c) and the reference build.

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline — never by the
product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_LIB_PATH = os.path.join(HERE, "_ref", "libfracref.so")

ITEM_DTYPE = np.dtype([("x", "<u4"), ("y", "<u4"), ("w", "<u4"), ("h", "<u4"), ("category", "<i4")])
RESULT_DTYPE = np.dtype([("x", "<u4"), ("y", "<u4"), ("dx", "<u4"), ("dy", "<u4"), ("dw", "<u4"), ("dh", "<u4"),
                         ("t", "<i4"), ("pad", "<i4"), ("dist", "<f8"), ("s", "<f8"), ("o", "<f8")])

_lib = None
_ref = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.or_category.restype = C.c_int
        L.or_category.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
        L.or_uniform_grid.restype = C.c_size_t
        L.or_uniform_grid.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_size_t]
        L.or_uniform_grid2.restype = C.c_size_t
        L.or_uniform_grid2.argtypes = [C.c_uint32] * 6 + [C.c_void_p, C.c_size_t]
        L.or_estimate.restype = C.c_int
        L.or_estimate.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t, C.c_void_p,
                                  C.c_size_t, C.c_int, C.c_double, C.c_double, C.c_int, C.c_int, C.c_void_p,
                                  C.POINTER(C.c_uint64), C.c_double, C.POINTER(C.c_size_t)]
        L.or_decode.restype = C.c_int
        L.or_decode.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_double,
                                C.c_void_p, C.POINTER(C.c_double)]
        _lib = L
    return _lib


def category(plane: np.ndarray, x: int, y: int, w: int, h: int | None = None) -> int:
    plane = np.ascontiguousarray(plane, dtype=np.uint8)
    return lib().or_category(plane.ctypes.data, plane.shape[1], x, y, w, w if h is None else h)


def uniform_grid(W: int, H: int, size, offset) -> np.ndarray:
    """createUniformGrid; size / offset an int or (x, y) (the reference's Size32u)."""
    sw, sh = (size, size) if np.isscalar(size) else size
    ox, oy = (offset, offset) if np.isscalar(offset) else offset
    n = lib().or_uniform_grid2(W, H, sw, sh, ox, oy, None, 0)
    out = np.zeros(n, dtype=ITEM_DTYPE)
    lib().or_uniform_grid2(W, H, sw, sh, ox, oy, out.ctypes.data, n)
    return out


def classify(plane: np.ndarray, items: np.ndarray) -> np.ndarray:
    """preclassify callback of main.cpp:155-159 (categories from `plane`)."""
    items = items.copy()
    for i in range(len(items)):
        items["category"][i] = category(plane, int(items["x"][i]), int(items["y"][i]), int(items["w"][i]),
                                        int(items["h"][i]))
    return items


def estimate(src: np.ndarray, domains: np.ndarray, ranges: np.ndarray, T: int = 4, thr: float = 0.0,
             smax: float = -1.0, use_classifier: bool = False, threads: int = 8, tgt: np.ndarray | None = None,
             budget_s: float = 0.0):
    """Oracle TransformEstimator2::estimate over `ranges`; returns (records, rejected, n_done)."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    tgt = src if tgt is None else np.ascontiguousarray(tgt, dtype=np.uint8)
    domains = np.ascontiguousarray(domains, dtype=ITEM_DTYPE)
    ranges = np.ascontiguousarray(ranges, dtype=ITEM_DTYPE)
    out = np.zeros(len(ranges), dtype=RESULT_DTYPE)
    rej = C.c_uint64(0)
    done = C.c_size_t(0)
    rc = lib().or_estimate(src.ctypes.data, src.shape[1], tgt.ctypes.data, tgt.shape[1], domains.ctypes.data,
                           len(domains), ranges.ctypes.data, len(ranges), T, thr, smax, int(use_classifier), threads,
                           out.ctypes.data, C.byref(rej), budget_s, C.byref(done))
    if rc != 0:
        raise RuntimeError(f"or_estimate failed: {rc}")
    return out, int(rej.value), int(done.value)


def decode(records: np.ndarray, range_size: int, W: int, H: int, max_iter: int = -1, eps: float = 1e-5,
           initial: np.ndarray | None = None):
    records = np.ascontiguousarray(records, dtype=RESULT_DTYPE)
    plane = np.zeros((H, W), np.uint8) if initial is None else np.ascontiguousarray(initial, np.uint8).copy()
    rms = C.c_double()
    it = lib().or_decode(records.ctypes.data, len(records), range_size, W, H, max_iter, eps, plane.ctypes.data,
                         C.byref(rms))
    return plane, it, rms.value


def rgb2yuv(rgb: np.ndarray):
    """ImageIO::rgb2yuv restated (fracoracle.c or_rgb2yuv) → (Y [H, W], U, V [H/2, W/2])."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W = rgb.shape[:2]
    y = np.zeros((H, W), np.uint8)
    cs = W // 2 + 1
    u = np.zeros(((H + 1) // 2, cs), np.uint8)
    v = np.zeros_like(u)
    L = lib()
    L.or_rgb2yuv.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p,
                             C.c_uint32, C.c_void_p, C.c_uint32]
    L.or_rgb2yuv(rgb.ctypes.data, W, H, 3 * W, y.ctypes.data, W, u.ctypes.data, cs, v.ctypes.data, cs)
    return y, np.ascontiguousarray(u[:H // 2, :W // 2]), np.ascontiguousarray(v[:H // 2, :W // 2])


def decode_sized(records: np.ndarray, sizes: np.ndarray, W: int, H: int, max_iter: int = -1, eps: float = 1e-5,
                 initial: np.ndarray | None = None):
    """Decoder2 over records with a range size each (quadtree encodings)."""
    records = np.ascontiguousarray(records, dtype=RESULT_DTYPE)
    sizes = np.ascontiguousarray(sizes, dtype=np.uint32)
    plane = np.zeros((H, W), np.uint8) if initial is None else np.ascontiguousarray(initial, np.uint8).copy()
    rms = C.c_double()
    L = lib()
    L.or_decode_sized.restype = C.c_int
    L.or_decode_sized.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                  C.c_double, C.c_void_p, C.POINTER(C.c_double)]
    it = L.or_decode_sized(records.ctypes.data, sizes.ctypes.data, len(records), 0, W, H, max_iter, eps,
                           plane.ctypes.data, C.byref(rms))
    return plane, it, rms.value


def ref_lib():
    """The reference build (oracle/_ref/libfracref.so) or None when absent."""
    global _ref
    if _ref is None and os.path.exists(REF_LIB_PATH):
        L = C.CDLL(REF_LIB_PATH)
        L.fr_estimate.restype = C.c_int
        L.fr_estimate.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.c_uint32, C.c_int, C.c_double, C.c_double, C.c_int, C.c_int, C.c_void_p,
                                  C.c_size_t, C.c_void_p, C.POINTER(C.c_uint64), C.c_double, C.POINTER(C.c_size_t)]
        _ref = L
    return _ref


def ref_uniform_grid(W: int, H: int, size, offset):
    """The REFERENCE's createUniformGrid (Size32u size / offset), or None when the build is absent.
    The reference FRAC_ASSERTs an area that is not a multiple of the size and offset (exit 0): only
    aligned arguments are passed here."""
    L = ref_lib()
    if L is None:
        return None
    sw, sh = (size, size) if np.isscalar(size) else size
    ox, oy = (offset, offset) if np.isscalar(offset) else offset
    assert W % sw == 0 and H % sh == 0 and W % ox == 0 and H % oy == 0, "unaligned: the reference exits"
    L.fr_uniform_grid.restype = C.c_size_t
    L.fr_uniform_grid.argtypes = [C.c_uint32] * 6 + [C.c_void_p, C.c_size_t]
    n = L.fr_uniform_grid(W, H, sw, sh, ox, oy, None, 0)
    out = np.zeros(n, dtype=ITEM_DTYPE)
    L.fr_uniform_grid(W, H, sw, sh, ox, oy, out.ctypes.data, n)
    return out


def ref_quantize(vmin: float, vmax: float, bits: int, values: np.ndarray):
    """Frac::Quantizerd of the REFERENCE build: (codes u64, dequantized f64), or None when absent."""
    L = ref_lib()
    if L is None:
        return None
    L.fr_quantize.restype = C.c_int
    L.fr_quantize.argtypes = [C.c_double, C.c_double, C.c_int, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
    v = np.ascontiguousarray(values, dtype=np.float64)
    q = np.zeros(len(v), np.uint64)
    back = np.zeros(len(v), np.float64)
    L.fr_quantize(vmin, vmax, bits, v.ctypes.data, len(v), q.ctypes.data, back.ctypes.data)
    return q, back


def ref_estimate(plane: np.ndarray, src_size: int, tgt_size: int, T: int = 4, thr: float = 0.0, smax: float = -1.0,
                 use_classifier: bool = False, sel=None, threads: int = 8, budget_s: float = 0.0):
    """Runs the REFERENCE (grids built as main.cpp does) on the selected range indices."""
    L = ref_lib()
    if L is None:
        raise RuntimeError("reference build oracle/_ref/libfracref.so not present")
    plane = np.ascontiguousarray(plane, dtype=np.uint8)
    H, W = plane.shape
    n_ranges = (W // tgt_size) * (H // tgt_size)
    sel_arr = None if sel is None else np.ascontiguousarray(sel, dtype=np.uint32)
    count = n_ranges if sel_arr is None else len(sel_arr)
    out = np.zeros(count, dtype=RESULT_DTYPE)
    rej = C.c_uint64(0)
    done = C.c_size_t(0)
    L.fr_estimate(plane.ctypes.data, plane.ctypes.data, W, H, W, src_size, tgt_size, T, thr, smax,
                  int(use_classifier), threads, None if sel_arr is None else sel_arr.ctypes.data, count,
                  out.ctypes.data, C.byref(rej), budget_s, C.byref(done))
    return out, int(rej.value), int(done.value)


def quadtree(plane: np.ndarray, max_size: int, min_size: int, split_distance: float, T: int = 4,
             use_classifier: bool = False, thr: float = 0.0, smax: float = -1.0):
    """The quadtree rule of include/fracenc.h (frac_encode_quadtree) restated on the oracle: per
    level n, ranges searched against createUniformGrid(W, H, 2n, n); a range whose distance
    exceeds split_distance (n > min_size) is replaced by its four quadrants.  No reference
    exists (main.cpp:75-76 ignores --quadtree); each level's search is the pinned oracle."""
    plane = np.ascontiguousarray(plane, dtype=np.uint8)
    H, W = plane.shape
    pending = uniform_grid(W, H, max_size, max_size)
    out = []
    n = max_size
    while len(pending) and n >= min_size:
        doms = uniform_grid(W, H, 2 * n, n)
        rngs = pending
        if use_classifier:
            doms = classify(plane, doms)
            rngs = classify(plane, rngs)
        res, _, _ = estimate(plane, doms, rngs, T=T, thr=thr, smax=smax, use_classifier=use_classifier)
        nxt = []
        for i, r in enumerate(res):
            if n > min_size and r["dist"] > split_distance:
                h = n // 2
                x, y = int(pending[i]["x"]), int(pending[i]["y"])
                nxt += [(x, y, h, h, -1), (x + h, y, h, h, -1), (x, y + h, h, h, -1), (x + h, y + h, h, h, -1)]
            else:
                out.append((r, n))
        pending = np.array(nxt, dtype=ITEM_DTYPE)
        n //= 2
    recs = np.zeros(len(out), dtype=RESULT_DTYPE)
    sizes = np.zeros(len(out), dtype=np.uint32)
    for i, (r, sz) in enumerate(out):
        recs[i] = r
        sizes[i] = sz
    return recs, sizes
