"""fractencode_amd — MI355X-native range×domain search for fractal block-matching.

Python binding of the C ABI in include/fracenc.h (libfracenc.so, built in-tree by
``__graft_entry__.build()``).  The product path is the HIP library; there is no
CPU fallback: constructing an :class:`Engine` without the library or without a
GPU raises.

The names mirror the reference's engine API for this path
(sebsgit/fractencode encode/EncodingEngine2.hpp, encode/TransformEstimator2.hpp):
  * :func:`create_uniform_grid`  — Frac2::createUniformGrid (image/partition2.hpp:109-135)
  * :func:`preclassify`          — BrightnessBlocksClassifier2::preclassify (Classifier2.cpp:64-68)
  * :class:`Engine`              — an AbstractEncodingEngine2 that encodes a whole batch
                                   of range items per call on one GPU
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# FRAC_LIB: an explicitly built alternative (tools/build_tuning.py's A/B library); the product is libfracenc.so.
# build_info() reports which library was loaded and whether it is a tuning build; bench.py refuses the
# headline with FRAC_LIB set.
PRODUCT_LIB = os.path.join(HERE, "libfracenc.so")
LIB_PATH = os.environ.get("FRAC_LIB") or PRODUCT_LIB

GRID_ITEM = np.dtype([("x", "<u4"), ("y", "<u4"), ("w", "<u4"), ("h", "<u4"), ("category", "<i4")])
ENCODE_ITEM = np.dtype([("x", "<u4"), ("y", "<u4"), ("w", "<u4"), ("h", "<u4"),
                        ("distance", "<f8"), ("contrast", "<f8"), ("brightness", "<f8"),
                        ("transform", "<i4"), ("_pad", "<i4"),
                        ("dx", "<u4"), ("dy", "<u4"), ("sw", "<u4"), ("sh", "<u4")])
# frac_tuple: (domain index, transform, s, o, rms) — the 32-byte record of the multi-GPU gather
TUPLE = np.dtype([("domain", "<u4"), ("transform", "<i4"), ("contrast", "<f8"), ("brightness", "<f8"),
                  ("distance", "<f8")])
# frac_run_timing: per-run device times (frac_timing_history)
RUN_TIMING = np.dtype([("ms_device", "<f8"), ("ms_prep", "<f8"), ("ms_search", "<f8"), ("ms_finish", "<f8")])
NO_DOMAIN = 0xFFFFFFFF
# frac_qt_leaf: a quadtree leaf in 32 bytes (frac_encode_quadtree_leaves, ABI 7)
QT_LEAF = np.dtype([("x", "<u2"), ("y", "<u2"), ("code", "<u4"), ("contrast", "<f8"), ("brightness", "<f8"),
                    ("distance", "<f8")])
QT_NO_DOMAIN = 0xFFFFFF
assert GRID_ITEM.itemsize == 20 and ENCODE_ITEM.itemsize == 64 and TUPLE.itemsize == 32 and QT_LEAF.itemsize == 32


def records_from_leaves(leaves: np.ndarray, width: int) -> np.ndarray:
    """encode_item_t records (ENCODE_ITEM) from 32-byte quadtree leaves (QT_LEAF) of a frame `width`
    pixels wide: the range at (x, y) of size n = 1 << (code >> 28), the winner domain `code & 0xffffff` of
    that level's grid createUniformGrid(W, H, 2n, n) (cols = (W − 2n)/n + 1), transform (code >> 24) & 15;
    QT_NO_DOMAIN is the reference's default record (domain (0, 0), size (0, 0))."""
    code = np.asarray(leaves["code"], np.uint32)
    n = (np.uint32(1) << (code >> np.uint32(28))).astype(np.uint32)
    d = (code & np.uint32(QT_NO_DOMAIN)).astype(np.int64)
    has = d != QT_NO_DOMAIN
    cols = np.where(width >= 2 * n, (np.int64(width) - 2 * n.astype(np.int64)) // n + 1, 1)
    rec = np.zeros(len(leaves), dtype=ENCODE_ITEM)
    rec["x"], rec["y"], rec["w"], rec["h"] = leaves["x"], leaves["y"], n, n
    for k in ("contrast", "brightness", "distance"):
        rec[k] = leaves[k]
    rec["transform"] = ((code >> np.uint32(24)) & np.uint32(15)).astype(np.int32)
    rec["dx"] = np.where(has, (d % cols) * n, 0)
    rec["dy"] = np.where(has, (d // cols) * n, 0)
    rec["sw"] = rec["sh"] = np.where(has, 2 * n, 0)
    return rec

ENGINE_AUTO, ENGINE_VALU, ENGINE_MFMA, ENGINE_SEA = 0, 1, 2, 3
FORM_DOT2, FORM_DIRECT, FORM_FOURIER, FORM_SEA, FORM_SEA_MFMA, FORM_SAMPLED = 0, 1, 2, 3, 4, 5
FORM_NAMES = {FORM_DOT2: "dot2", FORM_DIRECT: "direct", FORM_FOURIER: "fourier", FORM_SEA: "sea",
              FORM_SEA_MFMA: "sea_mfma", FORM_SAMPLED: "sampled"}
FLAG_TIMING = 1
# alternative exact forms (ABI 6; the product build refuses the old FRAC_MFMA_DFT / FRAC_SEA_TILED /
# FRAC_DECODE_UNFUSED environment knobs)
FLAG_DIRECT_FORM, FLAG_SEA_PER_RANGE, FLAG_DECODE_STEPWISE = 2, 4, 8

# Frac::TransformType (image/transform.h:16-25)
TRANSFORM_NAMES = ("Id", "Rotate_90", "Rotate_180", "Rotate_270", "Flip", "Flip_Rotate_90", "Flip_Rotate_180",
                   "Flip_Rotate_270")


class FracParams(C.Structure):
    _fields_ = [("transforms", C.c_uint32), ("use_classifier", C.c_int32), ("rms_threshold", C.c_double),
                ("s_max", C.c_double), ("engine", C.c_uint32), ("flags", C.c_uint32)]


class FracStats(C.Structure):
    _fields_ = [("rejected_mappings", C.c_uint64), ("total_mappings", C.c_uint64), ("hit_ranges", C.c_uint32),
                ("fallback_ranges", C.c_uint32), ("empty_ranges", C.c_uint32), ("engine", C.c_uint32),
                ("ms_device", C.c_double), ("ms_search", C.c_double), ("ms_prep", C.c_double),
                ("ms_finish", C.c_double), ("search_form", C.c_uint32), ("pad_", C.c_uint32),
                ("matrix_flops", C.c_uint64), ("evaluated_mappings", C.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class FracQuadtreeParams(C.Structure):
    _fields_ = [("max_size", C.c_uint32), ("min_size", C.c_uint32), ("split_distance", C.c_double)]


class FracError(RuntimeError):
    pass


_lib = None


# The product compile line (__graft_entry__.build): part of the source id, so a change of flags or
# of the ROCm toolchain rebuilds the library and re-keys the PMC measurements like a source change.
# -amdgpu-mfma-vgpr-form: MFMA accumulators in VGPRs (gfx950 has one unified register file), so the
# integer epilogue reads them without v_accvgpr_read copies.
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall",
               "-mllvm", "-amdgpu-mfma-vgpr-form"]
SOURCE_EXTS = (".hip", ".h", ".cuh")


def _rocm_version() -> str:
    try:
        with open("/opt/rocm/.info/version") as f:
            return f.read().strip()
    except OSError:
        return "unknown"


def source_id() -> str:
    """16 hex digits identifying the library's sources (the .hip / .h files of csrc/ and
    include/fracenc.h), its compile flags and the ROCm version: the key under which profiles/ records
    PMC measurements, so a measurement of another build is never reused."""
    import hashlib

    h = hashlib.sha256()
    csrc = os.path.join(HERE, "csrc")
    for name in sorted(os.listdir(csrc)):
        path = os.path.join(csrc, name)
        if not (os.path.isfile(path) and name.endswith(SOURCE_EXTS)):
            continue
        with open(path, "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    with open(os.path.join(os.path.dirname(HERE), "include", "fracenc.h"), "rb") as f:
        h.update(f.read())
    h.update(("\0".join(HIPCC_FLAGS) + "\0rocm " + _rocm_version()).encode())
    return h.hexdigest()[:16]


def lib() -> C.CDLL:
    """The HIP engine library; raises FracError when it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FracError(f"{LIB_PATH} not built: run __graft_entry__.build() (no CPU fallback exists)")
        # One HIP runtime per process: PyTorch bundles its own libamdhip64 (soname libamdhip64.so.7,
        # file name libamdhip64.so).  Loaded first, it also serves this library (same soname), so
        # torch streams and device tensors are valid here; loaded second, torch would open a second
        # runtime that finds no device.  Import torch (when installed) before the library.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if LIB_PATH != PRODUCT_LIB:
            import warnings

            warnings.warn(f"fractencode_amd: FRAC_LIB loads {LIB_PATH}, not the product library", stacklevel=2)
        L = C.CDLL(LIB_PATH)
        vp, u32, i32, sz = C.c_void_p, C.c_uint32, C.c_int, C.c_size_t
        sig = {
            "frac_abi_version": (i32, []),
            "frac_device_count": (i32, []),
            "frac_build_id": (C.c_char_p, []),
            "frac_build_flags": (i32, []),
            "frac_create": (vp, [i32, C.POINTER(FracParams)]),
            "frac_destroy": (None, [vp]),
            "frac_last_error": (C.c_char_p, [vp]),
            "frac_set_params": (i32, [vp, C.POINTER(FracParams)]),
            "frac_set_frame": (i32, [vp, vp, u32, u32, u32]),
            "frac_set_planes": (i32, [vp, vp, u32, u32, u32, vp, u32, u32, u32]),
            "frac_set_frame_device": (i32, [vp, vp, u32, u32, u32]),
            "frac_set_frame_device_async": (i32, [vp, vp, u32, u32, u32]),
            "frac_set_frame_async": (i32, [vp, vp, u32, u32, u32]),
            "frac_set_domains": (i32, [vp, vp, sz]),
            "frac_set_ranges": (i32, [vp, vp, sz]),
            "frac_run": (i32, [vp]),
            "frac_fetch": (i32, [vp, vp, C.POINTER(FracStats)]),
            "frac_sync": (i32, [vp]),
            "frac_timing_history": (i32, [vp, vp, sz, C.POINTER(C.c_size_t)]),
            "frac_search": (i32, [vp, vp, sz, vp, C.POINTER(FracStats)]),
            "frac_set_stream": (i32, [vp, vp]),
            "frac_get_stream": (vp, [vp]),
            "frac_device_results": (vp, [vp]),
            "frac_copy_results_device": (i32, [vp, vp]),
            "frac_copy_tuples_device": (i32, [vp, vp]),
            "frac_set_tuple_sink": (i32, [vp, vp]),
            "frac_pack_frc1": (i32, [vp, u32, u32, vp, sz, C.POINTER(C.c_size_t)]),
            "frac_fetch_tuples": (i32, [vp, vp]),
            "frac_decode": (i32, [vp, vp, sz, u32, u32, i32, C.c_double, vp, C.POINTER(C.c_int),
                                  C.POINTER(C.c_double)]),
            "frac_decode_results": (i32, [vp, u32, u32, i32, C.c_double, vp, C.POINTER(C.c_int),
                                          C.POINTER(C.c_double)]),
            "frac_classify_items": (i32, [vp, vp, sz, i32]),
            "frac_encode_quadtree": (i32, [vp, C.POINTER(FracQuadtreeParams), vp, sz, C.POINTER(sz),
                                           C.POINTER(FracStats)]),
            "frac_encode_quadtree_leaves": (i32, [vp, C.POINTER(FracQuadtreeParams), vp, sz, C.POINTER(sz),
                                                  C.POINTER(FracStats)]),
            "frac_rgb_to_yuv_device": (i32, [vp, vp, u32, u32, u32, vp, u32, vp, u32, vp, u32]),
            "frac_rgb_to_yuv": (i32, [vp, vp, u32, u32, u32, vp, vp, vp]),
            "frac_uniform_grid": (sz, [u32, u32, u32, u32, vp, sz]),
            "frac_uniform_grid2": (sz, [u32, u32, u32, u32, u32, u32, vp, sz]),
            "frac_classify": (i32, [vp, u32, u32, u32, vp, sz]),
            "frac_transform_index": (i32, [u32, u32, u32]),
            "frac_hit_limit": (C.c_int64, [C.c_double, u32]),
        }
        for name, (res, args) in sig.items():
            if os.environ.get("FRAC_LIB") and not hasattr(L, name):
                continue  # an A/B library built from older sources lacks the newer entry points
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


BUILD_TUNING = 1


def build_info() -> dict:
    """The loaded library: its path, the source id compiled into it (frac_build_id), whether it is
    a -DFRAC_TUNING build, and whether that id is the id of the sources next to it."""
    L = lib()
    bid = L.frac_build_id().decode()
    return {"lib": os.path.relpath(LIB_PATH, os.path.dirname(HERE)), "build_id": bid,
            "tuning": bool(L.frac_build_flags() & BUILD_TUNING), "matches_sources": bid == source_id()}


def last_error(ctx=None) -> str:
    msg = lib().frac_last_error(ctx)
    return msg.decode() if msg else ""


# ---- host helpers ----------------------------------------------------------------

def create_uniform_grid(width: int, height: int, item_size, item_offset) -> np.ndarray:
    """Frac2::createUniformGrid (image/partition2.hpp:109-135): row-major items, x fastest
    (categories -1).  item_size / item_offset: an int, or (x, y) like the reference's Size32u."""
    sw, sh = (item_size, item_size) if np.isscalar(item_size) else item_size
    ox, oy = (item_offset, item_offset) if np.isscalar(item_offset) else item_offset
    n = lib().frac_uniform_grid2(width, height, sw, sh, ox, oy, None, 0)
    out = np.zeros(n, dtype=GRID_ITEM)
    if n:
        lib().frac_uniform_grid2(width, height, sw, sh, ox, oy, out.ctypes.data, n)
    return out


def preclassify(plane: np.ndarray, items: np.ndarray) -> np.ndarray:
    """Categories of BrightnessBlocksClassifier2 computed on `plane` (returns a copy)."""
    plane = np.ascontiguousarray(plane, dtype=np.uint8)
    items = np.ascontiguousarray(items, dtype=GRID_ITEM).copy()
    rc = lib().frac_classify(plane.ctypes.data, plane.shape[1], plane.shape[0], plane.shape[1], items.ctypes.data,
                             len(items))
    if rc != 0:
        raise FracError(last_error())
    return items


def transform_index(n: int, t: int, pix: int) -> int:
    return lib().frac_transform_index(n, t, pix)


def hit_limit(rms_threshold: float, n: int) -> int:
    return lib().frac_hit_limit(rms_threshold, n)


# ---- engine ---------------------------------------------------------------------

class Engine:
    """One search context on one GPU (an AbstractEncodingEngine2 that takes batches).

    Parameters mirror encode_parameters_t / TransformMatcher: ``transforms`` 4 (the
    reference's TransformMatcher::match) or 8, ``use_classifier``, ``rms_threshold``,
    ``s_max``.
    """

    def __init__(self, device: int = 0, transforms: int = 4, use_classifier: bool = False,
                 rms_threshold: float = 0.0, s_max: float = -1.0, engine: int = ENGINE_AUTO, timing: bool = False,
                 flags: int = 0):
        """flags: FLAG_DIRECT_FORM / FLAG_SEA_PER_RANGE / FLAG_DECODE_STEPWISE select an alternative
        exact form (the same records from other kernels: cross-checks)."""
        self._p = FracParams(transforms, int(use_classifier), rms_threshold, s_max, engine,
                             (FLAG_TIMING if timing else 0) | flags)
        self._ctx = lib().frac_create(device, C.byref(self._p))
        if not self._ctx:
            raise FracError("frac_create failed: " + last_error())
        self._nr = 0
        self._keep = []
        self._frame_wh = (0, 0)

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            lib().frac_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int) -> None:
        if rc != 0:
            raise FracError(f"rc={rc}: {last_error(self._ctx)}")

    def set_params(self, transforms=None, use_classifier=None, rms_threshold=None, s_max=None, engine=None,
                   flags=None):
        if transforms is not None:
            self._p.transforms = transforms
        if use_classifier is not None:
            self._p.use_classifier = int(use_classifier)
        if rms_threshold is not None:
            self._p.rms_threshold = rms_threshold
        if s_max is not None:
            self._p.s_max = s_max
        if engine is not None:
            self._p.engine = engine
        if flags is not None:
            self._p.flags = (self._p.flags & FLAG_TIMING) | flags
        self._check(lib().frac_set_params(self._ctx, C.byref(self._p)))

    def set_frame(self, plane) -> None:
        """Source == target plane (Encoder2).  numpy uint8 [H, W] or a CUDA torch tensor."""
        self._frame_wh = (int(plane.shape[1]), int(plane.shape[0]))
        if hasattr(plane, "is_cuda") and plane.is_cuda:
            import torch

            if plane.dtype != torch.uint8 or plane.dim() != 2:
                raise FracError("set_frame: a device plane must be a 2-D uint8 tensor")
            if plane.stride(1) != 1 or plane.stride(0) < plane.shape[1]:
                raise FracError("set_frame: device plane rows must be contiguous (stride(1) == 1, "
                                "stride(0) >= width)")
            # the library copies on its own stream: work still pending on torch's current stream
            # (e.g. the kernel producing this plane) must land first
            torch.cuda.current_stream(plane.device).synchronize()
            self._check(lib().frac_set_frame_device(self._ctx, C.c_void_p(plane.data_ptr()), plane.shape[1],
                                                    plane.shape[0], plane.stride(0)))
            return
        plane = np.ascontiguousarray(plane, dtype=np.uint8)
        self._check(lib().frac_set_frame(self._ctx, plane.ctypes.data, plane.shape[1], plane.shape[0],
                                         plane.shape[1]))

    def set_frame_device_async(self, plane) -> None:
        """ABI 9: a CUDA uint8 [H, W] plane copied on this engine's stream without waiting (frame streaming).
        The caller orders the plane's producer before this engine's stream (e.g. an event the stream waits on)
        and keeps the plane unchanged until the stream has passed the copy."""
        if not (hasattr(plane, "is_cuda") and plane.is_cuda) or plane.dim() != 2 or plane.stride(1) != 1:
            raise FracError("set_frame_device_async: a 2-D CUDA uint8 plane with contiguous rows")
        self._frame_wh = (int(plane.shape[1]), int(plane.shape[0]))
        self._check(lib().frac_set_frame_device_async(self._ctx, C.c_void_p(plane.data_ptr()), plane.shape[1],
                                                      plane.shape[0], plane.stride(0)))

    def set_frame_async(self, plane) -> None:
        """ABI 9: frame streaming from host memory — a uint8 [H, W] plane (a pinned torch tensor or a numpy view
        of one, for an asynchronous copy) uploaded on the context's copy stream while the runs already enqueued
        search the previous frame; the next run() searches this one.  The plane must stay unchanged until the
        upload is done (a later sync() / fetch(), or an event on this engine's stream)."""
        if hasattr(plane, "is_cuda"):
            if plane.is_cuda:
                raise FracError("set_frame_async: a host plane (set_frame_device_async takes device planes)")
            plane = plane.numpy()
        if plane.dtype != np.uint8 or plane.ndim != 2 or plane.strides[1] != 1:
            raise FracError("set_frame_async: a 2-D uint8 host plane with contiguous rows")
        self._frame_wh = (int(plane.shape[1]), int(plane.shape[0]))
        self._keep_async = plane  # the memory stays referenced while the upload may run
        self._check(lib().frac_set_frame_async(self._ctx, C.c_void_p(plane.ctypes.data), plane.shape[1],
                                               plane.shape[0], plane.strides[0]))

    def set_planes(self, source: np.ndarray, target: np.ndarray) -> None:
        self._frame_wh = (int(source.shape[1]), int(source.shape[0]))
        s = np.ascontiguousarray(source, dtype=np.uint8)
        t = np.ascontiguousarray(target, dtype=np.uint8)
        self._check(lib().frac_set_planes(self._ctx, s.ctypes.data, s.shape[1], s.shape[0], s.shape[1], t.ctypes.data,
                                          t.shape[1], t.shape[0], t.shape[1]))

    def set_domains(self, items: np.ndarray) -> None:
        items = np.ascontiguousarray(items, dtype=GRID_ITEM)
        self._check(lib().frac_set_domains(self._ctx, items.ctypes.data if len(items) else None, len(items)))

    def set_ranges(self, items: np.ndarray) -> None:
        items = np.ascontiguousarray(items, dtype=GRID_ITEM)
        self._check(lib().frac_set_ranges(self._ctx, items.ctypes.data if len(items) else None, len(items)))
        self._nr = len(items)

    def run(self) -> None:
        self._check(lib().frac_run(self._ctx))

    def sync(self) -> None:
        self._check(lib().frac_sync(self._ctx))

    def fetch(self):
        out = np.zeros(self._nr, dtype=ENCODE_ITEM)
        st = FracStats()
        self._check(lib().frac_fetch(self._ctx, out.ctypes.data if self._nr else None, C.byref(st)))
        return out, st.as_dict()

    def timing_history(self) -> np.ndarray:
        """Device times (ms: device, prep, search, finish) of every run since the previous call
        (engine created with timing=True); waits for the stream."""
        n = C.c_size_t(0)
        self._check(lib().frac_timing_history(self._ctx, None, 0, C.byref(n)))
        out = np.zeros(n.value, dtype=RUN_TIMING)
        self._check(lib().frac_timing_history(self._ctx, out.ctypes.data if n.value else None, n.value, C.byref(n)))
        return out[: n.value]

    def search(self, ranges: np.ndarray):
        """set_ranges + run + fetch → (encode items in range order, stats dict)."""
        self.set_ranges(ranges)
        self.run()
        return self.fetch()

    def set_stream(self, stream_handle: int | None) -> None:
        self._check(lib().frac_set_stream(self._ctx, C.c_void_p(stream_handle) if stream_handle else None))

    def stream_handle(self) -> int:
        """The hipStream_t this context enqueues on (frac_get_stream), as an integer."""
        return lib().frac_get_stream(self._ctx) or 0

    def copy_results_device(self, dst_ptr: int) -> None:
        """Async D2D copy of the last run's results (64 B each) to a device buffer."""
        self._check(lib().frac_copy_results_device(self._ctx, C.c_void_p(dst_ptr)))

    def copy_tuples_device(self, dst_ptr: int) -> None:
        """Async pack of the last run's 32-byte (domain, transform, s, o, rms) tuples into a device buffer."""
        self._check(lib().frac_copy_tuples_device(self._ctx, C.c_void_p(dst_ptr)))

    def set_tuple_sink(self, dst_ptr: int | None) -> None:
        """Every later run also writes its 32-byte tuples to dst_ptr (device memory, or pinned host memory
        the device can write: they then cross PCIe while the resolve writes them); None clears it (ABI 8)."""
        self._check(lib().frac_set_tuple_sink(self._ctx, C.c_void_p(dst_ptr) if dst_ptr else None))

    def pack_frc1(self, contrast_bits: int = 5, brightness_bits: int = 7) -> bytes:
        """The last run's results as an FRC1 stream (codec.py layout), quantized and packed on the
        device (frac_pack_frc1)."""
        n = C.c_size_t(0)
        self._check(lib().frac_pack_frc1(self._ctx, contrast_bits, brightness_bits, None, 0, C.byref(n)))
        buf = np.empty(n.value, dtype=np.uint8)
        self._check(lib().frac_pack_frc1(self._ctx, contrast_bits, brightness_bits, buf.ctypes.data_as(C.c_void_p),
                                         n.value, C.byref(n)))
        return buf.tobytes()

    def fetch_tuples(self, out: np.ndarray | None = None) -> np.ndarray:
        """The last run's tuples (TUPLE records) on the host; `out` (TUPLE array of the range count,
        e.g. a view of pinned memory) is filled in place when given."""
        n = self._nr
        if out is None:
            out = np.zeros(n, dtype=TUPLE)
        elif out.dtype != TUPLE or len(out) != n or not out.flags.c_contiguous:
            raise FracError("fetch_tuples: out must be a contiguous TUPLE array of the range count")
        if n:
            self._check(lib().frac_fetch_tuples(self._ctx, out.ctypes.data_as(C.c_void_p)))
        return out

    def decode(self, items: np.ndarray | None, width: int, height: int, max_iter: int = -1, rms_eps: float = 1e-5,
               initial: np.ndarray | None = None):
        """Decoder2::decode on the GPU. items=None decodes the last run's results on the device.
        Returns (plane, iterations, rms)."""
        plane = np.zeros((height, width), np.uint8) if initial is None else np.ascontiguousarray(initial, np.uint8).copy()
        it = C.c_int()
        rms = C.c_double()
        if items is None:
            self._check(lib().frac_decode_results(self._ctx, width, height, max_iter, rms_eps, plane.ctypes.data,
                                                  C.byref(it), C.byref(rms)))
        else:
            items = np.ascontiguousarray(items, dtype=ENCODE_ITEM)
            self._check(lib().frac_decode(self._ctx, items.ctypes.data if len(items) else None, len(items), width,
                                          height, max_iter, rms_eps, plane.ctypes.data, C.byref(it), C.byref(rms)))
        return plane, it.value, rms.value

    def encode_quadtree(self, max_size: int = 16, min_size: int = 4, split_distance: float = 10.0, out=None,
                        allow_short: bool = False, leaves: bool = False):
        """Quadtree partition of the frame set on this engine (frac_encode_quadtree): ranges of
        max_size split into quadrants while their best distance exceeds split_distance, down to
        min_size.  Returns (encode items of mixed sizes, summed stats dict).  With `out` (an
        ENCODE_ITEM array of at least (W/min_size)·(H/min_size) items, e.g. pinned host memory)
        the items are written there and a view of it is returned, without a copy; pinned host memory is
        written by the device directly (no copy command).  allow_short: `out` may be shorter — the items
        past it are counted (the stats) but not written, and the returned view is cut to `out`.
        leaves=True: 32-byte QT_LEAF items instead (frac_encode_quadtree_leaves; records_from_leaves rebuilds
        the records), half the bytes across PCIe."""
        qp = FracQuadtreeParams(max_size, min_size, split_distance)
        n = C.c_size_t(0)
        st = FracStats()
        W, H = self._frame_wh
        cap = max((W // min_size) * (H // min_size), 1)
        dt = QT_LEAF if leaves else ENCODE_ITEM
        if out is not None:
            if out.dtype != dt or not out.flags.c_contiguous or (len(out) < cap and not allow_short):
                raise ValueError(f"out must be a contiguous {'QT_LEAF' if leaves else 'ENCODE_ITEM'} array of at "
                                 f"least {cap} items")
            buf = out
            cap = len(out)
        else:
            # one pass with a worst-case capacity (every range at min_size), in a buffer kept across
            # calls: a fresh one costs a page fault per 4 KiB on first touch
            attr = "_qt_leaf_buf" if leaves else "_qt_buf"
            buf = getattr(self, attr, None)
            if buf is None or len(buf) < cap:
                buf = np.empty(cap, dtype=dt)
                setattr(self, attr, buf)
        fn = lib().frac_encode_quadtree_leaves if leaves else lib().frac_encode_quadtree
        self._check(fn(self._ctx, C.byref(qp), buf.ctypes.data, cap, C.byref(n), C.byref(st)))
        d = st.as_dict()
        d["items"] = n.value
        return (buf[: min(n.value, cap)] if out is not None else buf[: n.value].copy()), d

    def classify(self, items: np.ndarray, target_plane: bool = False) -> np.ndarray:
        """BrightnessBlocksClassifier2 categories of `items` computed on the device plane set by
        set_frame / set_planes (returns a copy with the categories filled in)."""
        items = np.ascontiguousarray(items, dtype=GRID_ITEM).copy()
        self._check(lib().frac_classify_items(self._ctx, items.ctypes.data if len(items) else None, len(items),
                                              int(target_plane)))
        return items

    def rgb_to_yuv(self, rgb):
        """ImageIO::rgb2yuv on the device (image/ImageIO.cpp:43-58).

        rgb: numpy uint8 [H, W, 3] → numpy (Y [H, W], U [H/2, W/2], V [H/2, W/2]); or a CUDA
        uint8 tensor [H, W, 3] (rows may be strided) → CUDA tensors, enqueued on this
        engine's stream and synchronised before returning."""
        if hasattr(rgb, "is_cuda") and rgb.is_cuda:
            import torch

            assert rgb.dtype == torch.uint8 and rgb.dim() == 3 and rgb.shape[2] == 3
            assert rgb.stride(2) == 1 and rgb.stride(1) == 3, "pixels must be packed RGB"
            H, W = rgb.shape[0], rgb.shape[1]
            y = torch.empty((H, W), dtype=torch.uint8, device=rgb.device)
            u = torch.empty((H // 2, W // 2), dtype=torch.uint8, device=rgb.device)
            v = torch.empty_like(u)
            torch.cuda.current_stream(rgb.device).synchronize()  # rgb must be ready before our stream reads it
            self._check(lib().frac_rgb_to_yuv_device(self._ctx, C.c_void_p(rgb.data_ptr()), W, H, rgb.stride(0),
                                                     C.c_void_p(y.data_ptr()), W, C.c_void_p(u.data_ptr()),
                                                     max(W // 2, 1), C.c_void_p(v.data_ptr()), max(W // 2, 1)))
            self.sync()
            return y, u, v
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        assert rgb.ndim == 3 and rgb.shape[2] == 3
        H, W = rgb.shape[:2]
        y = np.zeros((H, W), np.uint8)
        u = np.zeros((H // 2, W // 2), np.uint8)
        v = np.zeros((H // 2, W // 2), np.uint8)
        self._check(lib().frac_rgb_to_yuv(self._ctx, rgb.ctypes.data, W, H, 3 * W, y.ctypes.data, u.ctypes.data,
                                          v.ctypes.data))
        return y, u, v

    def device_results_ptr(self) -> int:
        return lib().frac_device_results(self._ctx) or 0


def encode(plane: np.ndarray, range_size: int = 4, domain_size: int = 16, transforms: int = 4,
           use_classifier: bool = True, rms_threshold: float = 0.0, s_max: float = -1.0, device: int = 0,
           engine: int = ENGINE_AUTO):
    """Encoder2's search half for one plane, with grids built like main.cpp:142-162 and the CLI's
    defaults (encode/encode_parameters.h:6-13): 16×16 domains at offset 16 / latticeSize 2, 4×4
    ranges, the classifier on, rms threshold 0, sMax −1."""
    plane = np.ascontiguousarray(plane, dtype=np.uint8)
    H, W = plane.shape
    dsz = domain_size
    doms = create_uniform_grid(W, H, dsz, dsz // 2)
    rngs = create_uniform_grid(W, H, range_size, range_size)
    if use_classifier:
        doms = preclassify(plane, doms)
        rngs = preclassify(plane, rngs)
    with Engine(device, transforms, use_classifier, rms_threshold, s_max, engine) as e:
        e.set_frame(plane)
        e.set_domains(doms)
        return e.search(rngs)
