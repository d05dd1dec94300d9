"""Quantized encoded stream for the search's winners.

The reference has no file format: `encode_data_statistics` (main.cpp:106-140) only
builds `Frac::Quantizerd` over the frame's (contrast, brightness) range with 5 and 7
bits (main.cpp:120-121) and prints bucket counts.  This module keeps that quantizer
bit-for-bit and defines the record the reference leaves open:

    per range: (domain index, transform, q_contrast, q_brightness)

bit-packed LSB-first at a fixed width per field.  At C3 (261,121 domains, T=4,
5+7 bits) a record is 18+2+5+7 = 32 bits, i.e. 1 MiB per 4096² frame instead of
the 16 MiB of 64-byte encode_item_t records.

Stream layout ("FRC1", little-endian)::

    0   char[4]  magic "FRC1"
    4   u16      version (1)
    6   u16      flags (bit 0: classifier was on; informational)
    8   u32      width, height
    16  u32      range_size, domain_size, domain_stride
    28  u8       transforms, contrast_bits, brightness_bits, index_bits
    32  u32      n_ranges, n_domains
    40  f64      contrast_min, contrast_max, brightness_min, brightness_max
    72  u8[]     records, ceil(n_ranges * record_bits / 8) bytes

Ranges are the createUniformGrid(range_size, range_size) lattice in row-major order
(image/partition2.hpp:109-135); domain index i is position i of
createUniformGrid(domain_size, domain_stride); index == n_domains marks a range that
had no eligible domain (the reference's default record, encode/datatypes.h:8-26).
When every value of a field is equal the quantizer would be degenerate (the reference
asserts max > min, Quantizer.hpp:19): the header then stores min == max and every
record dequantizes to exactly that value.
"""
from __future__ import annotations

import struct
from fractions import Fraction

import numpy as np

MAGIC = b"FRC1"
VERSION = 1
HEADER = struct.Struct("<4sHHIIIIIBBBBIIdddd")
assert HEADER.size == 72
CONTRAST_BITS = 5  # main.cpp:120
BRIGHTNESS_BITS = 7  # main.cpp:121


class Quantizer:
    """Frac::Quantizer<double> (encode/Quantizer.hpp:7-45).

    step = |max − min| / 2^bits; quantized(v) = min(2^bits − 1, floor((v − min) / step));
    value(q) = q·step + min + step/2, where the built reference contracts q·step + min
    into one FMA (verified against oracle/_ref's fr_quantize), reproduced here exactly
    through a per-code table computed in rational arithmetic.
    """

    def __init__(self, vmin: float, vmax: float, bits: int):
        if not (vmax > vmin):
            raise ValueError("Quantizer: max must exceed min (Quantizer.hpp:19)")
        if not (1 < bits <= 24):
            raise ValueError("Quantizer: bits must be in (1, 24]")
        self.min = float(vmin)
        self.max = float(vmax)
        self.bits = int(bits)
        self.step = abs(self.max - self.min) / float(1 << self.bits)
        self.max_quantized = (1 << self.bits) - 1
        if not self.step > 0.0:
            raise ValueError("Quantizer: zero step (Quantizer.hpp:22)")
        self._table = None

    def quantized(self, v) -> np.ndarray:
        v = np.asarray(v, dtype=np.float64)
        q = np.floor((v - self.min) / self.step)
        return np.minimum(float(self.max_quantized), q).astype(np.uint64)

    def table(self) -> np.ndarray:
        """value(q) for every code q (fl(fl(q·step + min) + step/2), the first rounding fused)."""
        if self._table is None:
            step, mn, half = Fraction(self.step), Fraction(self.min), self.step / 2
            fused = [float(q * step + mn) for q in range(self.max_quantized + 1)]
            self._table = np.array(fused, dtype=np.float64) + half
        return self._table

    def value(self, q) -> np.ndarray:
        q = np.asarray(q, dtype=np.uint64)
        if q.size and int(q.max()) > self.max_quantized:
            raise ValueError("Quantizer: code out of range (Quantizer.hpp:34)")
        return self.table()[q.astype(np.int64)]


def psnr(a: np.ndarray, b: np.ndarray, peak: float = 255.0) -> float:
    """10·log10(peak² / MSE) over two equally shaped u8 planes (inf when identical)."""
    a = np.asarray(a, dtype=np.int64)
    b = np.asarray(b, dtype=np.int64)
    if a.shape != b.shape:
        raise ValueError("psnr: shape mismatch")
    mse = float(((a - b) ** 2).sum()) / a.size
    return float("inf") if mse == 0.0 else 10.0 * np.log10(peak * peak / mse)


def _grid_cols_rows(width: int, height: int, size: int, stride: int) -> tuple[int, int]:
    """Column / row count of createUniformGrid (image/partition2.hpp:123-133)."""
    if size > width or size > height:
        return 0, 0
    return (width - size) // stride + 1, (height - size) // stride + 1


class _Field:
    def __init__(self, v: np.ndarray, bits: int):
        lo, hi = (float(v.min()), float(v.max())) if len(v) else (0.0, 0.0)
        self.min, self.max, self.bits = lo, hi, bits
        self.q = None if not hi > lo else Quantizer(lo, hi, bits)

    def codes(self, v: np.ndarray) -> np.ndarray:
        return np.zeros(len(v), np.uint64) if self.q is None else self.q.quantized(v)


def _pack_bits(fields: list[tuple[np.ndarray, int]], n: int) -> bytes:
    """Record i's fields, concatenated LSB-first, occupy bits [i·width, (i+1)·width) of the body."""
    width = sum(b for _, b in fields)
    bits = np.zeros((n, width), dtype=np.uint8)
    shift = 0
    for vals, b in fields:
        v = vals.astype(np.uint64)
        if n and int(v.max()) >> b:
            raise ValueError("pack: field value does not fit its width")
        for k in range(b):
            bits[:, shift + k] = (v >> np.uint64(k)) & np.uint64(1)
        shift += b
    return np.packbits(bits.reshape(-1), bitorder="little").tobytes()


def _unpack_bits(buf: bytes, n: int, widths: list[int]) -> list[np.ndarray]:
    width = sum(widths)
    raw = np.frombuffer(buf, dtype=np.uint8)
    bits = np.unpackbits(raw, bitorder="little")[: n * width].reshape(n, width).astype(np.uint64)
    out, shift = [], 0
    for b in widths:
        w = np.zeros(n, dtype=np.uint64)
        for k in range(b):
            w |= bits[:, shift + k] << np.uint64(k)
        out.append(w)
        shift += b
    return out


def pack_stream(items: np.ndarray, width: int, height: int, range_size: int, domain_size: int | None = None,
                transforms: int = 4, use_classifier: bool = False, contrast_bits: int = CONTRAST_BITS,
                brightness_bits: int = BRIGHTNESS_BITS) -> bytes:
    """Quantize and pack encode_item_t records (fractencode_amd.ENCODE_ITEM, range order) into FRC1."""
    from . import ENCODE_ITEM

    items = np.ascontiguousarray(items, dtype=ENCODE_ITEM)
    dsz = domain_size or 2 * range_size
    dstride = dsz // 2  # latticeSize = 2 (encode/encode_parameters.h:8), main.cpp:147
    rc, rr = _grid_cols_rows(width, height, range_size, range_size)
    if len(items) != rc * rr:
        raise ValueError(f"pack_stream: {len(items)} records, the range grid has {rc * rr}")
    exp_x = (np.arange(rc * rr) % max(rc, 1)) * range_size
    exp_y = (np.arange(rc * rr) // max(rc, 1)) * range_size
    if len(items) and (np.any(items["x"] != exp_x) or np.any(items["y"] != exp_y)):
        raise ValueError("pack_stream: records are not in row-major range-grid order")
    dc, dr = _grid_cols_rows(width, height, dsz, dstride)
    nd = dc * dr
    has = (items["sw"] != 0) & (items["sh"] != 0)
    if np.any(has & ((items["dx"] % dstride != 0) | (items["dy"] % dstride != 0))):
        raise ValueError("pack_stream: a winner is not on the domain lattice")
    idx = np.where(has, (items["dy"] // dstride) * dc + items["dx"] // dstride, nd).astype(np.uint64)
    if np.any(has & (idx >= nd)):
        raise ValueError("pack_stream: a winner lies outside the domain grid")
    index_bits = max(1, int(nd).bit_length())
    t_bits = max(1, int(transforms - 1).bit_length())
    s_f = _Field(items["contrast"], contrast_bits)
    o_f = _Field(items["brightness"], brightness_bits)
    hdr = HEADER.pack(MAGIC, VERSION, 1 if use_classifier else 0, width, height, range_size, dsz, dstride, transforms,
                      contrast_bits, brightness_bits, index_bits, len(items), nd, s_f.min, s_f.max, o_f.min, o_f.max)
    body = _pack_bits([(idx, index_bits), (items["transform"].astype(np.uint64), t_bits),
                       (s_f.codes(items["contrast"]), contrast_bits), (o_f.codes(items["brightness"]), brightness_bits)],
                      len(items))
    return hdr + body


def read_header(buf: bytes) -> dict:
    if len(buf) < HEADER.size:
        raise ValueError("FRC1: truncated header")
    f = HEADER.unpack_from(buf, 0)
    if f[0] != MAGIC or f[1] != VERSION:
        raise ValueError("FRC1: bad magic or version")
    keys = ("magic", "version", "flags", "width", "height", "range_size", "domain_size", "domain_stride", "transforms",
            "contrast_bits", "brightness_bits", "index_bits", "n_ranges", "n_domains", "contrast_min",
            "contrast_max", "brightness_min", "brightness_max")
    return dict(zip(keys, f))


def unpack_stream(buf: bytes) -> tuple[np.ndarray, dict]:
    """FRC1 → (encode_item_t records with dequantized contrast/brightness, header dict).
    `distance` is not carried by the stream and comes back as 0."""
    from . import ENCODE_ITEM

    h = read_header(buf)
    n, nd = h["n_ranges"], h["n_domains"]
    t_bits = max(1, int(h["transforms"] - 1).bit_length())
    widths = [h["index_bits"], t_bits, h["contrast_bits"], h["brightness_bits"]]
    need = (n * sum(widths) + 7) // 8
    if len(buf) < HEADER.size + need:
        raise ValueError("FRC1: truncated records")
    idx, t, qs, qo = _unpack_bits(buf[HEADER.size:HEADER.size + need], n, widths)
    rc, _ = _grid_cols_rows(h["width"], h["height"], h["range_size"], h["range_size"])
    dc, _ = _grid_cols_rows(h["width"], h["height"], h["domain_size"], h["domain_stride"])
    out = np.zeros(n, dtype=ENCODE_ITEM)
    r = np.arange(n)
    out["x"] = (r % max(rc, 1)) * h["range_size"]
    out["y"] = (r // max(rc, 1)) * h["range_size"]
    out["w"] = out["h"] = h["range_size"]
    has = idx < nd
    if np.any(idx > nd):
        raise ValueError("FRC1: domain index out of range")
    di = np.where(has, idx, 0).astype(np.int64)
    out["dx"] = np.where(has, (di % max(dc, 1)) * h["domain_stride"], 0)
    out["dy"] = np.where(has, (di // max(dc, 1)) * h["domain_stride"], 0)
    out["sw"] = out["sh"] = np.where(has, h["domain_size"], 0)
    out["transform"] = t.astype(np.int32)

    def deq(codes, lo, hi, bits):
        if not hi > lo:
            return np.full(n, lo)
        return Quantizer(lo, hi, bits).value(codes)

    out["contrast"] = np.where(has, deq(qs, h["contrast_min"], h["contrast_max"], h["contrast_bits"]), 0.0)
    out["brightness"] = np.where(has, deq(qo, h["brightness_min"], h["brightness_max"], h["brightness_bits"]), 0.0)
    out["transform"] = np.where(has, out["transform"], 0)
    return out, h
