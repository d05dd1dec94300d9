"""Loading of the committed golden vectors (tests/golden/, made by tools/make_golden.py
from the unmodified reference build)."""
from __future__ import annotations

import json
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIELDS = ("x", "y", "dx", "dy", "dw", "dh", "t", "dist", "s", "o")


def manifest() -> dict:
    with open(os.path.join(GOLD, "manifest.json")) as f:
        return json.load(f)


def plane(name: str) -> np.ndarray:
    m = manifest()[name]
    if name == "s1_4096":
        from fractencode_amd.synth import value_noise
        p = value_noise(4096, 4096, 1234)
    elif name == "s1_2048":
        from fractencode_amd.synth import value_noise
        p = value_noise(4096, 4096, 1234)[:2048, :2048].copy()
    elif name in ("c5_y", "c5_u", "c5_v"):
        p = c5_planes()[("c5_y", "c5_u", "c5_v").index(name)]
    else:
        p = np.fromfile(os.path.join(GOLD, name + ".u8"), dtype=np.uint8).reshape(m["shape"])
    from fractencode_amd.synth import sha256
    assert sha256(p) == m["sha256"], f"fixture plane {name} drifted"
    return p


def c5_rgb() -> np.ndarray:
    """C5's frame: the S1 RGB 4096² (value noise seeds 1234, 1235, 1236 as R, G, B)."""
    from fractencode_amd.synth import value_noise
    return np.stack([value_noise(4096, 4096, 1234 + k) for k in range(3)], -1)


_C5 = None


def c5_planes():
    """Y, U, V of the C5 frame by the oracle's rgb2yuv (its digests are the reference's, manifest)."""
    global _C5
    if _C5 is None:
        from oracle import oracle as O
        _C5 = O.rgb2yuv(c5_rgb())
    return _C5


def golden(name: str):
    z = np.load(os.path.join(GOLD, name + ".npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    rec = {k: z[k] for k in FIELDS}
    return rec, meta


def selection(meta: dict, n_ranges: int):
    sel = meta.get("sel")
    if sel is None:
        return None
    if sel.startswith("arange("):
        a, b, c = (int(v) for v in sel[len("arange("):-1].split(","))
        return np.arange(a, b, c)
    raise ValueError(sel)


def grid_specs(meta: dict, W: int, H: int):
    """(domain spec, range spec) of a golden as createUniformGrid arguments (area W, H, item w, h,
    offset x, y): the CLI's square grids (domains src at offset src/2, main.cpp:147) for an int
    src/tgt, the stored Size32u specs of the rectangular goldens otherwise."""
    src, tgt = meta["src"], meta["tgt"]
    d = (W, H, src, src, src // 2, src // 2) if np.isscalar(src) else tuple(src)
    r = (W, H, tgt, tgt, tgt, tgt) if np.isscalar(tgt) else tuple(tgt)
    return d, r


def make_grids(uniform_grid, classify, p: np.ndarray, meta: dict):
    """The golden's domain and range grids by `uniform_grid(W, H, size, offset)` (the engine's or the
    oracle's), preclassified on the plane when the golden has the classifier (main.cpp:155-162)."""
    H, W = p.shape
    d, r = grid_specs(meta, W, H)
    doms = uniform_grid(d[0], d[1], (d[2], d[3]), (d[4], d[5]))
    rngs = uniform_grid(r[0], r[1], (r[2], r[3]), (r[4], r[5]))
    if meta["cls"]:
        doms = classify(p, doms)
        rngs = classify(p, rngs)
    return doms, rngs


# per-range search goldens (decode / quantizer / colour / classifier fixtures live beside them)
GOLDEN_NAMES = sorted(f[:-4] for f in os.listdir(GOLD)
                      if f.endswith(".npz") and not f.endswith(("_decode.npz", "_quant.npz"))
                      and not f.startswith(("rgb_", "opencl_")))


_MAP = (("x", "x"), ("y", "y"), ("dx", "dx"), ("dy", "dy"), ("sw", "dw"), ("sh", "dh"), ("transform", "t"),
        ("distance", "dist"), ("contrast", "s"), ("brightness", "o"))


def encode_items(rec: dict, range_size: int) -> np.ndarray:
    """Golden / oracle per-range records → encode_item_t records (fractencode_amd.ENCODE_ITEM)."""
    from fractencode_amd import ENCODE_ITEM

    out = np.zeros(len(rec["x"]), dtype=ENCODE_ITEM)
    for a, b in _MAP:
        out[a] = rec[b]
    out["w"] = out["h"] = range_size
    return out


def oracle_records(items: np.ndarray) -> np.ndarray:
    """encode_item_t records → the oracle's result records (oracle.RESULT_DTYPE)."""
    from oracle.oracle import RESULT_DTYPE

    out = np.zeros(len(items), dtype=RESULT_DTYPE)
    for a, b in _MAP:
        out[b] = items[a]
    return out
