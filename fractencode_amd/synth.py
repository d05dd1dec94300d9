"""Synthetic grayscale frames for the benches and the full-size parity tests.

S1 (headline): 7-octave value noise.  Octave o is a
(2^(o+2)+1)^2 lattice of U[0,1) values drawn from SplitMix64 on a counter
(seed, octave, lattice index), bilinearly upsampled to W×H (pixel centres),
weighted 0.6^o, summed, min/max-normalised to [0, 255] and truncated to u8.
Every step is an elementwise float64 numpy op or an exact uint64 op, so the
frame is bit-identical on any IEEE host (checked by SHA-256 in the goldens).

S2 (stress): i.i.d. uniform u8 from numpy's PCG64 ``default_rng(seed)``.
"""
from __future__ import annotations

import hashlib

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    z = z + _GOLDEN
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def _lattice(seed: int, octave: int, cells: int) -> np.ndarray:
    n = cells + 1
    idx = np.arange(n * n, dtype=np.uint64)
    ctr = (np.uint64(seed) << np.uint64(32)) + (np.uint64(octave) << np.uint64(24)) + idx
    bits = _splitmix64(ctr) >> np.uint64(11)  # top 53 bits
    return (bits.astype(np.float64) * (1.0 / 9007199254740992.0)).reshape(n, n)


def value_noise(width: int, height: int, seed: int = 1234, octaves: int = 7, persistence: float = 0.6) -> np.ndarray:
    """S1 value-noise frame, uint8 [height, width], row-major (stride = width)."""
    with np.errstate(over="ignore"):
        acc = np.zeros((height, width), dtype=np.float64)
        weight = 1.0
        for o in range(octaves):
            cells = 2 ** (o + 2)
            lat = _lattice(seed, o, cells)
            ux = (np.arange(width, dtype=np.float64) + 0.5) * (cells / width)
            uy = (np.arange(height, dtype=np.float64) + 0.5) * (cells / height)
            ix = np.minimum(np.floor(ux).astype(np.int64), cells - 1)
            iy = np.minimum(np.floor(uy).astype(np.int64), cells - 1)
            fx = ux - ix
            fy = uy - iy
            v00 = lat[iy[:, None], ix[None, :]]
            v01 = lat[iy[:, None], ix[None, :] + 1]
            v10 = lat[iy[:, None] + 1, ix[None, :]]
            v11 = lat[iy[:, None] + 1, ix[None, :] + 1]
            top = v00 * (1.0 - fx)[None, :] + v01 * fx[None, :]
            bot = v10 * (1.0 - fx)[None, :] + v11 * fx[None, :]
            acc += weight * (top * (1.0 - fy)[:, None] + bot * fy[:, None])
            weight *= persistence
        lo, hi = acc.min(), acc.max()
        out = np.floor((acc - lo) * (255.0 / (hi - lo)))
        return np.clip(out, 0, 255).astype(np.uint8)


def uniform_noise(width: int, height: int, seed: int = 42) -> np.ndarray:
    """S2 stress frame: i.i.d. uniform u8."""
    return np.random.default_rng(seed).integers(0, 256, size=(height, width), dtype=np.uint8)


def sha256(plane: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(plane).tobytes()).hexdigest()
