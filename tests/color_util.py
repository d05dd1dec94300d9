"""The all-colours RGB layout of tools/make_golden.py (data generator, shared by tests)."""
import numpy as np


def all_colours_rgb(chunk: int) -> np.ndarray:
    """Chunk k (of 4) of the 2^24 colours, colour c on the 2×2 block at ((c%2048)·2, (c//2048)·2)."""
    c = np.arange(chunk << 22, (chunk + 1) << 22, dtype=np.uint32).reshape(2048, 2048)
    rgb = np.stack([(c >> 16) & 255, (c >> 8) & 255, c & 255], -1).astype(np.uint8)
    return np.repeat(np.repeat(rgb, 2, 0), 2, 1)
