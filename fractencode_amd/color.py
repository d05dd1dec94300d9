"""Colour frames: main.cpp's --color mode on the device.

The reference loads a PNG, converts it with ImageIO::rgb2yuv (image/ImageIO.cpp:43-58)
and encodes the three planes independently, each with its own grids and classifier
(main.cpp:184-196 → encode_image2, main.cpp:142-180).  Here the RGB frame is uploaded
once, converted on the device (frac_rgb_to_yuv_device), and the Y, U and V searches
are enqueued on three engines that share one HIP stream, so the searches run in turn: the luma
search alone fills the GPU, and letting the small chroma searches overlap it on streams of their
own measured slower (C5: 12.73 vs 12.54 ms per frame for the three searches, 13.32 vs 12.69 ms with
the conversion; profiles/r03/session5/paths.jsonl).  streams="own" keeps one stream per engine.
"""
from __future__ import annotations

import numpy as np

from . import ENGINE_AUTO, Engine, create_uniform_grid

PLANES = ("Y", "U", "V")


class ColorEncoder:
    """Three-plane encoder.  load(rgb) → run() → sync() → fetch(), engines reused across frames."""

    def __init__(self, device: int = 0, range_size: int = 8, domain_size: int | None = None, transforms: int = 4,
                 use_classifier: bool = False, rms_threshold: float = 0.0, s_max: float = -1.0,
                 engine: int = ENGINE_AUTO, timing: bool = False, streams: str = "shared"):
        if streams not in ("shared", "own"):
            raise ValueError(f"streams must be 'shared' or 'own', not {streams!r}")
        self.device = device
        self.range_size = range_size
        self.domain_size = domain_size or 2 * range_size
        self.use_classifier = use_classifier
        self.engines = [Engine(device, transforms, use_classifier, rms_threshold, s_max, engine, timing) for _ in PLANES]
        self._stream = None
        if streams == "shared":
            import torch

            self._stream = torch.cuda.Stream(torch.device("cuda", device))
            for e in self.engines:
                e.set_stream(self._stream.cuda_stream)
        self.planes = None
        self.ranges = None

    def close(self) -> None:
        for e in self.engines:
            e.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def load(self, rgb) -> None:
        """rgb: numpy uint8 [H, W, 3] or a CUDA uint8 tensor [H, W, 3]; converted on the device."""
        import torch

        if not (hasattr(rgb, "is_cuda") and rgb.is_cuda):
            rgb = torch.from_numpy(np.ascontiguousarray(rgb, dtype=np.uint8)).to(f"cuda:{self.device}")
        planes = self.engines[0].rgb_to_yuv(rgb)
        self.planes = planes
        n, d = self.range_size, self.domain_size
        geom = [tuple(p.shape) for p in planes]
        same = geom == getattr(self, "_geom", None)
        if not same:
            self.ranges = []
        sharded = getattr(self, "_sharded", False)
        self._sharded = False
        for k, (e, p) in enumerate(zip(self.engines, planes)):
            H, W = p.shape
            e.set_frame(p)
            if same:
                if sharded:  # encode_sharded left each engine holding only this rank's shard
                    e.set_ranges(self.ranges[k])
                continue  # a frame of the same geometry keeps the grids (and, classifier off, the prepared state)
            # categories −1: with the classifier on, the engine classifies every item on the
            # device plane (main.cpp:155-162 preclassifies both grids on the same plane)
            doms = create_uniform_grid(W, H, d, d // 2)
            rngs = create_uniform_grid(W, H, n, n)
            e.set_domains(doms)
            e.set_ranges(rngs)
            self.ranges.append(rngs)
        self._geom = geom

    def run(self) -> None:
        """Enqueue the three searches (asynchronous; on the shared stream, or each engine's own)."""
        for e in self.engines:
            e.run()

    def sync(self) -> None:
        for e in self.engines:
            e.sync()

    def fetch(self):
        """[(encode items, stats)] for Y, U, V."""
        return [e.fetch() for e in self.engines]

    def encode_sharded(self, rank: int, world: int, device=None, group=None):
        """C5 over several GPUs (BASELINE configs[4]): after load(), every rank searches its
        contiguous shard of each plane's ranges and the (domain, transform, s, o, rms) tuples are
        all-gathered (fractencode_amd.distributed); returns the full Y, U, V encode_item_t arrays
        on every rank.  `device` = a CUDA device for nccl, None for gloo (host tuples)."""
        from .distributed import encode_sharded

        self._sharded = True  # the next load() of a same-geometry frame restores the full range lists
        out = []
        for e, rngs, p in zip(self.engines, self.ranges, self.planes):
            H, W = p.shape
            doms = create_uniform_grid(W, H, self.domain_size, self.domain_size // 2)
            out.append(encode_sharded(e, rngs, doms, rank, world, device=device, group=group))
        return out

    def host_planes(self):
        return [p.cpu().numpy() for p in self.planes]


def encode_color(rgb, **kw):
    """Convert + encode one RGB frame; returns ([Y, U, V] host planes, [(items, stats)] per plane)."""
    with ColorEncoder(**kw) as enc:
        enc.load(rgb)
        enc.run()
        enc.sync()
        return enc.host_planes(), enc.fetch()
