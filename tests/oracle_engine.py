"""Engine-interface stand-in on the CPU (test infrastructure): the oracle behind the methods the
multi-rank code and bench.main call on a HIP engine (set_frame / set_domains / set_ranges / run / fetch /
fetch_tuples / timing_history / rgb_to_yuv / classify / sync / close), so the sharding, the all-gathers and
bench.py's own main() run on `gloo` ranks in this container."""
import time

import numpy as np


class OracleEngine:
    """Engine-interface stand-in (CPU): the oracle's TransformEstimator2 restatement per run."""

    def __init__(self, plane=None, doms=None, use_classifier=False, transforms=4):
        from oracle import oracle as O
        self.O, self.plane = O, plane
        self.use_classifier = use_classifier
        self.T = transforms
        self.r = None
        self.rec = None
        self._times = []
        if doms is not None:
            self.set_domains(doms)

    @staticmethod
    def factory(dev, transforms, engine_id, timing=False):
        """bench.main's engine_factory signature."""
        return OracleEngine(transforms=transforms)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def close(self):
        pass

    def set_stream(self, handle):
        pass

    def set_frame(self, plane):
        self.plane = np.ascontiguousarray(plane, dtype=np.uint8)

    def set_domains(self, doms):
        self.doms = doms
        self.index = {(int(d["x"]), int(d["y"])): i for i, d in enumerate(doms)}

    def set_ranges(self, r):
        self.r = r

    def run(self):
        import fractencode_amd as F
        t0 = time.perf_counter()
        rec = np.zeros(len(self.r), dtype=F.ENCODE_ITEM)
        if len(self.r):
            out, _, _ = self.O.estimate(self.plane, self.doms, self.r.astype(self.O.ITEM_DTYPE), T=self.T, threads=2,
                                        use_classifier=self.use_classifier)
            rec["x"], rec["y"], rec["w"], rec["h"] = self.r["x"], self.r["y"], self.r["w"], self.r["h"]
            rec["distance"], rec["contrast"], rec["brightness"] = out["dist"], out["s"], out["o"]
            rec["transform"], rec["dx"], rec["dy"], rec["sw"], rec["sh"] = (out["t"], out["dx"], out["dy"], out["dw"],
                                                                            out["dh"])
        self.rec = rec
        ms = (time.perf_counter() - t0) * 1e3
        self._times.append((ms, 0.0, ms, 0.0))

    def fetch(self):
        nr, nd = len(self.rec), len(self.doms)
        return self.rec, {"engine": 1, "search_form": 0, "matrix_flops": 0, "fallback_ranges": 0,
                          "evaluated_mappings": nr * nd, "total_mappings": nr * nd, "rejected_mappings": 0}

    def timing_history(self):
        import fractencode_amd as F
        out = np.array(self._times[-256:], dtype=F.RUN_TIMING)
        self._times = []
        return out

    def classify(self, items, target_plane=False):
        out = items.copy()
        out["category"] = self.O.classify(self.plane, items.astype(self.O.ITEM_DTYPE))["category"]
        return out

    def rgb_to_yuv(self, rgb):
        return self.O.rgb2yuv(np.asarray(rgb))

    def fetch_tuples(self, out=None):
        import fractencode_amd as F
        t = np.zeros(len(self.rec), dtype=F.TUPLE) if out is None else out
        for k in ("transform", "contrast", "brightness", "distance"):
            t[k] = self.rec[k]
        t["domain"] = [self.index[(int(x), int(y))] if w else F.NO_DOMAIN
                       for x, y, w in zip(self.rec["dx"], self.rec["dy"], self.rec["sw"])]
        return t

    def sync(self):
        pass
