"""Engine-interface stand-in on the CPU (test infrastructure): the oracle behind the methods the
multi-rank code calls on a HIP engine (set_frame / set_ranges / run / fetch_tuples / classify / sync),
so the sharding, the all-gather and bench.py's step run on `gloo` ranks in this container."""
import numpy as np


class OracleEngine:
    """Engine-interface stand-in (CPU): set_ranges / run / fetch_tuples / sync."""

    def __init__(self, plane, doms, use_classifier=False):
        from oracle import oracle as O
        self.O, self.plane, self.doms = O, plane, doms
        self.use_classifier = use_classifier
        self.index = {(int(d["x"]), int(d["y"])): i for i, d in enumerate(doms)}

    def set_frame(self, plane):
        self.plane = np.ascontiguousarray(plane, dtype=np.uint8)

    def set_ranges(self, r):
        self.r = r

    def run(self):
        import fractencode_amd as F
        out, _, _ = self.O.estimate(self.plane, self.doms, self.r.astype(self.O.ITEM_DTYPE), threads=2,
                                    use_classifier=self.use_classifier)
        rec = np.zeros(len(out), dtype=F.ENCODE_ITEM)
        rec["x"], rec["y"], rec["w"], rec["h"] = self.r["x"], self.r["y"], self.r["w"], self.r["h"]
        rec["distance"], rec["contrast"], rec["brightness"] = out["dist"], out["s"], out["o"]
        rec["transform"], rec["dx"], rec["dy"], rec["sw"], rec["sh"] = out["t"], out["dx"], out["dy"], out["dw"], out["dh"]
        self.rec = rec

    def classify(self, items, target_plane=False):
        out = items.copy()
        out["category"] = self.O.classify(self.plane, items.astype(self.O.ITEM_DTYPE))["category"]
        return out

    def fetch_tuples(self):
        import fractencode_amd as F
        t = np.zeros(len(self.rec), dtype=F.TUPLE)
        for k in ("transform", "contrast", "brightness", "distance"):
            t[k] = self.rec[k]
        t["domain"] = [self.index[(int(x), int(y))] if w else F.NO_DOMAIN
                       for x, y, w in zip(self.rec["dx"], self.rec["dy"], self.rec["sw"])]
        return t

    def sync(self):
        pass
