"""GPU parity of the HIP search engine against the reference goldens and the oracle.

Bar: bit-exact (domain, transform, distance, contrast, brightness) — the fit is
exact in FP64 and the distance is the reference's fp32 value — plus the
reference's rejected-mapping counts.  All calls go through the C ABI.
"""
import zlib

import numpy as np
import pytest

import fractencode_amd as F
from golden_util import FIELDS, GOLDEN_NAMES, golden, make_grids, plane, selection

pytestmark = pytest.mark.gpu

# every golden runs on every engine: the ratio-2 path (domain = 2 × range, n ∈ {2, 4, 8, 16}) and
# the sampled form for every other geometry (16→4 — the CLI default — 32→8, 12→8, 8→3, 64→32 ...)
ENGINES = [F.ENGINE_VALU, F.ENGINE_MFMA, F.ENGINE_SEA]


def as_oracle_fields(out):
    return {"x": out["x"], "y": out["y"], "dx": out["dx"], "dy": out["dy"], "dw": out["sw"], "dh": out["sh"],
            "t": out["transform"], "dist": out["distance"], "s": out["contrast"], "o": out["brightness"]}


def run_engine(p, meta, engine, tgt=None, ranges_idx=None, flags=0):
    doms, rngs = make_grids(F.create_uniform_grid, F.preclassify, p, meta)
    if ranges_idx is not None:
        rngs = rngs[ranges_idx]
    with F.Engine(0, meta["T"], meta["cls"], meta["thr"], meta["smax"], engine, flags=flags) as e:
        e.set_frame(p)
        e.set_domains(doms)
        return e.search(rngs)


def assert_same(got, want, what):
    g = as_oracle_fields(got)
    for k in FIELDS:
        np.testing.assert_array_equal(g[k], want[k], err_msg=f"{what}: field {k}")


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_engine_matches_reference_goldens(name, engine):
    rec, meta = golden(name)
    p = plane(meta["plane"])
    sel = selection(meta, len(rec["x"]))
    out, st = run_engine(p, meta, engine, ranges_idx=sel)
    assert_same(out, rec, name)
    if sel is None:
        assert st["rejected_mappings"] == meta["rejected"]


def _random_plane(rng, W, H, kind):
    if kind == "uniform":
        return rng.integers(0, 256, (H, W), dtype=np.uint8)
    if kind == "flat":
        # many exact matches (threshold hits, ties)
        return (rng.integers(0, 3, (H // 4, W // 4), dtype=np.uint8) * 60).repeat(4, 0).repeat(4, 1)
    from fractencode_amd.synth import value_noise
    return value_noise(W, H, int(rng.integers(1 << 30)))


CASES = [
    # W, H, n, T, classifier, thr, smax, kind
    (64, 64, 8, 4, False, 0.0, -1.0, "uniform"),
    (96, 64, 8, 8, False, 0.0, -1.0, "noise"),
    (64, 96, 8, 4, True, 0.0, -1.0, "noise"),
    (64, 64, 8, 8, True, 2.5, 0.7, "flat"),
    (64, 64, 8, 4, False, 0.0, -1.0, "flat"),
    (48, 48, 4, 4, False, 1.0, -1.0, "noise"),
    (48, 32, 4, 8, True, 0.0, 2.0, "uniform"),
    (32, 32, 2, 4, False, 0.0, -1.0, "noise"),
    (32, 32, 2, 8, True, 0.0, -1.0, "flat"),
    (96, 96, 16, 4, False, 0.0, -1.0, "noise"),
    (128, 96, 16, 8, True, 30.0, -1.0, "uniform"),
    (64, 64, 16, 8, False, 0.0, -1.0, "flat"),     # n = 16 ties (MFMA integer epilogue)
    (96, 64, 16, 4, True, 0.0, 0.5, "noise"),
    (256, 256, 16, 4, False, 0.0, -1.0, "flat"),   # n = 16, 8 tiles: ties across tiles, first tile wins
    (256, 192, 16, 4, False, 40.0, -1.0, "flat"),  # n = 16 threshold hits across tiles (T = 4)
    (256, 256, 4, 4, False, 0.0, -1.0, "flat"),    # n = 4, 125 tiles in splits: ties across tiles and work items
    (256, 192, 4, 8, False, 40.0, -1.0, "flat"),   # n = 4 threshold hits across tiles and work items (T = 8)
    (70, 58, 4, 4, True, 0.0, -1.0, "noise"),      # classifier keys from block sums: plane sides not multiples of 4
    (98, 74, 8, 4, True, 0.0, -1.0, "uniform"),    # ... nor of 8 (partial blocks at the right and bottom edges)
    (64, 64, 8, 4, False, 1e9, -1.0, "noise"),   # every candidate hits: all-fallback mode
    (64, 64, 8, 8, False, 5000.0, -1.0, "uniform"),
]


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("case", range(len(CASES)))
def test_engine_matches_oracle_random(oracle, case, engine):
    W, H, n, T, cls, thr, smax, kind = CASES[case]
    rng = np.random.default_rng(1000 + case)
    p = _random_plane(rng, W, H, kind)
    meta = dict(src=2 * n, tgt=n, T=T, cls=cls, thr=thr, smax=smax)
    out, st = run_engine(p, meta, engine)
    doms = oracle.uniform_grid(W, H, 2 * n, n)
    rngs = oracle.uniform_grid(W, H, n, n)
    if cls:
        doms = oracle.classify(p, doms)
        rngs = oracle.classify(p, rngs)
    want, rej, _ = oracle.estimate(p, doms, rngs, T=T, thr=thr, smax=smax, use_classifier=cls)
    assert_same(out, {k: want[k] for k in FIELDS}, f"case {CASES[case]}")
    assert st["rejected_mappings"] == rej


@pytest.mark.parametrize("engine", ENGINES)
def test_distinct_planes_with_the_classifier(oracle, engine):
    """Source and target planes differ and the classifier is on: the domains' keys come from the source
    plane's block sums, the ranges' from the target's (bucket_keys_bs), against the oracle."""
    rng = np.random.default_rng(77)
    src = _random_plane(rng, 96, 80, "noise")
    tgt = _random_plane(rng, 48, 40, "uniform")
    with F.Engine(0, 4, True, 0.0, -1.0, engine) as e:
        e.set_planes(src, tgt)
        e.set_domains(F.create_uniform_grid(96, 80, 8, 4))
        e.set_ranges(F.create_uniform_grid(48, 40, 4, 4))
        e.run()
        out, st = e.fetch()
    doms = oracle.classify(src, oracle.uniform_grid(96, 80, 8, 4))
    rngs = oracle.classify(tgt, oracle.uniform_grid(48, 40, 4, 4))
    want, rej, _ = oracle.estimate(src, doms, rngs, T=4, use_classifier=True, tgt=tgt)
    assert_same(out, {k: want[k] for k in FIELDS}, "distinct planes, classifier")
    assert st["rejected_mappings"] == rej


@pytest.mark.parametrize("engine", ENGINES)
def test_distinct_source_and_target_planes(engine):
    # reference tests/TransformEstimatorTest.cpp:14-47 (source 8×8, target 4×4)
    src = np.array([[1, 1, 2, 2, 40, 41, 50, 51], [1, 1, 2, 2, 40, 41, 50, 51], [3, 3, 4, 4, 70, 71, 80, 81],
                    [3, 3, 4, 4, 70, 71, 80, 81], [10, 10, 10, 10, 0, 0, 0, 0], [11, 11, 11, 11, 1, 1, 1, 1],
                    [10, 10, 10, 10, 0, 0, 0, 0], [11, 11, 11, 11, 1, 1, 1, 1]], np.uint8)
    tgt = np.array([[40, 50, 2, 4], [70, 80, 1, 3], [0, 0, 10, 10], [1, 1, 11, 11]], np.uint8)
    with F.Engine(0, 4, False, 0.0, 100.0, engine) as e:
        e.set_planes(src, tgt)
        e.set_domains(F.create_uniform_grid(8, 8, 4, 2))
        out, _ = e.search(F.create_uniform_grid(4, 4, 2, 2))
    got = {(int(r["x"]), int(r["y"])): (int(r["dx"]), int(r["dy"])) for r in out}
    assert got == {(0, 0): (4, 0), (2, 0): (0, 0), (0, 2): (4, 4), (2, 2): (0, 4)}
    # TransformMatcherTest.cpp:13-35: range (0,0) vs domain (0,0) is an exact Rotate_270 match
    with F.Engine(0, 4, False, 0.0, 100.0, engine) as e:
        s2 = np.array([[1, 1, 2, 2, 40, 41, 50, 51], [1, 1, 2, 2, 40, 41, 50, 51], [3, 3, 4, 4, 70, 71, 80, 81],
                       [3, 3, 4, 4, 70, 71, 80, 81], [0] * 8, [1] * 8, [0] * 8, [1] * 8], np.uint8)
        t2 = np.array([[2, 4, 40, 50], [1, 3, 70, 80], [0, 0, 0, 0], [1, 1, 1, 1]], np.uint8)
        e.set_planes(s2, t2)
        e.set_domains(np.array([(0, 0, 4, 4, -1)], dtype=F.GRID_ITEM))
        out, _ = e.search(np.array([(0, 0, 2, 2, -1)], dtype=F.GRID_ITEM))
    assert out["distance"][0] == 0.0 and out["transform"][0] == 3
    assert out["contrast"][0] < 1.0 and out["brightness"][0] < 1.0


@pytest.mark.parametrize("engine", ENGINES)
def test_edge_cases(oracle, engine):
    rng = np.random.default_rng(5)
    p = rng.integers(0, 256, (64, 64), dtype=np.uint8)
    rngs = F.create_uniform_grid(64, 64, 8, 8)
    with F.Engine(0, 4, False, 0.0, -1.0, engine) as e:
        e.set_frame(p)
        # no domains at all: every range gets the default item_match_t (datatypes.h:8-19)
        e.set_domains(np.zeros(0, dtype=F.GRID_ITEM))
        out, st = e.search(rngs)
        assert (out["distance"] == 100000.0).all() and (out["sw"] == 0).all() and st["empty_ranges"] == 64
        # no ranges
        e.set_domains(F.create_uniform_grid(64, 64, 16, 8))
        out, st = e.search(np.zeros(0, dtype=F.GRID_ITEM))
        assert len(out) == 0
        # ragged range list in arbitrary order (results come back in that order)
        perm = rng.permutation(len(rngs))[:37]
        out, _ = e.search(rngs[perm])
        want, _, _ = oracle.estimate(p, oracle.uniform_grid(64, 64, 16, 8), oracle.uniform_grid(64, 64, 8, 8)[perm])
        assert_same(out, {k: want[k] for k in FIELDS}, "ragged")
        # repeated runs are deterministic
        out2, _ = e.search(rngs[perm])
        assert out.tobytes() == out2.tobytes()
    # classifier with a category that no domain has: rejected = nd for those ranges
    doms = F.preclassify(p, F.create_uniform_grid(64, 64, 16, 8))
    rg = F.preclassify(p, rngs)
    doms = doms[doms["category"] != rg["category"][0]]
    with F.Engine(0, 4, True, 0.0, -1.0, engine) as e:
        e.set_frame(p)
        e.set_domains(doms)
        out, st = e.search(rg)
        # the 32-byte gather tuples rebuild the same records, default records included
        from fractencode_amd.distributed import records_from_tuples
        tup = e.fetch_tuples()
        assert (tup["domain"] == F.NO_DOMAIN).sum() == st["empty_ranges"]
        assert records_from_tuples(tup, rg, doms).tobytes() == out.tobytes()
    want, rej, _ = oracle.estimate(p, doms, rg, use_classifier=True)
    assert_same(out, {k: want[k] for k in FIELDS}, "empty bucket")
    assert st["rejected_mappings"] == rej and st["empty_ranges"] > 0


@pytest.mark.parametrize("engine", ENGINES)
def test_invalid_geometry_is_an_error(engine):
    # what the reference CLI rejects (main.cpp:99: target >= source) or cannot express
    p = np.zeros((64, 64), np.uint8)
    with F.Engine(0, 4, engine=engine) as e:
        e.set_frame(p)
        e.set_domains(F.create_uniform_grid(64, 64, 8, 4))  # domains no larger than the ranges
        with pytest.raises(F.FracError):
            e.search(F.create_uniform_grid(64, 64, 8, 8))
        mixed = np.concatenate([F.create_uniform_grid(64, 64, 16, 8), F.create_uniform_grid(64, 64, 12, 6)])
        with pytest.raises(F.FracError):  # domains of two sizes: refused when set
            e.set_domains(mixed)
        e.set_domains(F.create_uniform_grid(64, 64, 16, 8))
        bad = np.array([(60, 60, 8, 8, -1)], dtype=F.GRID_ITEM)  # outside the plane
        with pytest.raises(F.FracError):
            e.search(bad)
    with F.Engine(0, 4, engine=engine) as e:
        e.set_frame(np.zeros((512, 512), np.uint8))
        e.set_domains(F.create_uniform_grid(512, 512, 512, 256))
        with pytest.raises(F.FracError, match="at least 2"):
            e.search(np.array([(0, 0, 1, 1, -1)], dtype=F.GRID_ITEM))
        out, _ = e.search(np.array([(0, 0, 256, 256, -1)], dtype=F.GRID_ITEM))  # the largest exact-search side
        assert out["sw"][0] == 512 and out["distance"][0] == 0.0


@pytest.mark.parametrize("cls", [False, True])
@pytest.mark.parametrize("engine", ENGINES)
def test_range_sides_above_256(oracle, engine, cls):
    """Range sides above 256 (the CLI accepts any 2 <= target < source, main.cpp:99; match_generic any size,
    transformmatcher.h:80-111): every candidate in the reference's fp32 arithmetic (gen_fallback), records
    equal to the oracle's — 320×320 ranges against 640×640 domains at stride 320 on a 1024² S1 frame, and
    rectangles of 272×300 against 544×600 at stride (272, 300)."""
    from fractencode_amd.synth import value_noise

    p = value_noise(1024, 1024, 77)
    for (rw, rh) in ((320, 320), (272, 300)):
        doms = F.create_uniform_grid(1024, 1024, (2 * rw, 2 * rh), (rw, rh))
        rngs = F.create_uniform_grid(1024, 1024, (rw, rh), (rw, rh))
        if cls:
            doms, rngs = F.preclassify(p, doms), F.preclassify(p, rngs)
        with F.Engine(0, 4, cls, 0.0, -1.0, engine) as e:
            e.set_frame(p)
            e.set_domains(doms)
            out, st = e.search(rngs)
        want, rej, _ = oracle.estimate(p, doms.astype(oracle.ITEM_DTYPE), rngs.astype(oracle.ITEM_DTYPE),
                                       use_classifier=cls)
        assert_same(out, {k: want[k] for k in FIELDS}, f"{rw}x{rh}")
        assert st["fallback_ranges"] == len(rngs) - st["empty_ranges"]
        if cls:
            assert st["rejected_mappings"] == rej


def _recompute_s16(p, out, n=8):
    """Independent numpy recomputation of the exact error of each chosen (domain, t)."""
    rx, ry, dx, dy, t = (out[k].astype(np.int64) for k in ("x", "y", "dx", "dy", "transform"))
    yy, xx = np.divmod(np.arange(n * n), n)
    r = p[ry[:, None] + yy[None, :], rx[:, None] + xx[None, :]].astype(np.int64)
    fwd = np.array([[F.transform_index(n, tt, q) for q in range(n * n)] for tt in range(8)])
    q = fwd[t]  # [N, n²] decimated cell met by each range pixel
    qy, qx = np.divmod(q, n)
    X0 = dx[:, None] + 2 * qx
    Y0 = dy[:, None] + 2 * qy
    pi = p.astype(np.int64)
    D = pi[Y0, X0] + pi[Y0, X0 + 1] + pi[Y0 + 1, X0] + pi[Y0 + 1, X0 + 1]
    return ((4 * r - D) ** 2).sum(1)


@pytest.mark.parametrize("engine", ENGINES)
def test_full_4096_frame(engine):
    """C3 at full size: the 1,024 reference-sampled ranges match bit-exactly, and every
    range's distance is the exact error of the (domain, transform) it reports."""
    rec, meta = golden("s1_4096_sample")
    p = plane("s1_4096")
    doms = F.create_uniform_grid(4096, 4096, 16, 8)
    rngs = F.create_uniform_grid(4096, 4096, 8, 8)
    with F.Engine(0, 4, False, 0.0, -1.0, engine, timing=True) as e:
        e.set_frame(p)
        e.set_domains(doms)
        out, st = e.search(rngs)
    sel = selection(meta, len(rngs))
    assert_same(out[sel], rec, "s1_4096 sample")
    s16 = _recompute_s16(p, out)
    exact = s16 < (1 << 24)
    np.testing.assert_array_equal(out["distance"][exact], (s16[exact] / 16.0) / 256.0)
    assert st["fallback_ranges"] == int((~exact).sum())
    assert (out["sw"] == 16).all()


def test_sea_n16_runs_the_exhaustive_search():
    """SEA covers n ≤ 8; a valid 32→16 geometry runs the exhaustive MFMA search (same records)."""
    rec, meta = golden("lenna_n16")
    out, st = run_engine(plane("lenna_y"), meta, F.ENGINE_SEA)
    assert_same(out, rec, "lenna_n16 via SEA")
    assert st["engine"] == F.ENGINE_MFMA


def test_engines_agree_on_stress_frame():
    """VALU, MFMA and SEA engines on a uniform-noise 1024² frame (S2, where the SEA bound is
    loose): identical records."""
    from fractencode_amd.synth import uniform_noise
    p = uniform_noise(1024, 1024, 42)
    outs = []
    for eng in (F.ENGINE_VALU, F.ENGINE_MFMA, F.ENGINE_SEA):
        with F.Engine(0, 8, False, 0.0, -1.0, eng) as e:
            e.set_frame(p)
            e.set_domains(F.create_uniform_grid(1024, 1024, 16, 8))
            out, st = e.search(F.create_uniform_grid(1024, 1024, 8, 8))
            assert st["engine"] == eng
            outs.append(out)
    assert outs[0].tobytes() == outs[1].tobytes()
    assert outs[0].tobytes() == outs[2].tobytes()


DFT_CASES = [
    # W, H, classifier, thr, smax, kind — n = 8, T = 4 (the C4-Fourier MFMA path)
    (128, 128, False, 0.0, -1.0, "uniform"),
    (128, 96, True, 0.0, -1.0, "noise"),
    (96, 96, False, 2.5, -1.0, "flat"),      # threshold hits (first hit in (domain, t) order)
    (96, 64, True, 0.0, 0.5, "flat"),        # exact matches, ties across transforms
    (64, 64, False, 0.0, -1.0, "flat"),
    (160, 96, False, 40.0, -1.0, "noise"),
]


@pytest.mark.parametrize("form", ["fourier", "direct"])
@pytest.mark.parametrize("case", range(len(DFT_CASES)))
def test_mfma_fourier_and_direct_match_oracle(oracle, case, form):
    # the shipped Fourier form (six MFMAs, guarded constant-folded epilogue) and the direct form
    # (FRAC_FLAG_DIRECT_FORM); the A/B variants of the tuning build are not in the product library
    flags = F.FLAG_DIRECT_FORM if form == "direct" else 0
    W, H, cls, thr, smax, kind = DFT_CASES[case]
    rng = np.random.default_rng(2000 + case)
    p = _random_plane(rng, W, H, kind)
    meta = dict(src=16, tgt=8, T=4, cls=cls, thr=thr, smax=smax)
    out, st = run_engine(p, meta, F.ENGINE_MFMA, flags=flags)
    assert st["search_form"] == (F.FORM_DIRECT if flags else F.FORM_FOURIER)
    doms = oracle.uniform_grid(W, H, 16, 8)
    rngs = oracle.uniform_grid(W, H, 8, 8)
    if cls:
        doms = oracle.classify(p, doms)
        rngs = oracle.classify(p, rngs)
    want, rej, _ = oracle.estimate(p, doms, rngs, T=4, thr=thr, smax=smax, use_classifier=cls)
    assert_same(out, {k: want[k] for k in FIELDS}, f"{form} case {DFT_CASES[case]}")
    assert st["rejected_mappings"] == rej


def _extreme_plane(rng, S, kind):
    # frames that drive the Fourier operands to their bounds: pixels only 0 or 255, as i.i.d.
    # noise, as 8×8 / 2×2 constant blocks, and as per-orbit patterns (one rotation orbit of an
    # 8×8 block bright, its image under Rotate_90 dark: |α|, |β|, |γ|, |δ| at their maxima)
    if kind == "binary":
        return (rng.integers(0, 2, (S, S)) * 255).astype(np.uint8)
    if kind == "blocks8":
        return (rng.integers(0, 2, (S // 8, S // 8)) * 255).astype(np.uint8).repeat(8, 0).repeat(8, 1)
    if kind == "blocks2":
        return (rng.integers(0, 2, (S // 2, S // 2)) * 255).astype(np.uint8).repeat(2, 0).repeat(2, 1)
    # "orbits": every 8×8 block and every 2×2-decimated 16×16 block alternates 0/255 around
    # each rotation orbit, with a random phase per block
    yy, xx = np.mgrid[0:8, 0:8]
    ring = ((yy + xx) % 2) ^ ((yy < 4) & (xx < 4)).astype(int)
    tiles = [ring, np.rot90(ring), 1 - ring, np.rot90(1 - ring)]
    pick = rng.integers(0, 4, (S // 8, S // 8))
    out = np.block([[tiles[k] for k in row] for row in pick]) * 255
    return out.astype(np.uint8)


@pytest.mark.parametrize("form", ["fourier", "direct"])
@pytest.mark.parametrize("kind", ["binary", "blocks8", "blocks2", "orbits"])
def test_mfma_forms_at_operand_extremes(kind, form):
    """The six-MFMA Fourier form's guarded fast path (P from −Σb²/2 where 2·R6·D6 + Σb² < 2^24) has
    the tightest exactness margin, 2Pr / 2Pi the next (partial sums up to 33.3M < 2^25): on 0/255
    frames that drive every operand to its bound the shipped form and the direct form
    (FRAC_FLAG_DIRECT_FORM) return the exhaustive VALU engine's records, with and without the
    classifier."""
    rng = np.random.default_rng(zlib.crc32(kind.encode()))  # reproducible across processes
    S = 256
    p = _extreme_plane(rng, S, kind)
    doms, rngs = F.create_uniform_grid(S, S, 16, 8), F.create_uniform_grid(S, S, 8, 8)
    for cls in (False, True):
        with F.Engine(0, 4, cls, 0.0, -1.0, F.ENGINE_VALU) as e:
            e.set_frame(p)
            e.set_domains(doms)
            want, wst = e.search(rngs)
        with F.Engine(0, 4, cls, 0.0, -1.0, F.ENGINE_MFMA,
                      flags=F.FLAG_DIRECT_FORM if form == "direct" else 0) as e:
            e.set_frame(p)
            e.set_domains(doms)
            out, st = e.search(rngs)
        assert out.tobytes() == want.tobytes(), f"{kind} cls={cls}"
        assert st["rejected_mappings"] == wst["rejected_mappings"]


@pytest.mark.parametrize("n", [2, 4])
@pytest.mark.parametrize("kind", ["binary", "blocks2", "noise"])
def test_float_c_epilogue_at_operand_extremes(n, kind):
    """n ≤ 4 runs the direct form with the float-C epilogue (search_mfma VAR 386): the accumulator starts
    from the domain row's ΣD4² − 1024·ΣD4 and the B operand is 8·(128 − r), exact while every partial sum
    stays below 2^24 (2^22 + 8·n²·128·510).  On 0/255 frames that drive both to their bounds, with T = 4 / 8,
    the classifier and a hit threshold, the records and reject counts equal the VALU engine's; the sampled
    form's T = 1 rows (16→4) too."""
    rng = np.random.default_rng(zlib.crc32(f"fc{kind}{n}".encode()))
    S = 128
    p = rng.integers(0, 256, (S, S), dtype=np.uint8) if kind == "noise" else _extreme_plane(rng, S, kind)
    cases = [(2 * n, 4, False, 0.0), (2 * n, 8, True, 0.0), (2 * n, 4, False, 30.0)]
    if n == 4:
        cases.append((16, 4, True, 0.0))  # 16 → 4: the sampled form's search_mfma<4, 1>
    for src, T, cls, thr in cases:
        doms, rngs = F.create_uniform_grid(S, S, src, src // 2), F.create_uniform_grid(S, S, n, n)
        outs = {}
        for eng in (F.ENGINE_VALU, F.ENGINE_MFMA):
            with F.Engine(0, T, cls, thr, -1.0, eng) as e:
                e.set_frame(p)
                e.set_domains(doms)
                outs[eng] = e.search(rngs)
        (a, sa), (b, sb) = outs[F.ENGINE_VALU], outs[F.ENGINE_MFMA]
        assert sb["engine"] == F.ENGINE_MFMA
        assert a.tobytes() == b.tobytes(), f"{kind} n={n} src={src} T={T} cls={cls} thr={thr}"
        assert sa["rejected_mappings"] == sb["rejected_mappings"] and sa["hit_ranges"] == sb["hit_ranges"]


@pytest.mark.parametrize("kind", ["binary", "blocks8", "orbits", "noise"])
def test_t8_fourier_flipped_copies_at_operand_extremes(kind):
    """T = 8 on the Fourier path: each range block runs a second time read through Flip
    (Flip_Rotate_k = Flip ∘ Rotate_k, dft_range_prep flip_from) and resolve_dft keeps the lesser key of
    the two copies, with the copy's rotation t' as transform 4 + (−t' mod 4).  On the operand-extreme
    frames and on noise, with and without the classifier and with a hit threshold (the first hit in
    (domain, transform) order, image/metrics.h + TransformEstimator2.hpp:34-41), the records equal the
    exhaustive VALU engine's and the direct MFMA form's."""
    rng = np.random.default_rng(zlib.crc32(("t8" + kind).encode()))
    S = 256
    p = rng.integers(0, 256, (S, S), dtype=np.uint8) if kind == "noise" else _extreme_plane(rng, S, kind)
    doms, rngs = F.create_uniform_grid(S, S, 16, 8), F.create_uniform_grid(S, S, 8, 8)
    for cls, thr in ((False, 0.0), (True, 0.0), (False, 40.0)):
        outs = {}
        for name, eng, fl in (("valu", F.ENGINE_VALU, 0), ("direct", F.ENGINE_MFMA, F.FLAG_DIRECT_FORM),
                              ("fourier", F.ENGINE_MFMA, 0)):
            with F.Engine(0, 8, cls, thr, -1.0, eng, flags=fl) as e:
                e.set_frame(p)
                e.set_domains(doms)
                outs[name], st = e.search(rngs)
            if name == "fourier":
                assert st["search_form"] == F.FORM_FOURIER
        for name in ("direct", "fourier"):
            assert outs[name].tobytes() == outs["valu"].tobytes(), f"{kind} cls={cls} thr={thr}: {name}"
        if kind in ("binary", "noise") and thr == 0.0:  # exact copies (blocks8) are hits: transform 0 first
            assert (outs["fourier"]["transform"] >= 4).any(), "the flipped copies win somewhere"


def test_fourier_direct_and_valu_agree_on_stress_frame():
    """n = 8, T = 4 on a uniform-noise 1024² frame: C4-Fourier MFMA, direct MFMA and VALU
    engines give identical records."""
    from fractencode_amd.synth import uniform_noise
    p = uniform_noise(1024, 1024, 43)
    outs = []
    for eng, fl in ((F.ENGINE_VALU, 0), (F.ENGINE_MFMA, F.FLAG_DIRECT_FORM), (F.ENGINE_MFMA, 0), (F.ENGINE_SEA, 0)):
        with F.Engine(0, 4, False, 0.0, -1.0, eng, flags=fl) as e:
            e.set_frame(p)
            e.set_domains(F.create_uniform_grid(1024, 1024, 16, 8))
            out, st = e.search(F.create_uniform_grid(1024, 1024, 8, 8))
            assert st["engine"] == eng
            outs.append(out)
    assert outs[0].tobytes() == outs[1].tobytes()
    assert outs[0].tobytes() == outs[2].tobytes()
    assert outs[0].tobytes() == outs[3].tobytes()


def test_sea_skips_most_candidates_with_identical_records():
    """Lenna Y, n = 8, T = 8: the SEA engine evaluates a small fraction of the candidates the
    exhaustive engines do, and returns the same records."""
    p = plane("lenna_y")
    doms = F.create_uniform_grid(512, 512, 16, 8)
    rngs = F.create_uniform_grid(512, 512, 8, 8)
    res = {}
    for eng in (F.ENGINE_MFMA, F.ENGINE_SEA):
        with F.Engine(0, 8, False, 0.0, -1.0, eng) as e:
            e.set_frame(p)
            e.set_domains(doms)
            res[eng] = e.search(rngs)
    (a, sa), (b, sb) = res[F.ENGINE_MFMA], res[F.ENGINE_SEA]
    assert a.tobytes() == b.tobytes()
    assert sa["evaluated_mappings"] == len(doms) * len(rngs)
    assert 0 < sb["evaluated_mappings"] < 0.2 * sa["evaluated_mappings"]
    assert sb["search_form"] == F.FORM_SEA


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("n", [4, 8])
def test_unaligned_origins(oracle, engine, n):
    """Ranges and domains at origins off the 4- and 8-pixel grid (a grid offset by (3, 5) with
    odd strides): every engine's loaders realign the rows and match the oracle."""
    rng = np.random.default_rng(11 + n)
    W, H = 96, 80
    p = rng.integers(0, 256, (H, W), dtype=np.uint8)

    def grid(size, step, x0, y0):
        out = [(x, y, size, size, 0) for y in range(y0, H - size + 1, step) for x in range(x0, W - size + 1, step)]
        return np.array(out, dtype=F.GRID_ITEM)

    doms = grid(2 * n, n + 1, 3, 5)
    rngs = grid(n, n + 3, 1, 2)
    with F.Engine(0, 4, False, 0.0, -1.0, engine) as e:
        e.set_frame(p)
        e.set_domains(doms)
        out, _ = e.search(rngs)
    want, _, _ = oracle.estimate(p, doms, rngs)
    assert_same(out, {k: want[k] for k in FIELDS}, f"unaligned n={n}")


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("cls", [False, True])
@pytest.mark.parametrize("T,thr", [(4, 0.0), (8, 0.0), (4, 2.0), (8, 2.0)])
def test_new_frame_same_geometry(engine, cls, T, thr):
    """A second frame of the same geometry into a prepared context (the video case: the
    classifier-off path keeps the prepared structures, the classifier-on path re-prepares)
    gives the records a fresh context gives for that frame. Each run resets its winners
    (on the Fourier path inside dft_prep, not by a memset), with and without flipped copies
    and hit thresholds."""
    rng = np.random.default_rng(21)
    a = rng.integers(0, 256, (128, 128), dtype=np.uint8)
    b = np.ascontiguousarray(np.rot90(a)) // 2 + rng.integers(0, 100, (128, 128), dtype=np.uint8)
    doms = F.create_uniform_grid(128, 128, 16, 8)
    rngs = F.create_uniform_grid(128, 128, 8, 8)
    with F.Engine(0, T, cls, thr, -1.0, engine) as e:
        e.set_frame(a)
        e.set_domains(doms)
        e.set_ranges(rngs)
        e.run()
        first, _ = e.fetch()
        e.set_frame(b)
        e.run()
        second, _ = e.fetch()
    with F.Engine(0, T, cls, thr, -1.0, engine) as e:
        e.set_frame(b)
        e.set_domains(doms)
        want, _ = e.search(rngs)
    assert second.tobytes() == want.tobytes()
    assert first.tobytes() != second.tobytes()


# the sampled form (fracenc_gen.hip): domain sizes other than 2n, and range sizes outside {2,4,8,16}
GEN_CASES = [
    # W, H, src, tgt, T, classifier, thr, smax, kind
    (64, 64, 16, 4, 4, False, 0.0, -1.0, "noise"),    # the CLI default (match_16to4)
    (64, 64, 16, 4, 8, True, 0.0, -1.0, "uniform"),
    (64, 64, 16, 4, 4, False, 3.0, -1.0, "flat"),     # threshold hits: first (domain, t)
    (96, 64, 32, 8, 4, False, 0.0, 0.8, "noise"),
    (48, 48, 24, 8, 8, True, 0.0, -1.0, "flat"),      # ratio 3, ties
    (48, 48, 12, 8, 4, False, 0.0, -1.0, "noise"),    # metric ratio 1, fit at (x·12)/8
    (60, 60, 10, 4, 4, False, 0.0, -1.0, "uniform"),  # ratio 2 in the metric, 2.5 in the fit
    (48, 48, 12, 6, 4, True, 0.0, -1.0, "noise"),     # n = 6: gen_search
    (48, 48, 9, 3, 8, False, 2.0, -1.0, "flat"),      # n = 3, threshold
    (64, 64, 64, 16, 4, False, 0.0, -1.0, "noise"),   # n = 16, ratio 4
    (64, 64, 64, 32, 4, False, 0.0, -1.0, "uniform"), # n = 32 (fp32 fallback regime)
    (40, 40, 20, 5, 4, False, 1e9, -1.0, "noise"),    # every candidate hits: all-fallback mode
]


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("case", range(len(GEN_CASES)))
def test_sampled_form_matches_oracle_random(oracle, case, engine):
    W, H, src, tgt, T, cls, thr, smax, kind = GEN_CASES[case]
    rng = np.random.default_rng(3000 + case)
    p = _random_plane(rng, W, H, kind)
    meta = dict(src=src, tgt=tgt, T=T, cls=cls, thr=thr, smax=smax)
    out, st = run_engine(p, meta, engine)
    doms = oracle.uniform_grid(W, H, src, src // 2)
    rngs = oracle.uniform_grid(W, H, tgt, tgt)
    if cls:
        doms = oracle.classify(p, doms)
        rngs = oracle.classify(p, rngs)
    want, rej, _ = oracle.estimate(p, doms, rngs, T=T, thr=thr, smax=smax, use_classifier=cls)
    assert_same(out, {k: want[k] for k in FIELDS}, f"case {GEN_CASES[case]}")
    assert st["rejected_mappings"] == rej
    if tgt not in (2, 4, 8, 16):
        assert st["search_form"] == F.FORM_SAMPLED


@pytest.mark.parametrize("engine", ENGINES)
def test_default_cli_geometry_4096(engine):
    """The reference's default geometry (16→4, encode_parameters.h:6-7) on the 4096² C3 frame —
    1,048,576 ranges × 261,121 domains × 4 transforms: every reported distance is the exact error of
    the reported (domain, transform) sampled as match_16to4 does (numpy), and a strided sample of
    ranges matches the oracle."""
    p = plane("s1_4096")
    doms = F.create_uniform_grid(4096, 4096, 16, 8)
    rngs = F.create_uniform_grid(4096, 4096, 4, 4)
    with F.Engine(0, 4, False, 0.0, -1.0, engine, timing=True) as e:
        e.set_frame(p)
        e.set_domains(doms)
        out, st = e.search(rngs)
    # exact error of each winner: 2×2 sums at the transformed (4x, 4y) corners (transform.h:96-109)
    lut = [(1, 0, 0, 0, 0, 1, 0, 0), (0, 1, 0, 0, -1, 0, 1, 0), (-1, 0, 1, 0, 0, -1, 0, 1), (0, -1, 0, 1, 1, 0, 0, 0)]
    A = np.array(lut, np.int64)[out["transform"].astype(np.int64)]
    yy, xx = np.divmod(np.arange(16), 4)
    lx, ly = 4 * xx[None, :], 4 * yy[None, :]
    S = 16
    px = out["dx"].astype(np.int64)[:, None] + A[:, 0:1] * lx + A[:, 1:2] * ly + (A[:, 2:3] + A[:, 3:4]) * (S - 1)
    py = out["dy"].astype(np.int64)[:, None] + A[:, 4:5] * lx + A[:, 5:6] * ly + (A[:, 6:7] + A[:, 7:8]) * (S - 1)
    pi = p.astype(np.int64)
    D = (pi[py, px] + pi[py + A[:, 4:5], px + A[:, 0:1]] + pi[py + A[:, 5:6], px + A[:, 1:2]]
         + pi[py + A[:, 4:5] + A[:, 5:6], px + A[:, 0:1] + A[:, 1:2]])
    r = p[out["y"].astype(np.int64)[:, None] + yy[None, :], out["x"].astype(np.int64)[:, None] + xx[None, :]]
    s16 = ((4 * r.astype(np.int64) - D) ** 2).sum(1)
    np.testing.assert_array_equal(out["distance"], (s16 / 16.0) / 256.0)
    assert st["fallback_ranges"] == 0 and (out["sw"] == 16).all()
    from oracle import oracle as O
    sel = np.arange(0, len(rngs), 8191)
    want, _, _ = O.estimate(p, O.uniform_grid(4096, 4096, 16, 8), O.uniform_grid(4096, 4096, 4, 4)[sel], threads=16)
    assert_same(out[sel], {k: want[k] for k in FIELDS}, "16to4 4096 sample")


def test_encode_defaults_are_the_reference_cli_defaults():
    # fractencode_amd.encode() with no options = the CLI's encode_parameters_t (16 -> 4, offset 8,
    # classifier on, threshold 0, sMax -1): the reference's own run of that configuration
    rec, meta = golden("lenna_16to4_cls")
    out, st = F.encode(plane(meta["plane"]))
    assert_same(out, rec, "encode() defaults")
    assert st["rejected_mappings"] == meta["rejected"]


@pytest.mark.parametrize("n,T", [(8, 4), (4, 4), (8, 8), (16, 4)])
def test_every_product_form_gives_the_same_records(monkeypatch, n, T):
    # the product library holds the shipped forms only: the default (Fourier for ratio-2 n = 8) and
    # FRAC_FLAG_DIRECT_FORM must give the records of the exhaustive VALU engine, and an A/B knob of
    # the tuning build fails the run instead of selecting anything
    from fractencode_amd.synth import value_noise
    S = 256
    p = value_noise(S, S, 77)
    doms, rngs = F.create_uniform_grid(S, S, 2 * n, n), F.create_uniform_grid(S, S, n, n)
    with F.Engine(0, T, False, 0.0, -1.0, F.ENGINE_VALU) as e:
        e.set_frame(p)
        e.set_domains(doms)
        want, _ = e.search(rngs)
    for fl in (0, F.FLAG_DIRECT_FORM):
        with F.Engine(0, T, False, 0.0, -1.0, F.ENGINE_MFMA, flags=fl) as e:
            e.set_frame(p)
            e.set_domains(doms)
            out, _ = e.search(rngs)
        assert out.tobytes() == want.tobytes(), f"flags {fl} (n={n}, T={T})"
    for knob, val in (("FRAC_MFMA_VARIANT", "21"), ("FRAC_MFMA_DFT", "0"), ("FRAC_DFT_WGS", "2048")):
        monkeypatch.setenv(knob, val)
        with F.Engine(0, T, False, 0.0, -1.0, F.ENGINE_MFMA) as e:
            e.set_frame(p)
            e.set_domains(doms)
            with pytest.raises(F.FracError, match="FRAC_TUNING"):
                e.search(rngs)
        monkeypatch.delenv(knob)


# --- rectangular items (Size32u grids) and grid validation ---------------------------------------

def test_rectangular_domains_sampling_outside_the_plane_are_refused():
    # a Rotate_90 of a 16×8 domain reads 16 rows below its origin (image/transform.h:96-109): over the
    # whole plane's domain grid the bottom row's samples leave the image, where the reference reads
    # out of bounds — the engine refuses the search instead (the goldens cut the grid, make_golden.py)
    p = plane("crop64")
    with F.Engine(0, 4, False, 0.0, -1.0) as e:
        e.set_frame(p)
        e.set_domains(F.create_uniform_grid(64, 64, (16, 8), (8, 4)))
        with pytest.raises(F.FracError, match="samples outside the source plane"):
            e.search(F.create_uniform_grid(64, 64, (8, 4), (8, 4)))
        # the cut grid (rect64_8x4_16x8's) searches
        e.set_domains(F.create_uniform_grid(64, 56, (16, 8), (8, 4)))
        out, _ = e.search(F.create_uniform_grid(64, 64, (8, 4), (8, 4)))
        assert (out["sw"] == 16).all() and (out["sh"] == 8).all()


def test_domain_grid_is_validated_when_set():
    # frac_set_domains checks what it can (one item size, inside the plane, categories) so that the
    # reference-side engine fails in its constructor (EncodingEngine2.cpp:27-29), not on a worker
    p = plane("crop64")
    with F.Engine(0) as e:
        e.set_frame(p)
        mixed = np.concatenate([F.create_uniform_grid(64, 64, 16, 8), F.create_uniform_grid(64, 64, 8, 8)])
        with pytest.raises(F.FracError, match="one size"):
            e.set_domains(mixed)
        outside = F.create_uniform_grid(64, 64, 16, 8)
        outside["x"][-1] = 60
        with pytest.raises(F.FracError, match="outside the source plane"):
            e.set_domains(outside)
        bad = F.create_uniform_grid(64, 64, 16, 8)
        bad["category"][0] = 9
        with pytest.raises(F.FracError, match="category"):
            e.set_domains(bad)
        e.set_domains(F.create_uniform_grid(64, 64, 16, 8))  # a valid grid is accepted afterwards


@pytest.mark.parametrize("engine", ENGINES)
def test_rectangular_ranges_random_planes_match_oracle(oracle, engine):
    # rectangles beyond the reference-pinned goldens (rect*): random planes, T = 8, classifier,
    # thresholds; the oracle (pinned by those goldens) is the checker
    rng = np.random.default_rng(77)
    for (W, H, rs, ds, doff, T, cls, thr) in [(64, 64, (8, 4), (16, 8), (8, 4), 8, False, 0.0),
                                              (64, 64, (4, 8), (8, 16), (4, 8), 4, True, 0.0),
                                              (48, 48, (6, 4), (12, 12), (6, 6), 4, False, 3.0),
                                              (64, 64, (16, 8), (32, 16), (16, 8), 4, False, 0.0)]:
        p = rng.integers(0, 256, (H, W), dtype=np.uint8)
        M = max(ds)
        dW, dH = W - (M - ds[0]), H - (M - ds[1])
        doms = F.create_uniform_grid(dW, dH, ds, doff)
        rngs = F.create_uniform_grid(W, H, rs, rs)
        if cls:
            doms, rngs = F.preclassify(p, doms), F.preclassify(p, rngs)
        with F.Engine(0, T, cls, thr, -1.0, engine) as e:
            e.set_frame(p)
            e.set_domains(doms)
            out, st = e.search(rngs)
        want, rej, _ = oracle.estimate(p, doms, rngs, T=T, thr=thr, use_classifier=cls)
        assert_same(out, {k: want[k] for k in FIELDS}, f"rect {rs} {ds} T={T}")
        assert st["rejected_mappings"] == rej


@pytest.mark.parametrize("n,T", [(8, 4), (8, 8), (16, 4), (16, 8)])
def test_fp32_regime_through_the_fallback_grid(n, T):
    """Ranges whose best exact error is at least 2^24 (S16) take the reference's fp32 arithmetic
    (image/metrics.h:37-50).  The MFMA engine's fused resolvers (resolve_dft / resolve_mfma) list them and
    fallback_grid settles them before the records are read (frac_fetch here); the VALU engine runs
    fallback_grid at the end of every run.  Isolated bright n×n blocks 4n apart on a black frame: every
    domain is mostly dark (at most a quarter of its cells bright: S16 ≥ 48·1020² at n = 8), so each bright range
    is in the fp32 regime.  Records, fallback counts and reject counts agree, and the fallback count is the
    bright blocks'.  (n ≤ 4 never reaches the regime: 16 cells · 1020² < 2^24.)"""
    S = 32 * n
    p = np.zeros((S, S), np.uint8)
    nb = 0
    for y in range(n, S - n, 4 * n):
        for x in range(n, S - n, 4 * n):
            p[y:y + n, x:x + n] = 255
            nb += 1
    doms, rngs = F.create_uniform_grid(S, S, 2 * n, n), F.create_uniform_grid(S, S, n, n)
    outs = {}
    for eng in (F.ENGINE_VALU, F.ENGINE_MFMA):
        with F.Engine(0, T, False, 0.0, -1.0, eng) as e:
            e.set_frame(p)
            e.set_domains(doms)
            outs[eng] = e.search(rngs)
    (a, sa), (b, sb) = outs[F.ENGINE_VALU], outs[F.ENGINE_MFMA]
    assert sb["engine"] == F.ENGINE_MFMA
    assert sa["fallback_ranges"] == sb["fallback_ranges"] == nb, (sa["fallback_ranges"], sb["fallback_ranges"], nb)
    assert a.tobytes() == b.tobytes()
    assert sa["rejected_mappings"] == sb["rejected_mappings"]


def _white_ranges_frame(S, k, seed=17):
    """tools/fallback_probe.py's frame: S1 value noise scaled into [0, 60] with k white 8×8 ranges, each alone in a
    black 24×24 patch — the white ranges' best error is ≥ 2^24 (fp32 regime), the rest are ordinary."""
    from fractencode_amd.synth import value_noise
    p = (value_noise(S, S, 1234).astype(np.float64) * (60.0 / 255.0)).astype(np.uint8)
    rng = np.random.default_rng(seed)
    where = []
    for c in rng.choice((S // 24) ** 2, size=k, replace=False):
        y0, x0 = (c // (S // 24)) * 24, (c % (S // 24)) * 24
        p[y0:y0 + 24, x0:x0 + 24] = 0
        p[y0 + 8:y0 + 16, x0 + 8:x0 + 16] = 255
        where.append((x0 + 8, y0 + 8))
    return p, where


@pytest.mark.parametrize("T,cls", [(4, False), (8, False), (4, True)])
def test_fp32_regime_at_scale_every_consumer(oracle, T, cls):
    """A 1024² frame with 6 fp32-regime ranges among 16,384: every consumer of the run's records — the device
    tuples (frac_copy_tuples_device → fetch_tuples), frac_fetch, the device decode's input — sees the
    fp32 winners fallback_grid writes, and those equal the oracle's (the reference's fp32 loop restated)."""
    S = 1024
    p, where = _white_ranges_frame(S, 6)
    doms, rngs = F.create_uniform_grid(S, S, 16, 8), F.create_uniform_grid(S, S, 8, 8)
    if cls:
        doms, rngs = F.preclassify(p, doms), F.preclassify(p, rngs)
    with F.Engine(0, T, cls, 0.0, -1.0, F.ENGINE_MFMA) as e:
        e.set_frame(p)
        e.set_domains(doms)
        e.set_ranges(rngs)
        e.run()
        tup = e.fetch_tuples()  # an asynchronous consumer first (the pack runs after the settle)
        out, st = e.fetch()
    idx = np.array([(y // 8) * (S // 8) + x // 8 for x, y in where])
    if not cls:  # with the classifier a white range may meet no domain of its category (the default record)
        assert st["fallback_ranges"] >= len(where)
    want, _, _ = oracle.estimate(p, doms.astype(oracle.ITEM_DTYPE), rngs[idx].astype(oracle.ITEM_DTYPE), T=T,
                                 use_classifier=cls, threads=8)
    for a, b in (("dx", "dx"), ("dy", "dy"), ("transform", "t"), ("distance", "dist"), ("contrast", "s"),
                 ("brightness", "o")):
        np.testing.assert_array_equal(out[a][idx], want[b], err_msg=a)
    assert (out["distance"][idx] * 16 * 256 >= (1 << 24)).all()  # they are in the fp32 regime
    for k in ("transform", "contrast", "brightness", "distance"):
        np.testing.assert_array_equal(tup[k], out[k], err_msg=k)
