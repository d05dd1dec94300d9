"""CPU checks of the C-ABI boundary (no compute calls on a device):
the library loads, exports every symbol include/fracenc.h declares, the record
layouts match the reference's structs, and the host helpers agree with the oracle.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import fractencode_amd as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fracenc.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(frac_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = F.lib()
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.frac_abi_version() == 9


def test_library_carries_the_source_id():
    # build() compiles fractencode_amd.source_id() into the library (frac_build_id); a stale or
    # foreign binary shows up here and in bench.py's line
    info = F.build_info()
    assert info["build_id"] == F.source_id(), info
    assert info["matches_sources"] and not info["tuning"]


def test_record_layouts_match_reference_structs(tmp_path):
    # frac_* mirror Frac::transform_score_t / item_match_t / encode_item_t and
    # Frac2::UniformGridItem (encode/datatypes.h:8-26, image/partition2.hpp:93-99)
    src = tmp_path / "layout.c"
    src.write_text(
        '#include "fracenc.h"\n#include <stddef.h>\n'
        "_Static_assert(sizeof(frac_grid_item) == 20, \"item\");\n"
        "_Static_assert(sizeof(frac_score) == 32, \"score\");\n"
        "_Static_assert(sizeof(frac_match) == 48, \"match\");\n"
        "_Static_assert(sizeof(frac_encode_item) == 64, \"encode\");\n"
        "_Static_assert(offsetof(frac_encode_item, match) == 16, \"match off\");\n"
        "_Static_assert(offsetof(frac_match, x) == 32, \"x off\");\n"
        "_Static_assert(offsetof(frac_score, transform) == 24, \"t off\");\n"
        f"_Static_assert(sizeof(frac_stats) == {C.sizeof(F.FracStats)}, \"stats (ctypes mirror)\");\n"
        f"_Static_assert(offsetof(frac_stats, matrix_flops) == {F.FracStats.matrix_flops.offset}, \"flops off\");\n"
        f"_Static_assert(offsetof(frac_stats, evaluated_mappings) == {F.FracStats.evaluated_mappings.offset}, "
        "\"evaluated off\");\n"
        "int main(void) { return 0; }\n")
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-c", str(src), "-o",
                           str(tmp_path / "layout.o")])
    assert F.ENCODE_ITEM.itemsize == 64 and F.GRID_ITEM.itemsize == 20
    assert F.ENCODE_ITEM.fields["distance"][1] == 16 and F.ENCODE_ITEM.fields["dx"][1] == 48


@pytest.mark.parametrize("W,H,size,off", [(64, 64, 16, 8), (512, 512, 8, 8), (96, 64, 8, 4), (48, 80, 4, 2),
                                          (64, 64, 64, 32)])
def test_uniform_grid_matches_oracle(oracle, W, H, size, off):
    g = F.create_uniform_grid(W, H, size, off)
    o = oracle.uniform_grid(W, H, size, off)
    assert len(g) == len(o)
    for k in ("x", "y", "w", "h", "category"):
        np.testing.assert_array_equal(g[k], o[k])


@pytest.mark.parametrize("W,H,size,off", [(512, 512, (4, 4), (4, 2)), (64, 48, (16, 8), (8, 4)), (96, 64, (8, 4), (4, 2)),
                                          (64, 64, (8, 16), (2, 4)), (48, 40, (12, 8), (6, 8))])
def test_anisotropic_uniform_grid(oracle, W, H, size, off):
    # createUniformGrid's Size32u item size and offset (image/partition2.hpp:110-113): the engine's grid
    # equals the oracle's and — when the reference build is present — the reference's own
    g = F.create_uniform_grid(W, H, size, off)
    o = oracle.uniform_grid(W, H, size, off)
    assert len(g) == len(o) > 0
    for k in ("x", "y", "w", "h", "category"):
        np.testing.assert_array_equal(g[k], o[k])
    r = oracle.ref_uniform_grid(W, H, size, off)
    if r is not None:
        for k in ("x", "y", "w", "h", "category"):
            np.testing.assert_array_equal(g[k], r[k])


def test_preclassify_matches_oracle(oracle):
    from golden_util import plane
    y = plane("lenna_y")
    for size, off in [(8, 8), (16, 8), (4, 4), (32, 16)]:
        items = F.create_uniform_grid(512, 512, size, off)
        a = F.preclassify(y, items)["category"]
        b = oracle.classify(y, oracle.uniform_grid(512, 512, size, off))["category"]
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_transform_tables_are_the_reference_sampler(n):
    # the kernel's permutation must equal SamplerBilinear's 2×2 block under each
    # transform (image/sampler.h:21-38, image/transform.h:96-109) at ratio 2
    lut = [(1, 0, 0, 0, 0, 1, 0, 0), (0, 1, 0, 0, -1, 0, 1, 0), (-1, 0, 1, 0, 0, -1, 0, 1), (0, -1, 0, 1, 1, 0, 0, 0),
           (1, 0, 0, 0, 0, -1, 0, 1), (0, 1, 0, 0, 1, 0, 0, 0), (-1, 0, 1, 0, 0, 1, 0, 0), (0, -1, 0, 1, -1, 0, 1, 0)]
    S = 2 * n
    for t in range(8):
        a = lut[t]
        seen = set()
        for pix in range(n * n):
            x, y = pix % n, pix // n
            lx, ly = 2 * x, 2 * y
            px = a[0] * lx + a[1] * ly + a[2] * (S - 1) + a[3] * (S - 1)
            py = a[4] * lx + a[5] * ly + a[6] * (S - 1) + a[7] * (S - 1)
            pts = [(px, py), (px + a[0], py + a[4]), (px + a[1], py + a[5]), (px + a[0] + a[1], py + a[4] + a[5])]
            x0 = min(p[0] for p in pts)
            y0 = min(p[1] for p in pts)
            assert x0 % 2 == 0 and y0 % 2 == 0
            q = F.transform_index(n, t, pix)
            assert q == (y0 // 2) * n + (x0 // 2), (t, pix)
            seen.add(q)
        assert len(seen) == n * n


def test_hit_limit():
    # dist = (S16/16)/(4n²) <= thr  (transformmatcher.h:32-34)
    assert F.hit_limit(0.0, 8) == 0
    assert F.hit_limit(-0.5, 8) == -1
    assert F.hit_limit(float("nan"), 8) == -1
    for thr in (0.25, 1.0, 10.0, 123.456):
        for n in (2, 4, 8, 16):
            H = F.hit_limit(thr, n)
            assert (H / 16.0) / (4 * n * n) <= thr < ((H + 1) / 16.0) / (4 * n * n)


def test_engine_without_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    with pytest.raises(F.FracError):
        F.Engine()


def _kernel_instances(pattern):
    """Demangled host-side launch stubs of one kernel template in the product library."""
    out = subprocess.run(["nm", "-C", F.LIB_PATH], capture_output=True, text=True, check=True).stdout
    return [m.group(1) for m in re.finditer(pattern, out)]


def test_product_library_has_no_ablation_kernels():
    # the "tuning only, wrong results" ablations exist only in a -DFRAC_TUNING build; unknown or
    # ablation FRAC_MFMA_VARIANT values fail the run (fracenc_api.hip mfma_variant)
    dft = _kernel_instances(r"fracenc::search_dft<(?:true|false), (\d+)")
    mfma = _kernel_instances(r"fracenc::search_mfma<\d+, \d+, (?:true|false), (\d+)>")
    assert dft and mfma
    assert all(int(v) & (8 | 16 | 32 | 64 | 256 | 512) == 0 for v in dft), sorted(set(dft))
    assert all(int(v) & (8 | 16) == 0 for v in mfma), sorted(set(mfma))
    # and no A/B variant either (round 4): the Fourier search as shipped (variant 35 =
    # 1|kDftChain|kDft6|kDftFast6|kDftUnroll|kDftBufDma) and the SEA tiled form's exact six-MFMA
    # tile (1|kDftChain|kDft6); the direct form's shipped schedule (130)
    assert set(map(int, dft)) == {123905, 9217}, sorted(set(dft))
    assert set(map(int, mfma)) == {130, 386}, sorted(set(mfma))  # 386: the float-C epilogue, n <= 4
    assert not _kernel_instances(r"fracenc::(search_dft2)<"), "the two-block A/B form is tuning-only"


def test_uniform_grid_closed_form_count_and_cap(oracle):
    """frac_uniform_grid2 counts in closed form and fills row by row (round 6: the loop's count cost 0.2 ms per
    quadtree call): count, items and a short `cap` (the first cap items, the full count returned) equal
    createUniformGrid's loop (the oracle, and the reference's own build when present) over random geometries,
    edge cases included (item = plane, offset past the edge, degenerate sizes)."""
    import ctypes as C

    rng = np.random.default_rng(5)
    cases = [(64, 64, (64, 64), (1, 1)), (64, 64, (8, 8), (100, 100)), (7, 5, (8, 8), (1, 1)), (9, 9, (1, 1), (1, 1)),
             (64, 64, (0, 8), (8, 8)), (64, 64, (8, 8), (0, 8))]
    for _ in range(40):
        W, H = (int(v) for v in rng.integers(1, 200, 2))
        cases.append((W, H, tuple(int(v) for v in rng.integers(1, 40, 2)), tuple(int(v) for v in rng.integers(1, 40, 2))))
    lib = F.lib()
    for W, H, (sw, sh), (ox, oy) in cases:
        n = lib.frac_uniform_grid2(W, H, sw, sh, ox, oy, None, 0)
        if 0 in (sw, sh, ox, oy) or sw > W or sh > H:  # no grid (the loop never ends / its item leaves the plane)
            assert n == 0, (W, H, sw, sh, ox, oy)
            continue
        want = oracle.lib().or_uniform_grid2(W, H, sw, sh, ox, oy, None, 0)
        assert n == want, (W, H, sw, sh, ox, oy)
        if not n:
            continue
        g = F.create_uniform_grid(W, H, (sw, sh), (ox, oy))
        o = oracle.uniform_grid(W, H, (sw, sh), (ox, oy))
        assert g.tobytes() == o.tobytes(), (W, H, sw, sh, ox, oy)
        cap = max(1, n // 3)
        short = np.zeros(cap + 1, dtype=F.GRID_ITEM)
        assert lib.frac_uniform_grid2(W, H, sw, sh, ox, oy, short.ctypes.data_as(C.c_void_p), cap) == n
        assert short[:cap].tobytes() == g[:cap].tobytes() and short[cap].tobytes() == bytes(F.GRID_ITEM.itemsize)
