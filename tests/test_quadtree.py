"""Quadtree partition (include/fracenc.h frac_encode_quadtree).  The reference parses
--quadtree and never builds one (main.cpp:75-76): the rule is this library's, so parity is
against the oracle's restatement of the same rule (oracle.quadtree), whose every level is the
reference-pinned search; the level searches themselves are pinned by lenna_n4 / lenna_n16.
CPU: properties of the oracle partition.  GPU: the engine equals the oracle item for item,
and the mixed-size decode equals the oracle decoder."""
import numpy as np
import pytest

import fractencode_amd as F
from golden_util import plane


def _coverage(recs, sizes, W, H, max_size):
    cov = np.zeros((H, W), np.int32)
    for r, s in zip(recs, sizes):
        cov[r["y"]:r["y"] + s, r["x"]:r["x"] + s] += 1
    return cov


@pytest.mark.parametrize("split", [0.0, 2.0, 1e9])
def test_oracle_quadtree_partition_properties(oracle, split):
    p = plane("crop64")
    recs, sizes = oracle.quadtree(p, 16, 4, split)
    cov = _coverage(recs, sizes, 64, 64, 16)
    assert (cov == 1).all()  # the leaves tile the frame exactly once
    if split == 1e9:
        assert (sizes == 16).all() and len(recs) == 16
    if split == 0.0:  # only exact matches stop the split
        assert (recs["dist"][sizes > 4] == 0.0).all()
    assert set(np.unique(sizes)) <= {4, 8, 16}


def _as_oracle(items):
    from oracle.oracle import RESULT_DTYPE

    out = np.zeros(len(items), dtype=RESULT_DTYPE)
    for a, b in (("x", "x"), ("y", "y"), ("dx", "dx"), ("dy", "dy"), ("sw", "dw"), ("sh", "dh"), ("transform", "t"),
                 ("distance", "dist"), ("contrast", "s"), ("brightness", "o")):
        out[b] = items[a]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("cls,split,T", [(False, 1.0, 4), (False, 8.0, 4), (True, 1.0, 4), (True, 8.0, 4),
                                         (True, 8.0, 8), (False, 1.0, 8)])
def test_gpu_quadtree_matches_oracle(oracle, cls, split, T):
    # T = 8: the n = 8 level runs the Fourier form with the flipped range copies
    p = plane("lenna_y")
    with F.Engine(0, T, cls) as e:
        e.set_frame(p)
        items, st = e.encode_quadtree(16, 4, split)
        want, sizes = oracle.quadtree(p, 16, 4, split, T=T, use_classifier=cls)
        got = _as_oracle(items)
        for k in want.dtype.names:
            if k != "pad":
                np.testing.assert_array_equal(got[k], want[k], err_msg=k)
        np.testing.assert_array_equal(items["w"], sizes)
        assert (_coverage(want, sizes, 512, 512, 16) == 1).all()
        dec, it, rms = e.decode(items, 512, 512)
    wdec, wit, wrms = oracle.decode_sized(want, sizes, 512, 512)
    assert (it, rms) == (wit, wrms)
    np.testing.assert_array_equal(dec, wdec)
    from fractencode_amd.codec import psnr
    assert psnr(p, dec) > 25.0


@pytest.mark.gpu
@pytest.mark.parametrize("cls,thr", [(True, 0.0), (True, 2.0), (False, 2.0)])
def test_gpu_quadtree_stats_are_the_levels_stats(cls, thr):
    # the quadtree's summed statistics (accumulated on the device level by level) equal the sum of
    # the same levels searched one by one; the caller's `out` buffer receives the same items
    p = plane("lenna_y")
    split = 8.0
    with F.Engine(0, 4, cls, thr) as e:
        e.set_frame(p)
        buf = np.empty((512 // 4) ** 2, dtype=F.ENCODE_ITEM)
        items, st = e.encode_quadtree(16, 4, split, out=buf)
        assert np.shares_memory(items, buf)
        items2, st2 = e.encode_quadtree(16, 4, split)
        np.testing.assert_array_equal(items, items2)
        # (round 4: the device-planned levels count total / evaluated pairs and the search's MFMA flops
        # on the device, from their own layout: they must equal the host-planned searches' counts)
        keys = ("rejected_mappings", "total_mappings", "hit_ranges", "fallback_ranges", "empty_ranges",
                "evaluated_mappings", "matrix_flops")
        want = dict.fromkeys(keys, 0)
        ranges = F.create_uniform_grid(512, 512, 16, 16)
        leaves = []
        for n in (16, 8, 4):
            e.set_domains(F.create_uniform_grid(512, 512, 2 * n, n))
            out, s = e.search(ranges)
            for k in keys:
                want[k] += s[k]
            if n == 4:
                leaves.append(out)
                break
            sp = out["distance"] > split
            leaves.append(out[~sp])
            par = ranges[sp]
            h = n // 2
            nxt = np.zeros(4 * len(par), dtype=F.GRID_ITEM)
            for q, (ox, oy) in enumerate(((0, 0), (h, 0), (0, h), (h, h))):
                nxt["x"][q::4], nxt["y"][q::4] = par["x"] + ox, par["y"] + oy
            nxt["w"], nxt["h"], nxt["category"] = h, h, -1
            ranges = nxt
        assert st["hit_ranges"] > 0 or thr == 0.0
        for k in keys:
            assert st[k] == want[k], k
            assert st2[k] == want[k], k
        np.testing.assert_array_equal(items, np.concatenate(leaves))


@pytest.mark.gpu
def test_gpu_quadtree_restores_the_list_state():
    # the quadtree swaps its level grids in and out: the caller's domain list (set or not) comes
    # back, and the consumed range list is unset, so a later run without set_ranges is a state error
    p = plane("crop64")
    with F.Engine(0, 4) as e:
        e.set_frame(p)
        e.encode_quadtree(16, 4, 2.0)
        with pytest.raises(RuntimeError):
            e.run()  # no domains were ever set
        doms = F.create_uniform_grid(64, 64, 8, 4)
        e.set_domains(doms)
        e.encode_quadtree(16, 4, 2.0)
        with pytest.raises(RuntimeError):
            e.run()  # the ranges were consumed
        rngs = F.create_uniform_grid(64, 64, 4, 4)
        out, _ = e.search(rngs)  # the caller's own domain list is back
        with F.Engine(0, 4) as f:
            f.set_frame(p)
            f.set_domains(doms)
            want, _ = f.search(rngs)
        np.testing.assert_array_equal(out, want)


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", [(16, 4), (16, 2), (8, 2), (16, 16), (4, 2)])
@pytest.mark.parametrize("cls,T,thr,split", [(True, 4, 0.0, 8.0), (False, 8, 2.0, 1.0), (True, 8, 0.0, 1e9),
                                             (True, 4, 0.0, 0.0), (False, 4, 0.0, 20.0)])
def test_gpu_quadtree_device_planned_equals_host_planned(sizes, cls, T, thr, split):
    """The MFMA engine's quadtree levels are laid out on the device (qt_plan: bucket bounds, work lists,
    CSR map and every count stay in HBM; worst-case grids; one round trip per frame).  The VALU engine
    keeps the host-planned levels (bucket counts and split counts read back per level).  Both must give
    the same leaves and the same summed counters, for every level-size range, with and without the
    classifier, T = 4 / 8 (the n = 8 level's Fourier form with flipped copies), a hit threshold, a
    split that empties the later levels (1e9) and one that splits every inexact range (0)."""
    p = plane("lenna_y")
    res = {}
    for eng in (F.ENGINE_VALU, F.ENGINE_AUTO):
        with F.Engine(0, T, cls, thr, -1.0, eng, timing=True) as e:
            e.set_frame(p)
            res[eng] = e.encode_quadtree(*sizes, split)
    (a, sa), (b, sb) = res[F.ENGINE_VALU], res[F.ENGINE_AUTO]
    np.testing.assert_array_equal(a, b)
    for k in ("rejected_mappings", "total_mappings", "hit_ranges", "fallback_ranges", "empty_ranges",
              "evaluated_mappings"):
        assert sa[k] == sb[k], k
    assert sb["engine"] == F.ENGINE_MFMA and sb["matrix_flops"] > 0
    assert sb["ms_device"] > 0 and sb["ms_search"] > 0
    assert (_coverage(b, b["w"], 512, 512, sizes[0]) == 1).all()


@pytest.mark.gpu
def test_gpu_quadtree_device_planned_across_frames():
    # one engine, frames of different content and size in turn (the cached level grids, the plans and
    # the buffers sized by the first frame are reused or regrown): each equals a fresh engine's frame
    lenna = plane("lenna_y")
    frames = [lenna, lenna[::-1, ::-1].copy(), plane("crop64"), lenna[:256, :384].copy(), lenna]
    with F.Engine(0, 4, True) as e:
        for i, p in enumerate(frames):
            e.set_frame(p)
            got, sg = e.encode_quadtree(16, 4, 4.0)
            with F.Engine(0, 4, True, 0.0, -1.0, F.ENGINE_VALU) as f:
                f.set_frame(p)
                want, sw = f.encode_quadtree(16, 4, 4.0)
            np.testing.assert_array_equal(got, want, err_msg=f"frame {i}")
            assert sg["rejected_mappings"] == sw["rejected_mappings"], i


@pytest.mark.gpu
def test_gpu_quadtree_leaves_into_pinned_memory():
    # a pinned `out` is written by the device directly (the emit kernels, over PCIe); the same items as a
    # pageable buffer's copy path, and a short pinned buffer receives exactly its prefix
    import torch
    p = plane("lenna_y")
    cap = (512 // 4) ** 2
    pinned = torch.empty(cap * F.ENCODE_ITEM.itemsize, dtype=torch.uint8).pin_memory().numpy().view(F.ENCODE_ITEM)
    with F.Engine(0, 4, True) as e:
        e.set_frame(p)
        want, sw = e.encode_quadtree(16, 4, 4.0)
        got, sg = e.encode_quadtree(16, 4, 4.0, out=pinned)
        np.testing.assert_array_equal(got, want)
        assert np.shares_memory(got, pinned) and sg["rejected_mappings"] == sw["rejected_mappings"]
        pinned[:] = np.zeros(1, dtype=F.ENCODE_ITEM)
        short = pinned[: len(want) // 3]
        part, sp = e.encode_quadtree(16, 4, 4.0, out=short, allow_short=True)
        assert sp["items"] == len(want) and len(part) == len(short)
        np.testing.assert_array_equal(part, want[: len(short)])
        assert (pinned[len(short):] == np.zeros(1, dtype=F.ENCODE_ITEM)).all()  # nothing past the capacity


@pytest.mark.gpu
@pytest.mark.parametrize("leaves", [False, True])
def test_gpu_quadtree_levels_into_pinned_memory_across_frames(leaves):
    """Pinned output at C4 size, every level's emit writing across PCIe: frames in turn (different frames, so a
    stale item shows) and a capacity that ends inside the 8-pixel level's leaves equal the pageable path's items.
    (Round 6 measured staging the earlier levels in HBM with a side-stream copy during the next level: slower,
    C4q 1.305 → 1.336 ms, profiles/r06/c4q_host/.)"""
    import torch

    from fractencode_amd.synth import value_noise

    big = value_noise(4096, 4096, 1234)
    frames = [big[:2048, :2048].copy(), big[2048:, 2048:].copy(), big[:2048, 2048:].copy()]
    dt = F.QT_LEAF if leaves else F.ENCODE_ITEM
    cap = (2048 // 4) ** 2
    pinned = torch.empty(cap * dt.itemsize, dtype=torch.uint8).pin_memory().numpy().view(dt)
    with F.Engine(0, 4, True) as e:
        for k, fr in enumerate(frames * 2):
            e.set_frame(fr)
            want, sw = e.encode_quadtree(16, 4, 0.05, leaves=leaves)
            pinned[:] = np.zeros(1, dtype=dt)
            got, sg = e.encode_quadtree(16, 4, 0.05, out=pinned, leaves=leaves)
            assert np.shares_memory(got, pinned) and got.tobytes() == want.tobytes(), k
            assert sg["items"] == sw["items"] and sg["rejected_mappings"] == sw["rejected_mappings"], k
            sizes = want["w"] if not leaves else 1 << (want["code"] >> 28)
            n16 = int((sizes == 16).sum())
            m = n16 + int((sizes == 8).sum()) // 2  # inside the staged 8-pixel level
            pinned[:] = np.zeros(1, dtype=dt)
            part, sp = e.encode_quadtree(16, 4, 0.05, out=pinned[:m], leaves=leaves, allow_short=True)
            assert sp["items"] == len(want) and part.tobytes() == want[:m].tobytes(), k
            assert not pinned[m:].tobytes().strip(b"\0"), k  # nothing past the capacity


def _leaves_from_records(rec, W):
    """numpy restatement of frac_qt_leaf packing (include/fracenc.h): the test's independent packer."""
    n = rec["w"].astype(np.int64)
    cols = (W - 2 * n) // n + 1
    has = rec["sw"] != 0
    d = np.where(has, (rec["dy"].astype(np.int64) // n) * cols + rec["dx"].astype(np.int64) // n, F.QT_NO_DOMAIN)
    lv = np.log2(n).astype(np.int64)
    out = np.zeros(len(rec), dtype=F.QT_LEAF)
    out["x"], out["y"] = rec["x"], rec["y"]
    out["code"] = (d & 0xFFFFFF) | ((rec["transform"].astype(np.int64) & 15) << 24) | (lv << 28)
    for k in ("contrast", "brightness", "distance"):
        out[k] = rec[k]
    return out


def test_records_from_leaves_round_trip():
    # mixed sizes 2..16 on a 96×64 frame, the no-domain default record included
    rng = np.random.default_rng(9)
    W, H = 96, 64
    rec = np.zeros(200, dtype=F.ENCODE_ITEM)
    n = rng.choice([2, 4, 8, 16], size=len(rec))
    rec["w"] = rec["h"] = n
    rec["x"] = rng.integers(0, W // 16, len(rec)) * 16
    rec["y"] = rng.integers(0, H // 16, len(rec)) * 16
    cols, rows = (W - 2 * n) // n + 1, (H - 2 * n) // n + 1
    d = (rng.random(len(rec)) * cols * rows).astype(np.int64)
    rec["dx"], rec["dy"] = (d % cols) * n, (d // cols) * n
    rec["sw"] = rec["sh"] = 2 * n
    rec["transform"] = rng.integers(0, 8, len(rec))
    rec["distance"], rec["contrast"], rec["brightness"] = rng.random(len(rec)) * 100, rng.normal(size=len(rec)), \
        rng.normal(size=len(rec)) * 50
    none = rng.random(len(rec)) < 0.1  # the default record: domain (0, 0), size (0, 0), Id, dist 1e5, s = o = 0
    rec["dx"][none] = rec["dy"][none] = rec["sw"][none] = rec["sh"][none] = 0
    rec["transform"][none] = 0
    rec["distance"][none], rec["contrast"][none], rec["brightness"][none] = 1e5, 0.0, 0.0
    leaves = _leaves_from_records(rec, W)
    assert ((leaves["code"][none] & 0xFFFFFF) == F.QT_NO_DOMAIN).all()
    np.testing.assert_array_equal(F.records_from_leaves(leaves, W), rec)


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [F.ENGINE_AUTO, F.ENGINE_VALU], ids=["device_planned", "host_planned"])
@pytest.mark.parametrize("cls,T", [(True, 4), (False, 8)])
def test_gpu_quadtree_32_byte_leaves(engine, cls, T):
    # frac_encode_quadtree_leaves: the 32-byte leaves are the records' packing (independent numpy packer),
    # rebuild the records bit for bit, into pageable and pinned buffers, on both the device-planned and the
    # host-planned levels
    import torch
    p = plane("lenna_y")
    cap = (512 // 4) ** 2
    pinned = torch.empty(cap * F.QT_LEAF.itemsize, dtype=torch.uint8).pin_memory().numpy().view(F.QT_LEAF)
    with F.Engine(0, T, cls, 0.0, -1.0, engine) as e:
        e.set_frame(p)
        want, sw = e.encode_quadtree(16, 4, 4.0)
        got, sg = e.encode_quadtree(16, 4, 4.0, leaves=True)
        pin, sp = e.encode_quadtree(16, 4, 4.0, out=pinned, leaves=True)
    assert got.dtype == F.QT_LEAF and len(got) == len(want) == sg["items"] == sp["items"]
    np.testing.assert_array_equal(got, _leaves_from_records(want, 512))
    np.testing.assert_array_equal(pin, got)
    assert np.shares_memory(pin, pinned)
    np.testing.assert_array_equal(F.records_from_leaves(got, 512), want)
    assert sg["rejected_mappings"] == sw["rejected_mappings"]


@pytest.mark.gpu
def test_device_count_and_quadtree_on_a_context_of_another_device():
    # frac_device_count (ABI 7) sees the devices torch sees; a quadtree frame on a context of device 1 while the
    # calling thread's current device is 0 lands every buffer and launch on device 1 (frac_encode_quadtree sets
    # the context's device first: ADVICE r04) — the same leaves as on device 0
    import torch
    n = F.lib().frac_device_count()
    assert n == torch.cuda.device_count() and n >= 1
    with pytest.raises(F.FracError):
        F.Engine(n, 4)  # past the last device: frac_create refuses it
    if n < 2:
        pytest.skip("one GPU on this box: the cross-device half needs two")
    p = plane("lenna_y")
    with F.Engine(0, 4, True) as e0:
        e0.set_frame(p)
        want, _ = e0.encode_quadtree(16, 4, 4.0)
    with F.Engine(1, 4, True) as e1:
        e1.set_frame(p)
        torch.cuda.set_device(0)
        got, _ = e1.encode_quadtree(16, 4, 4.0)
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
def test_gpu_quadtree_fp32_regime_levels():
    # isolated white blocks on a dark frame push ranges of the 16 and 8 levels into the fp32 regime (S16 ≥ 2^24):
    # the device-planned levels list them and fallback_grid settles each level before its split decision reads
    # the distances; the leaves equal the host-planned VALU engine's (which runs fallback_grid in every run)
    from fractencode_amd.synth import value_noise
    S = 512
    p = (value_noise(S, S, 1234).astype(np.float64) * (60.0 / 255.0)).astype(np.uint8)
    for k, (y0, x0) in enumerate([(24, 48), (120, 240), (312, 96), (408, 432), (216, 360)]):
        p[y0:y0 + 24, x0:x0 + 24] = 0
        p[y0 + 8:y0 + 16, x0 + 8:x0 + 16] = 255
    out = {}
    for eng in (F.ENGINE_AUTO, F.ENGINE_VALU):
        with F.Engine(0, 4, False, 0.0, -1.0, eng) as e:
            e.set_frame(p)
            out[eng] = e.encode_quadtree(16, 4, 2.0)
    (a, sa), (b, sb) = out[F.ENGINE_AUTO], out[F.ENGINE_VALU]
    assert sa["fallback_ranges"] == sb["fallback_ranges"] > 0
    np.testing.assert_array_equal(a, b)
