"""Quantizer + FRC1 stream (fractencode_amd/codec.py), CPU only.

Pinned against the reference's Frac::Quantizerd (encode/Quantizer.hpp:7-45) two ways:
the committed golden tests/golden/lenna_t4_quant.npz (the reference build quantizing
the Lenna T=4 winners with main.cpp:120-121's 5/7 bits), and — when oracle/_ref is
built — the reference quantizer on random values.
"""
import numpy as np
import pytest

from fractencode_amd import ENCODE_ITEM
from fractencode_amd import codec
from golden_util import GOLD, encode_items, golden, oracle_records


def test_quantizer_matches_reference_golden():
    rec, _ = golden("lenna_t4")
    z = np.load(f"{GOLD}/lenna_t4_quant.npz")
    for key, bits in (("s", 5), ("o", 7)):
        q = codec.Quantizer(rec[key].min(), rec[key].max(), bits)
        codes = q.quantized(rec[key])
        np.testing.assert_array_equal(codes, z["q_" + key])
        np.testing.assert_array_equal(q.value(codes), z["v_" + key])  # bit-exact, FMA included


def test_quantizer_matches_reference_build_random(oracle):
    rng = np.random.default_rng(5)
    got_any = False
    for bits in (2, 5, 7, 8, 12):
        lo, hi = sorted(rng.normal(0, 100, 2))
        v = np.concatenate([[lo, hi], rng.uniform(lo, hi, 2000)])
        ref = oracle.ref_quantize(lo, hi, bits, v)
        if ref is None:
            pytest.skip("oracle/_ref not built (no /root/reference here)")
        got_any = True
        q = codec.Quantizer(lo, hi, bits)
        np.testing.assert_array_equal(q.quantized(v), ref[0])
        np.testing.assert_array_equal(q.value(q.quantized(v)), ref[1])
    assert got_any


def test_quantizer_edges():
    q = codec.Quantizer(-1.0, 3.0, 2)
    assert q.step == 1.0
    np.testing.assert_array_equal(q.quantized([-1.0, -0.5, 0.0, 2.99, 3.0]), [0, 0, 1, 3, 3])  # max clamps to 2^b-1
    np.testing.assert_array_equal(q.value([0, 1, 2, 3]), [-0.5, 0.5, 1.5, 2.5])
    with pytest.raises(ValueError):
        codec.Quantizer(1.0, 1.0, 5)
    with pytest.raises(ValueError):
        codec.Quantizer(0.0, 1.0, 1)
    with pytest.raises(ValueError):
        q.value([4])


def _lenna_items(name="lenna_t4"):
    rec, meta = golden(name)
    return encode_items(rec, meta["tgt"]), meta


@pytest.mark.parametrize("name", ["lenna_t4", "lenna_t8", "lenna_cls", "lenna_n4", "lenna_n16", "crop64_n2_t8"])
def test_stream_roundtrip(name):
    items, meta = _lenna_items(name)
    n = meta["tgt"]
    side = int(round((len(items)) ** 0.5)) * n
    buf = codec.pack_stream(items, side, side, n, meta["src"], transforms=meta["T"], use_classifier=meta["cls"])
    back, h = codec.unpack_stream(buf)
    assert h["n_ranges"] == len(items) and h["transforms"] == meta["T"]
    for k in ("x", "y", "w", "h", "dx", "dy", "sw", "sh", "transform"):
        np.testing.assert_array_equal(back[k], items[k], err_msg=k)
    for key, field, bits in (("s", "contrast", 5), ("o", "brightness", 7)):
        v = items[field]
        q = codec.Quantizer(v.min(), v.max(), bits)
        np.testing.assert_array_equal(back[field], q.value(q.quantized(v)))
        # dequantization error is at most one step (half a step except at the clamped top code)
        assert np.all(np.abs(back[field] - v) <= q.step)
    rec_bits = h["index_bits"] + max(1, (meta["T"] - 1).bit_length()) + 12
    assert len(buf) == codec.HEADER.size + (len(items) * rec_bits + 7) // 8


def test_stream_size_at_c3():
    # 4096² / n=8: 261,121 domains → 18 index bits, T=4 → 2, 5 + 7 → 32 bits per range
    items = np.zeros(512 * 512, dtype=ENCODE_ITEM)
    r = np.arange(len(items))
    items["x"], items["y"] = (r % 512) * 8, (r // 512) * 8
    items["w"] = items["h"] = 8
    items["dx"], items["dy"] = (r % 511) * 8, (r % 509) * 8
    items["sw"] = items["sh"] = 16
    items["contrast"] = np.linspace(-1, 1, len(items))
    items["brightness"] = np.linspace(0, 255, len(items))
    buf = codec.pack_stream(items, 4096, 4096, 8)
    assert len(buf) == codec.HEADER.size + 4 * len(items)
    back, h = codec.unpack_stream(buf)
    assert h["index_bits"] == 18
    np.testing.assert_array_equal(back["dx"], items["dx"])
    np.testing.assert_array_equal(back["dy"], items["dy"])


def test_stream_empty_and_degenerate_records():
    items, meta = _lenna_items("crop64_t4")
    items = items.copy()
    items[3]["sw"] = items[3]["sh"] = 0  # a range with no eligible domain (default record)
    items[3]["dx"] = items[3]["dy"] = 0
    items["contrast"] = 0.25  # degenerate field: every value equal
    buf = codec.pack_stream(items, 64, 64, 8)
    back, h = codec.unpack_stream(buf)
    assert back[3]["sw"] == 0 and back[3]["contrast"] == 0.0 and back[3]["brightness"] == 0.0
    assert h["contrast_min"] == h["contrast_max"] == 0.25
    assert np.all(np.delete(back["contrast"], 3) == 0.25)


def test_stream_rejects_bad_input():
    items, _ = _lenna_items("crop64_t4")
    with pytest.raises(ValueError):
        codec.pack_stream(items[:-1], 64, 64, 8)
    bad = items.copy()
    bad[[0, 1]] = bad[[1, 0]]
    with pytest.raises(ValueError):
        codec.pack_stream(bad, 64, 64, 8)
    bad = items.copy()
    bad[0]["dx"] = 3
    with pytest.raises(ValueError):
        codec.pack_stream(bad, 64, 64, 8)
    buf = codec.pack_stream(items, 64, 64, 8)
    with pytest.raises(ValueError):
        codec.unpack_stream(b"XXXX" + buf[4:])
    with pytest.raises(ValueError):
        codec.unpack_stream(buf[:-3])


def test_quantized_decode_oracle_psnr(oracle):
    # the full CPU chain the GPU path is checked against: reference winners → FRC1 →
    # dequantized records → Decoder2 (oracle) → PSNR against the source plane
    from golden_util import plane

    items, meta = _lenna_items("lenna_t4")
    src = plane("lenna_y")
    dec_full, _, _ = oracle.decode(oracle_records(items), 8, 512, 512)
    back, _ = codec.unpack_stream(codec.pack_stream(items, 512, 512, 8))
    dec_q, it, _ = oracle.decode(oracle_records(back), 8, 512, 512)
    p_full, p_q = codec.psnr(src, dec_full), codec.psnr(src, dec_q)
    assert 25.0 < p_q <= p_full + 0.5, (p_full, p_q)
    assert codec.psnr(src, src) == float("inf")
