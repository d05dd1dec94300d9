"""GPU Decoder2 (fracenc_decode.hip) and the quantized-stream chain against the
reference / oracle decoders.  Bar: the decoded plane, the iteration count and the
final rms are identical (the decode is fixed-point given identical records:
fma(s, D/4, o) with a truncating clamp, encode/DecodeUtils.hpp:9-25).
"""
import json

import numpy as np
import pytest

import fractencode_amd as F
from fractencode_amd import codec
from golden_util import GOLD, encode_items, golden, oracle_records, plane

pytestmark = pytest.mark.gpu


def _encode(p, src, tgt, T=4, cls=False, engine=F.ENGINE_AUTO):
    H, W = p.shape
    doms = F.create_uniform_grid(W, H, src, src // 2)
    rngs = F.create_uniform_grid(W, H, tgt, tgt)
    if cls:
        doms, rngs = F.preclassify(p, doms), F.preclassify(p, rngs)
    return doms, rngs


def test_decode_matches_reference_golden():
    rec, _ = golden("lenna_t4")
    z = np.load(f"{GOLD}/lenna_t4_decode.npz")
    dmeta = json.loads(bytes(z["meta"]).decode())
    with F.Engine(0, 4) as e:
        dec, it, rms = e.decode(encode_items(rec, 8), 512, 512)
    assert it == dmeta["iterations"] and rms == dmeta["rms"]
    np.testing.assert_array_equal(dec, z["plane"])


@pytest.mark.parametrize("name", ["lenna_t8", "lenna_cls", "lenna_n4", "lenna_n16", "lenna_16to4", "lenna_u_t4",
                                  "crop64_n2_t8", "checker64_t8"])
def test_decode_matches_oracle(oracle, name):
    rec, meta = golden(name)
    p = plane(meta["plane"])
    H, W = p.shape
    items = encode_items(rec, meta["tgt"])
    want, wit, wrms = oracle.decode(oracle_records(items), meta["tgt"], W, H)
    with F.Engine(0, meta["T"]) as e:
        got, it, rms = e.decode(items, W, H)
        # a bounded run stops at max_iter like the reference
        got3, it3, _ = e.decode(items, W, H, max_iter=3)
    want3, wit3, _ = oracle.decode(oracle_records(items), meta["tgt"], W, H, max_iter=3)
    assert (it, rms) == (wit, wrms)
    np.testing.assert_array_equal(got, want)
    assert it3 == wit3 <= 3
    np.testing.assert_array_equal(got3, want3)


@pytest.mark.parametrize("engine", [F.ENGINE_VALU, F.ENGINE_MFMA])
def test_decode_results_on_device(oracle, engine):
    # encode on the GPU, decode the device-resident winners without a host round trip
    p = plane("lenna_y")
    doms, rngs = _encode(p, 16, 8)
    with F.Engine(0, 4, engine=engine) as e:
        e.set_frame(p)
        e.set_domains(doms)
        out, _ = e.search(rngs)
        got, it, rms = e.decode(None, 512, 512)
    want, wit, wrms = oracle.decode(oracle_records(out), 8, 512, 512)
    assert (it, rms) == (wit, wrms)
    np.testing.assert_array_equal(got, want)


def test_quantized_stream_decode_and_psnr(oracle):
    # GPU encode → FRC1 → dequantized records → GPU decode, against the oracle decoding the
    # same stream; PSNR of both against the source plane is then identical by construction
    p = plane("lenna_y")
    doms, rngs = _encode(p, 16, 8)
    with F.Engine(0, 4) as e:
        e.set_frame(p)
        e.set_domains(doms)
        out, _ = e.search(rngs)
        buf = codec.pack_stream(out, 512, 512, 8)
        back, _ = codec.unpack_stream(buf)
        got, it, rms = e.decode(back, 512, 512)
    want, wit, wrms = oracle.decode(oracle_records(back), 8, 512, 512)
    assert (it, rms) == (wit, wrms)
    np.testing.assert_array_equal(got, want)
    assert codec.psnr(p, got) == codec.psnr(p, want) > 25.0


def test_decode_skips_empty_records_and_large_plane(oracle):
    # ranges with no eligible domain (default record, 0×0 source) are left untouched, and a
    # 1024² random encoding checks the int32 wrap of the reference's rms sum (metrics.h:29)
    rng = np.random.default_rng(3)
    W = H = 1024
    n = 8
    nr = (W // n) * (H // n)
    items = np.zeros(nr, dtype=F.ENCODE_ITEM)
    r = np.arange(nr)
    items["x"], items["y"] = (r % (W // n)) * n, (r // (W // n)) * n
    items["w"] = items["h"] = n
    items["dx"] = rng.integers(0, (W - 2 * n) // n + 1, nr) * n
    items["dy"] = rng.integers(0, (H - 2 * n) // n + 1, nr) * n
    items["sw"] = items["sh"] = 2 * n
    items["transform"] = rng.integers(0, 8, nr)
    items["contrast"] = rng.uniform(-1.2, 1.2, nr)
    items["brightness"] = rng.uniform(-60, 300, nr)
    items["sw"][::97] = 0
    items["sh"][::97] = 0
    init = rng.integers(0, 256, (H, W), dtype=np.uint8)
    with F.Engine(0, 8) as e:
        got, it, rms = e.decode(items, W, H, max_iter=6, initial=init)
    want, wit, wrms = oracle.decode(oracle_records(items), n, W, H, max_iter=6, initial=init)
    assert (it, rms) == (wit, wrms)
    np.testing.assert_array_equal(got, want)


def test_decode_rejects_bad_items():
    rec, _ = golden("crop64_t4")
    items = encode_items(rec, 8)
    bad = items.copy()
    bad[0]["dx"] = 60
    with F.Engine(0, 4) as e:
        with pytest.raises(F.FracError):
            e.decode(bad, 64, 64)
        bad = items.copy()
        bad[1]["transform"] = 9
        with pytest.raises(F.FracError):
            e.decode(bad, 64, 64)
        with pytest.raises(F.FracError):
            e.decode(None, 64, 64)  # nothing ran yet


@pytest.mark.parametrize("name", ["lenna_t4", "lenna_n4", "crop64_n2_t8"])
def test_fused_and_stepwise_decoders_agree(name):
    # the fused decoder (exact coverage: rms accumulated while writing, buffer swap, device-side
    # convergence test) against the step-by-step form, including bounded iteration counts
    rec, meta = golden(name)
    p = plane(meta["plane"])
    H, W = p.shape
    items = encode_items(rec, meta["tgt"])
    outs = []
    for fl in (0, F.FLAG_DECODE_STEPWISE):
        with F.Engine(0, 4, flags=fl) as e:
            outs.append([e.decode(items, W, H, max_iter=m) for m in (-1, 0, 1, 2, 9)])
    for (a, ia, ra), (b, ib, rb) in zip(*outs):
        assert (ia, ra) == (ib, rb)
        np.testing.assert_array_equal(a, b)
