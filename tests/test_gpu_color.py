"""Device colour conversion (fracenc_color.hip) and the three-plane colour encode
against the reference's goldens: bit-exact Y/U/V, per-plane winners identical to the
reference encoding each plane (main.cpp:184-196)."""
import json

import numpy as np
import pytest

import fractencode_amd as F
from color_util import all_colours_rgb
from fractencode_amd.synth import sha256
from golden_util import FIELDS, GOLD, golden, oracle_records, plane

pytestmark = pytest.mark.gpu


def test_rgb_to_yuv_lenna_host_buffers():
    with F.Engine(0) as e:
        y, u, v = e.rgb_to_yuv(plane("lenna_rgb"))
    np.testing.assert_array_equal(y, plane("lenna_y"))
    np.testing.assert_array_equal(u, plane("lenna_u"))
    np.testing.assert_array_equal(v, plane("lenna_v"))


def test_rgb_to_yuv_odd_sizes_generic_path():
    z = np.load(f"{GOLD}/rgb_synth_yuv.npz")
    with F.Engine(0) as e:
        y, u, v = e.rgb_to_yuv(z["rgb"])
    for got, k in ((y, "y"), (u, "u"), (v, "v")):
        np.testing.assert_array_equal(got, z[k], err_msg=k)


@pytest.mark.parametrize("pad", [0, 5, 64])
def test_rgb_to_yuv_device_strided_rows(oracle, pad):
    import torch

    rng = np.random.default_rng(pad)
    H, W = 130, 260
    big = rng.integers(0, 256, size=(H, W * 3 + pad), dtype=np.uint8)
    rgb = big[:, : W * 3].reshape(H, W, 3)
    t = torch.from_numpy(big).cuda()[:, : W * 3].view(H, W, 3) if pad == 0 else \
        torch.from_numpy(big).cuda().as_strided((H, W, 3), (W * 3 + pad, 3, 1))
    with F.Engine(0) as e:
        y, u, v = e.rgb_to_yuv(t)
    wy, wu, wv = oracle.rgb2yuv(rgb)
    np.testing.assert_array_equal(y.cpu().numpy(), wy)
    np.testing.assert_array_equal(u.cpu().numpy(), wu)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)


def test_rgb_to_yuv_all_colours():
    import torch

    digests = json.load(open(f"{GOLD}/rgb_all_colours.json"))["chunks"]
    with F.Engine(0) as e:
        for k in range(4):
            y, u, v = e.rgb_to_yuv(torch.from_numpy(all_colours_rgb(k)).cuda())
            assert sha256(np.ascontiguousarray(y.cpu().numpy()[::2, ::2])) == digests[k]["y"], k
            assert sha256(u.cpu().numpy()) == digests[k]["u"], k
            assert sha256(v.cpu().numpy()) == digests[k]["v"], k


@pytest.mark.parametrize("engine", [F.ENGINE_VALU, F.ENGINE_MFMA])
def test_color_encoder_matches_reference_planes(oracle, engine):
    from fractencode_amd.color import ColorEncoder
    from fractencode_amd import codec

    with ColorEncoder(0, 8, 16, 4, engine=engine) as enc:
        enc.load(plane("lenna_rgb"))
        enc.run()
        enc.sync()
        results = enc.fetch()
        planes = enc.host_planes()
    for (out, st), name, pname, p in zip(results, ("lenna_t4", "lenna_u_t4", "lenna_v_t4"),
                                         ("lenna_y", "lenna_u", "lenna_v"), planes):
        np.testing.assert_array_equal(p, plane(pname))
        rec, meta = golden(name)
        got = {"x": out["x"], "y": out["y"], "dx": out["dx"], "dy": out["dy"], "dw": out["sw"], "dh": out["sh"],
               "t": out["transform"], "dist": out["distance"], "s": out["contrast"], "o": out["brightness"]}
        for k in FIELDS:
            np.testing.assert_array_equal(got[k], rec[k], err_msg=f"{name}:{k}")
        # decode each plane on the GPU: identical to the oracle decoder, PSNR reported
        H, W = p.shape
        with F.Engine(0) as e:
            dec, it, rms = e.decode(out, W, H)
        want, wit, wrms = oracle.decode(oracle_records(out), 8, W, H)
        assert (it, rms) == (wit, wrms)
        np.testing.assert_array_equal(dec, want)
        assert codec.psnr(p, dec) > 25.0


def test_color_encoder_streams_give_the_same_records():
    # the default runs the three plane searches in turn on one shared stream; streams="own" overlaps
    # them on one stream per engine: the same records either way, frame after frame
    from fractencode_amd.color import ColorEncoder

    rgb = plane("lenna_rgb")
    res = {}
    for streams in ("shared", "own"):
        with ColorEncoder(0, 8, 16, 4, streams=streams) as enc:
            for _ in range(2):
                enc.load(rgb)
                enc.run()
            enc.sync()
            res[streams] = [out.tobytes() for out, _ in enc.fetch()]
    assert res["shared"] == res["own"]
    with pytest.raises(ValueError):
        ColorEncoder(0, streams="two")


def test_color_encoder_with_classifier(oracle):
    # Y against the reference's classifier golden; U and V against the oracle (the engine
    # classifies every plane's grids on the device)
    from fractencode_amd.color import ColorEncoder

    with ColorEncoder(0, 8, 16, 4, use_classifier=True) as enc:
        enc.load(plane("lenna_rgb"))
        enc.run()
        enc.sync()
        results = enc.fetch()
        planes = enc.host_planes()
    rec, meta = golden("lenna_cls")
    out, st = results[0]
    np.testing.assert_array_equal(out["dx"], rec["dx"])
    np.testing.assert_array_equal(out["dy"], rec["dy"])
    np.testing.assert_array_equal(out["transform"], rec["t"])
    np.testing.assert_array_equal(out["distance"], rec["dist"])
    assert st["rejected_mappings"] == meta["rejected"]
    for (out, st), p in zip(results[1:], planes[1:]):
        H, W = p.shape
        doms = oracle.classify(p, oracle.uniform_grid(W, H, 16, 8))
        rngs = oracle.classify(p, oracle.uniform_grid(W, H, 8, 8))
        want, rej, _ = oracle.estimate(p, doms, rngs, T=4, use_classifier=True)
        np.testing.assert_array_equal(out["dx"], want["dx"])
        np.testing.assert_array_equal(out["dy"], want["dy"])
        np.testing.assert_array_equal(out["transform"], want["t"])
        np.testing.assert_array_equal(out["distance"], want["dist"])
        np.testing.assert_array_equal(out["contrast"], want["s"])
        np.testing.assert_array_equal(out["brightness"], want["o"])
        assert st["rejected_mappings"] == rej


def test_c5_chain_quantized_stream_decode_parity(oracle):
    """C5's chain on Lenna RGB: device rgb2yuv → Y/U/V searches → FRC1 packed on the device (Quantizer
    5/7 bits) → dequantized records → GPU Decoder2 per plane, against the oracle decoding the same
    records: identical planes, iteration counts and rms, so identical PSNR."""
    from fractencode_amd.color import ColorEncoder
    from fractencode_amd import codec

    with ColorEncoder(0, 8, 16, 4) as enc:
        enc.load(plane("lenna_rgb"))
        enc.run()
        enc.sync()
        results = enc.fetch()
        planes = enc.host_planes()
        streams = [e.pack_frc1() for e in enc.engines]
    for (out, _), p, buf in zip(results, planes, streams):
        H, W = p.shape
        assert buf == codec.pack_stream(out, W, H, 8)
        back, hdr = codec.unpack_stream(buf)
        with F.Engine(0) as e:
            dec, it, rms = e.decode(back, W, H)
        want, wit, wrms = oracle.decode(oracle_records(back), 8, W, H)
        assert (it, rms) == (wit, wrms)
        np.testing.assert_array_equal(dec, want)
        assert codec.psnr(p, dec) == codec.psnr(p, want) > 20.0


def _c5_worker(rank, world, port, path):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist

    from fractencode_amd.color import ColorEncoder
    from golden_util import plane as gplane

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    with ColorEncoder(0, 8, 16, 4) as enc:  # every rank on GPU 0 (one-GPU box)
        enc.load(gplane("lenna_rgb"))
        full = enc.encode_sharded(rank, world)
    if rank == 0:
        np.savez(path, y=full[0], u=full[1], v=full[2])
    dist.barrier()
    dist.destroy_process_group()


def test_c5_sharded_over_two_ranks_matches_single_rank(tmp_path):
    """world-size-2 ranks shard each plane's ranges and all-gather the 32-byte tuples; the rebuilt
    Y/U/V records equal the single-rank colour encode."""
    import socket

    import torch.multiprocessing as mp
    from fractencode_amd.color import ColorEncoder

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    path = str(tmp_path / "c5.npz")
    mp.spawn(_c5_worker, args=(2, port, path), nprocs=2, join=True)
    got = np.load(path)
    with ColorEncoder(0, 8, 16, 4) as enc:
        enc.load(plane("lenna_rgb"))
        enc.run()
        enc.sync()
        want = [o for o, _ in enc.fetch()]
    for k, w in zip("yuv", want):
        assert got[k].tobytes() == w.tobytes(), k


def test_c5_load_after_sharded_encode_restores_full_ranges():
    """encode_sharded leaves each engine holding one shard; the next load() of a same-geometry frame
    must search every range again (world 1 without a process group: one shard = all ranges, so
    the check uses world 2 / rank 1 and compares with a fresh encoder)."""
    import torch.distributed as dist
    from fractencode_amd.color import ColorEncoder
    from fractencode_amd.distributed import shard_plan

    assert not dist.is_initialized()
    rgb = plane("lenna_rgb")
    with ColorEncoder(0, 8, 16, 4) as enc:
        enc.load(rgb)
        # rank 1 of 2, without a collective: search only the shard (what encode_sharded leaves behind)
        for e, rngs in zip(enc.engines, enc.ranges):
            a, b = shard_plan(len(rngs), 2)[1]
            e.set_ranges(rngs[a:b])
            e.run()
        enc._sharded = True
        enc.load(rgb)
        enc.run()
        enc.sync()
        again = [o for o, _ in enc.fetch()]
    with ColorEncoder(0, 8, 16, 4) as fresh:
        fresh.load(rgb)
        fresh.run()
        fresh.sync()
        want = [o for o, _ in fresh.fetch()]
    for g, w in zip(again, want):
        assert len(g) == len(w) and g.tobytes() == w.tobytes()


def test_set_frame_device_rejects_strided_columns():
    import torch

    t = torch.zeros((64, 128), dtype=torch.uint8, device="cuda")
    with F.Engine(0) as e:
        with pytest.raises(F.FracError):
            e.set_frame(t[:, ::2])
        with pytest.raises(F.FracError):
            e.set_frame(t.to(torch.int16))
        e.set_frame(t[:, :64])  # row stride 128 >= width 64: fine
