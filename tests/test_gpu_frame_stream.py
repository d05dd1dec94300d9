"""Frame streaming on one context (ABI 9, frac_set_frame_device_async): each frame is uploaded on a copy stream
of its own while the previous one searches, the context's stream waits for the upload (an event), copies the
plane device-to-device without a host wait and runs with the tuple sink into pinned memory.  Every frame's
tuples and records equal a synchronous search of that frame (the reference goldens for Lenna), with the
classifier off and on (on: the host re-prepares per frame), and with fp32-regime ranges in flight."""
import os
import sys

import numpy as np
import pytest

import fractencode_amd as F
from golden_util import FIELDS, golden, plane

pytestmark = pytest.mark.gpu


def _sync_search(p, cls, doms, rngs):
    with F.Engine(0, 4, cls) as e:
        e.set_frame(p)
        e.set_domains(doms)
        out, _ = e.search(rngs)
        return out, e.fetch_tuples().tobytes()


@pytest.mark.parametrize("cls", [False, True])
def test_host_streamed_frames_equal_synchronous_searches(cls):
    """frac_set_frame_async: frames from pinned host memory uploaded on the context's copy stream into its second
    plane buffer while the previous frame searches; every frame's tuples (sink) and the last records equal a
    synchronous search of that frame."""
    import torch

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from fallback_probe import frame as fp32_frame

    y = plane("lenna_y")
    frames = [y, np.ascontiguousarray(y[::-1]), fp32_frame(6, 512), np.ascontiguousarray(y[:, ::-1])] * 2
    doms = F.create_uniform_grid(512, 512, 16, 8)
    rngs = F.create_uniform_grid(512, 512, 8, 8)
    want = [_sync_search(p, cls, doms, rngs) for p in frames[:4]]
    hosts = [torch.from_numpy(p).pin_memory() for p in frames]
    sinks = [torch.zeros(len(rngs) * F.TUPLE.itemsize, dtype=torch.uint8).pin_memory() for _ in frames]
    with F.Engine(0, 4, cls) as e:
        e.set_frame(frames[0])
        e.set_domains(doms)
        e.set_ranges(rngs)
        for k, h in enumerate(hosts):
            e.set_frame_async(h)
            e.set_tuple_sink(sinks[k].data_ptr())
            e.run()
        e.set_tuple_sink(None)
        last, _ = e.fetch()
        e.set_frame(frames[1])  # a synchronous frame after the streamed ones
        again, _ = e.search(rngs)
    for k, s in enumerate(sinks):
        assert s.numpy().tobytes() == want[k % 4][1], k
    assert last.tobytes() == want[3][0].tobytes()
    assert again.tobytes() == want[1][0].tobytes()


@pytest.mark.parametrize("cls", [False, True])
def test_streamed_frames_equal_synchronous_searches(cls):
    import torch

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from fallback_probe import frame as fp32_frame

    y = plane("lenna_y")
    frames = [y, np.ascontiguousarray(y[::-1]), fp32_frame(6, 512), np.ascontiguousarray(y[:, ::-1])] * 2
    dev = torch.device("cuda", 0)
    doms = F.create_uniform_grid(512, 512, 16, 8)
    rngs = F.create_uniform_grid(512, 512, 8, 8)
    want = [_sync_search(p, cls, doms, rngs) for p in frames[:4]]
    compute, up = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    hosts = [torch.from_numpy(p).pin_memory() for p in frames]
    bufs = [torch.empty((512, 512), dtype=torch.uint8, device=dev) for _ in range(2)]
    sinks = [torch.zeros(len(rngs) * F.TUPLE.itemsize, dtype=torch.uint8).pin_memory() for _ in frames]
    up_ev = [torch.cuda.Event() for _ in range(2)]
    free_ev = [torch.cuda.Event() for _ in range(2)]
    with F.Engine(0, 4, cls) as e:
        e.set_stream(compute.cuda_stream)
        e.set_frame(frames[0])
        e.set_domains(doms)
        e.set_ranges(rngs)
        for ev in free_ev:
            ev.record(compute)
        for k, h in enumerate(hosts):
            j = k & 1
            up.wait_event(free_ev[j])
            with torch.cuda.stream(up):
                bufs[j].copy_(h, non_blocking=True)
            up_ev[j].record(up)
            compute.wait_event(up_ev[j])
            e.set_frame_device_async(bufs[j])
            free_ev[j].record(compute)
            e.set_tuple_sink(sinks[k].data_ptr())
            e.run()
        e.set_tuple_sink(None)
        last, _ = e.fetch()
        torch.cuda.synchronize(dev)
    for k, s in enumerate(sinks):
        assert s.numpy().tobytes() == want[k % 4][1], k
    assert last.tobytes() == want[3][0].tobytes()
    rec, meta = golden("lenna_cls" if cls else "lenna_t4")
    got = want[0][0]
    fields = {"x": got["x"], "y": got["y"], "dx": got["dx"], "dy": got["dy"], "dw": got["sw"], "dh": got["sh"],
              "t": got["transform"], "dist": got["distance"], "s": got["contrast"], "o": got["brightness"]}
    for k in FIELDS:
        np.testing.assert_array_equal(fields[k], rec[k], err_msg=k)


def test_set_frame_device_async_rejects_host_planes():
    with F.Engine(0) as e:
        with pytest.raises(F.FracError):
            e.set_frame_device_async(np.zeros((64, 64), np.uint8))


def test_stream_switch_settles_the_pending_fp32_fallback():
    """A run whose fp32-regime ranges wait for the deferred fallback_grid, then frac_set_stream to another
    stream before anything reads the records: the fallback runs on the stream the search and
    resolve ran on, the new stream waits for that work, and the records fetched on it equal a fresh context's."""
    import torch

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from fallback_probe import frame as fp32_frame

    p = fp32_frame(6, 512)
    doms = F.create_uniform_grid(512, 512, 16, 8)
    rngs = F.create_uniform_grid(512, 512, 8, 8)
    want = _sync_search(p, False, doms, rngs)[0]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with F.Engine(0, 4) as e:
        e.set_stream(s1.cuda_stream)
        e.set_frame(p)
        e.set_domains(doms)
        e.set_ranges(rngs)
        e.run()  # the fused resolvers list the fp32-regime ranges; their fallback is deferred
        e.set_stream(s2.cuda_stream)  # settles it on s1 first
        got, st = e.fetch()
    assert st["fallback_ranges"] > 0
    assert got.tobytes() == want.tobytes()
