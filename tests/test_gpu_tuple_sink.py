"""frac_set_tuple_sink (ABI 8): every run also writes its 32-byte tuples into a caller's buffer — the fused
resolvers (and fallback_grid) write them beside the records, other fits are packed after the run.  The sink's
bytes equal frac_fetch_tuples' for device memory and for pinned host memory, on every engine, with the
classifier, all 8 transforms, a hit threshold, fp32-regime ranges and empty ranges; the quadtree ignores it."""
import os
import sys

import numpy as np
import pytest

import fractencode_amd as F
from golden_util import plane

pytestmark = pytest.mark.gpu

ENGINES = [F.ENGINE_VALU, F.ENGINE_MFMA, F.ENGINE_SEA]


def _sink_bytes(e, nr, where):
    import torch

    n = nr * F.TUPLE.itemsize
    buf = torch.full((n,), 0xAB, dtype=torch.uint8, device="cuda:0") if where == "device" else \
        torch.full((n,), 0xAB, dtype=torch.uint8).pin_memory()
    e.set_tuple_sink(buf.data_ptr())
    e.run()
    e.set_tuple_sink(None)
    e.sync()
    torch.cuda.synchronize()
    return buf.cpu().numpy().tobytes()


@pytest.mark.parametrize("where", ["device", "pinned"])
@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("T,cls,thr", [(4, False, 0.0), (8, False, 0.0), (4, True, 0.0), (8, True, 2.0)])
@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_sink_equals_fetch_tuples(engine, where, T, cls, thr, n):
    # every range size with a templated engine (the fused resolvers at n = 2/4/8/16, the SEA paths, the
    # separate fits), domains 2n at stride n; n = 2 on a 128² crop to keep the pool small
    y = plane("lenna_y")
    if n == 2:
        y = np.ascontiguousarray(y[192:320, 192:320])
    H, W = y.shape
    rngs = F.create_uniform_grid(W, H, n, n)
    with F.Engine(0, T, cls, thr, -1.0, engine) as e:
        e.set_frame(y)
        e.set_domains(F.create_uniform_grid(W, H, 2 * n, n))
        e.set_ranges(rngs)
        got = _sink_bytes(e, len(rngs), where)
        want = e.fetch_tuples().tobytes()
    assert got == want


def test_sampled_run_after_a_fused_run_on_one_context():
    """A context that ran the fused n = 8 Fourier search (its resolvers write the records and the sink, and
    list fp32-regime ranges for a deferred fallback) and then gets 6×6 ranges (the sampled form: a separate
    fit, tuples packed after the run): the second run's sink, tuples and records are its own — no stale
    fused state or deferred fallback of the first run leaks into them."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from fallback_probe import frame

    p = frame(6, 512)  # fp32-regime ranges: the first run leaves a deferred fallback behind
    doms = F.create_uniform_grid(512, 512, 16, 8)
    r8 = F.create_uniform_grid(512, 512, 8, 8)
    r6 = F.create_uniform_grid(512, 512, 6, 6)
    with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_MFMA) as fresh:
        fresh.set_frame(p)
        fresh.set_domains(doms)
        want, _ = fresh.search(r6)
        want_t = fresh.fetch_tuples().tobytes()
    with F.Engine(0, 4, False, 0.0, -1.0, F.ENGINE_MFMA) as e:
        e.set_frame(p)
        e.set_domains(doms)
        e.set_ranges(r8)
        _sink_bytes(e, len(r8), "device")  # the fused run, settled by sync()
        e.set_ranges(r8)
        e.run()  # a second fused run whose fallback stays pending (nothing read its records)
        e.set_ranges(r6)
        got_sink = _sink_bytes(e, len(r6), "pinned")
        got, st = e.fetch()
        got_t = e.fetch_tuples().tobytes()
    assert st["search_form"] == F.FORM_SAMPLED
    assert got_sink == want_t and got_t == want_t
    assert got.tobytes() == want.tobytes()


def test_sink_with_fp32_regime_and_empty_ranges():
    # white 8×8 ranges in black patches over dimmed noise: their best errors are ≥ 2^24 (fallback_grid writes
    # their records and tuples); with the classifier the resolvers and fallback_grid write the sink alike
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from fallback_probe import frame

    p = frame(6, 512)
    rngs = F.create_uniform_grid(512, 512, 8, 8)
    for cls in (False, True):
        with F.Engine(0, 4, cls, 0.0, -1.0, F.ENGINE_AUTO) as e:
            e.set_frame(p)
            e.set_domains(F.create_uniform_grid(512, 512, 16, 8))
            e.set_ranges(rngs)
            got = _sink_bytes(e, len(rngs), "pinned")
            _, st = e.fetch()
            want = e.fetch_tuples().tobytes()
        if not cls:
            assert st["fallback_ranges"] > 0
        assert got == want


def test_quadtree_ignores_the_sink():
    import torch

    y = plane("lenna_y")
    rngs = F.create_uniform_grid(512, 512, 8, 8)
    buf = torch.full((len(rngs) * F.TUPLE.itemsize,), 0xAB, dtype=torch.uint8, device="cuda:0")
    with F.Engine(0, 4, True) as e:
        e.set_frame(y)
        e.set_tuple_sink(buf.data_ptr())
        e.encode_quadtree(16, 4, 0.05)
        torch.cuda.synchronize()
        assert bool((buf == 0xAB).all())  # the levels wrote nothing into it
        e.set_domains(F.create_uniform_grid(512, 512, 16, 8))
        e.set_ranges(rngs)
        e.run()  # the sink is still set for the context's own runs
        e.sync()
        torch.cuda.synchronize()
        assert buf.cpu().numpy().tobytes() == e.fetch_tuples().tobytes()
