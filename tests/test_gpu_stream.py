"""FRC1 packed on the device (frac_pack_frc1) equals the host restatement (codec.pack_stream)
byte for byte; the stream decodes back to the search's (domain, transform) and quantized
(contrast, brightness)."""
import numpy as np
import pytest

import fractencode_amd as F
from fractencode_amd import codec
from golden_util import plane

pytestmark = pytest.mark.gpu


def _search(p, T, cls, n=8):
    H, W = p.shape
    doms = F.create_uniform_grid(W, H, 2 * n, n)
    rngs = F.create_uniform_grid(W, H, n, n)
    e = F.Engine(0, T, cls)
    e.set_frame(p)
    e.set_domains(F.preclassify(p, doms) if cls else doms)
    out, st = e.search(F.preclassify(p, rngs) if cls else rngs)
    return e, out, st


@pytest.mark.parametrize("T,cls,bits", [(4, False, (5, 7)), (8, False, (5, 7)), (4, True, (5, 7)), (4, False, (9, 16))])
def test_device_frc1_matches_host_packer(T, cls, bits):
    p = plane("lenna_y")
    e, out, _ = _search(p, T, cls)
    with e:
        dev = e.pack_frc1(*bits)
    host = codec.pack_stream(out, 512, 512, 8, transforms=T, use_classifier=cls, contrast_bits=bits[0],
                             brightness_bits=bits[1])
    assert dev == host
    rec, h = codec.unpack_stream(dev)
    np.testing.assert_array_equal(rec["dx"], out["dx"])
    np.testing.assert_array_equal(rec["transform"], out["transform"])


def test_device_frc1_empty_ranges_and_full_frame():
    # classifier on a small random frame: some ranges have no domain of their category
    rng = np.random.default_rng(0)
    p = rng.integers(0, 256, (32, 32), dtype=np.uint8)  # 5 of its 16 ranges have no domain
    e, out, st = _search(p, 4, True)
    with e:
        dev = e.pack_frc1()
    assert st["empty_ranges"] > 0
    assert dev == codec.pack_stream(out, 32, 32, 8, use_classifier=True)
    # C3 size: 262,144 records of 32 bits
    big = plane("s1_4096")
    e, out, _ = _search(big, 4, False)
    with e:
        dev = e.pack_frc1()
    assert len(dev) == codec.HEADER.size + 262144 * 4
    assert dev == codec.pack_stream(out, 4096, 4096, 8)


def test_device_frc1_rejects_non_lattice_results():
    p = plane("lenna_y")
    with F.Engine(0, 4) as e:
        e.set_frame(p)
        e.set_domains(F.create_uniform_grid(512, 512, 16, 8))
        e.search(F.create_uniform_grid(512, 512, 8, 8)[::-1])  # not row-major
        with pytest.raises(F.FracError):
            e.pack_frc1()
