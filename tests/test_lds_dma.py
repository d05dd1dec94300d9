"""Static guard of the LDS-DMA stage hand-off ("A stage hand-off race, fixed").

On the GPU the race showed once in about twenty full suites (one C5 range got another domain):
a loop-head `__syncthreads()` compiled to `s_waitcnt lgkmcnt(0); s_barrier` without vmcnt(0), so a
stage could be read before all of its LDS-DMA pieces had landed.  stage_barrier()
(fracenc_mfma.hip) waits vmcnt(0) first.  These CPU tests disassemble gfx950 code and require
that every barrier a pending `global_load_lds` can reach is preceded by `s_waitcnt vmcnt(0)`
on every path (tools/lds_dma_check.py): over the product library's search kernels, and — as the
negative control that shows the check sees the hazard — over the same kernels compiled with the
barrier reduced to a plain `__syncthreads()`.
"""
import os
import subprocess
import sys

import pytest

import fractencode_amd as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import lds_dma_check  # noqa: E402

CSRC = os.path.join(ROOT, "fractencode_amd", "csrc")
FAMILIES = ("search_dft<", "search_mfma<", "search_mfma16<")
# one instance per family, as the product library instantiates them: the shipped C3 search first
# (variant 35 = 1|kDftChain|kDft6|kDftFast6|kDftUnroll|kDftBufDma: buffer_load … lds stages and the
# zero-tail reads of the guarded epilogue), then the SEA tiled form's exact six-MFMA tile (9217,
# global_load_lds stages) and the direct form's shipped schedule for n <= 4 (386, the float-C epilogue)
INSTANCES = {
    "search_dft35": "template __global__ void fracenc::search_dft<false, 123905, 8u, 4u, false>(fracenc::DftArgs);",
    "search_dft35_hits": "template __global__ void fracenc::search_dft<true, 123905, 8u, 4u, false>(fracenc::DftArgs);",
    "search_dft": "template __global__ void fracenc::search_dft<false, 9217, 8u, 4u, true>(fracenc::DftArgs);",
    "search_dft_hits": "template __global__ void fracenc::search_dft<true, 9217, 8u, 4u, true>(fracenc::DftArgs);",
    "search_mfma": "template __global__ void fracenc::search_mfma<4, 4, false, 386>(fracenc::MfmaSearchArgs);",
    "search_mfma16": "template __global__ void fracenc::search_mfma16<4, false>(fracenc::MfmaSearchArgs);",
}


def test_product_search_kernels_wait_for_their_dma_before_every_barrier():
    bad, checked = lds_dma_check.check(F.PRODUCT_LIB, r"fracenc::search_")
    for fam in FAMILIES:
        assert any(fam in k for k in checked), (fam, "no instance with LDS-DMA found")
    assert not bad, {k: v[:3] for k, v in bad.items()}


def test_every_lds_dma_kernel_in_the_library_is_guarded():
    bad, checked = lds_dma_check.check(F.PRODUCT_LIB)
    assert len(checked) >= 20
    assert not bad, sorted(bad)[:5]


def _compile(tmp_path, name, plain):
    src = tmp_path / f"{name}.hip"
    src.write_text('#include "fracenc_common.h"\n#include "fracenc_mfma.hip"\n#include "fracenc_dft.hip"\n'
                   + INSTANCES[name] + "\n")
    out = tmp_path / f"{name}{'_plain' if plain else ''}.co"
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-mllvm",
           "-amdgpu-mfma-vgpr-form", "--cuda-device-only", "--no-gpu-bundle-output", "-c", "-I", CSRC, str(src),
           "-o", str(out)]
    if plain:
        cmd.insert(1, "-DFRAC_TEST_PLAIN_STAGE_BARRIER")
    subprocess.run(cmd, check=True, capture_output=True)
    return str(out)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not present")
@pytest.mark.parametrize("name", sorted(INSTANCES))
def test_each_instance_is_guarded_compiled_alone(tmp_path, name):
    good, checked = lds_dma_check.check(_compile(tmp_path, name, plain=False))
    assert checked and not good


# The negative control: with the barrier reduced to a plain __syncthreads() the check must flag the
# hazard.  (The SEA tiled form's instance is left out: its chunk-entry stores before each barrier
# happen to make the compiler emit vmcnt(0) even there, so it shows no hazard to detect.)
@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not present")
@pytest.mark.parametrize("name", ["search_dft35", "search_dft35_hits", "search_mfma"])
def test_check_flags_a_plain_barrier(tmp_path, name):
    bad, checked = lds_dma_check.check(_compile(tmp_path, name, plain=True))
    assert checked and bad, f"{name}: the check did not see the hazard of a plain __syncthreads() stage barrier"
