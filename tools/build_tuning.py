#!/usr/bin/env python3
"""Builds the A/B tuning library: the product sources with -DFRAC_TUNING, so the ablation
variants of FRAC_MFMA_VARIANT (MFMA-only, VALU-only, no LDS-DMA, no barrier — wrong results by
design) exist.  Output fractencode_amd/libfracenc_tuning.so; use it with FRAC_LIB=<that path>
(tools/ab_mfma.py).  The product build (__graft_entry__.build) never sets FRAC_TUNING.

--stamps: the diagnostic clock build instead (adds -DFRAC_CLOCK_STAMP: search_dft stamps
s_memtime / s_memrealtime around its loop; tools/clock_stamp.py), fractencode_amd/libfracenc_stamps.so."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402

if "--stamps" in sys.argv[1:]:
    out = os.path.join(ROOT, "fractencode_amd", "libfracenc_stamps.so")
    subprocess.check_call(G.hipcc_cmd(out, "-DFRAC_TUNING", "-DFRAC_CLOCK_STAMP"), cwd=G.CSRC)
else:
    out = os.path.join(ROOT, "fractencode_amd", "libfracenc_tuning.so")
    subprocess.check_call(G.hipcc_cmd(out, "-DFRAC_TUNING"), cwd=G.CSRC)
print(out)
