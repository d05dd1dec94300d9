#!/usr/bin/env python3
"""The C3 frame through the reference's core (oracle/_ref/core_driver, --nocpu, one HIP engine) with the
library's host trace on (FRAC_TRACE): where core.encode()'s time goes beyond the search.
usage: tools/drop_in_trace.py [MODE]   (MODE: ref | batch:K)"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fractencode_amd.synth import value_noise  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "ref"
with tempfile.TemporaryDirectory() as td:
    plane = os.path.join(td, "c3.u8")
    value_noise(4096, 4096, 1234).tofile(plane)
    for rep in range(2):
        r = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "core_driver"), plane, "4096", "4096", "16", "8", "0",
                            "0", "-1", os.path.join(td, "out.bin"), "0", "0", mode],
                           env=dict(os.environ, FRAC_TRACE="1"), capture_output=True, text=True, timeout=120)
        print(f"--- run {rep} rc={r.returncode}")
        print(r.stdout.strip().splitlines()[0] if r.stdout else "")
        print(r.stderr)
