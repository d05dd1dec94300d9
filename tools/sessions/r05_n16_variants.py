#!/usr/bin/env python3
"""Round 5, n = 16 A/B libraries: search_mfma16 with
  p16  s_setprio(1) around each tile's 32-MFMA cluster, 0 before the epilogue (cdna_hip_programming.md T5)
  sc2  each transform's 16-deep accumulation split into two 8-deep chains (even / odd K-steps), summed
       before the integer conversion (exact: each half < 128·128·510 < 2^23, the sum < 2^24)
built from the working tree by tools/build_variant.py into fractencode_amd/libfracenc_ab_{p16,sc2}.so."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BV = os.path.join(ROOT, "tools", "build_variant.py")
LOOP = """            floatx16_t acc[TPW];
#pragma unroll
            for (int j = 0; j < TPW; ++j)
                acc[j] = zero;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const half8_t af = __builtin_bit_cast(half8_t, la[(q * KS + s) * 64 + lane]);
#pragma unroll
                for (int j = 0; j < TPW; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf[j][s], acc[j], 0, 0, 0);
            }
            uint32_t e[16];"""
P16 = LOOP.replace("#pragma unroll\n            for (int s = 0;", "__builtin_amdgcn_s_setprio(1);\n#pragma unroll\n            for (int s = 0;") \
          .replace("            uint32_t e[16];", "            __builtin_amdgcn_s_setprio(0);\n            uint32_t e[16];")
SC2 = """            floatx16_t acc[TPW], acc2[TPW];
#pragma unroll
            for (int j = 0; j < TPW; ++j) {
                acc[j] = zero;
                acc2[j] = zero;
            }
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const half8_t af = __builtin_bit_cast(half8_t, la[(q * KS + s) * 64 + lane]);
#pragma unroll
                for (int j = 0; j < TPW; ++j) {
                    if (s & 1)
                        acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf[j][s], acc2[j], 0, 0, 0);
                    else
                        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf[j][s], acc[j], 0, 0, 0);
                }
            }
#pragma unroll
            for (int j = 0; j < TPW; ++j)
                acc[j] += acc2[j];
            uint32_t e[16];"""
assert P16 != LOOP
for name, new in (("p16", P16), ("sc2", SC2)):
    out = os.path.join(ROOT, "fractencode_amd", f"libfracenc_ab_{name}.so")
    subprocess.check_call([sys.executable, BV, out, f"fracenc_mfma.hip:{LOOP}=>{new}"])
