#!/bin/bash
# round 4 session 16: resolver occupancy A/B on the C4 quadtree — resolve_small at 5 / 6 waves per SIMD and
# resolve_mfma<16> at 4 (libfracenc_ab_occ.so: resolve_small 93 VGPRs, resolve_mfma<16> 128 with 16 spilled;
# libfracenc_ab_occ6.so: resolve_small 80 with 2 spilled) against the product; one kernel trace each.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s16
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in prod ab_occ ab_occ6 prod2 ab_occ2; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_occ2) lib=$R/fractencode_amd/libfracenc_ab_occ.so ;; ab_*) lib=$R/fractencode_amd/libfracenc_$v.so ;; esac
  FRAC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/$v.jsonl 2> $O/$v.err
  grep -h "resolve_small<4>\|resolve_mfma<16>" $(find $O/$v -name '*kernel_stats.csv') | cut -d, -f1-4
done
echo ok
