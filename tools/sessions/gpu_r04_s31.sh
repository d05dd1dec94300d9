#!/bin/bash
# round 4 session 31: search_mfma at n <= 4, T = 4 bounded to 5 waves per SIMD (96 VGPRs, 2 spilled;
# libfracenc_ab_s5.so) against the committed build: C4q rate and a C4q kernel trace each.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s31
mkdir -p $O
for v in prod ab_s5 prod2 ab_s52; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_s5*) lib=$R/fractencode_amd/libfracenc_ab_s5.so ;; esac
  FRAC_LIB=$lib timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths_$v.jsonl 2> $O/paths_$v.err
  echo "== $v"; cat $O/paths_$v.jsonl
done
cd /tmp && export TMPDIR=/tmp
for v in prod ab_s5; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_*) lib=$R/fractencode_amd/libfracenc_$v.so ;; esac
  FRAC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/$v.jsonl 2> $O/$v.err
  grep -h "search_mfma<4\|resolve_small" $(find $O/$v -name '*kernel_stats.csv') | cut -d, -f1-4
done
echo ok
