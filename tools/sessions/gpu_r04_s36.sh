#!/bin/bash
# round 4 session 36: search_mfma16's target workgroup count (kMfma16TargetWgs) 2048 (product) against 1024
# and 4096 (libfracenc_ab_t1024.so, libfracenc_ab_t4096.so): C4q rate and a C4q kernel trace each.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s36
mkdir -p $O
for v in prod ab_t1024 ab_t4096 prod2; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_*) lib=$R/fractencode_amd/libfracenc_$v.so ;; esac
  FRAC_LIB=$lib timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths_$v.jsonl 2> $O/paths_$v.err
  echo "== $v"; cut -c1-420 $O/paths_$v.jsonl
done
cd /tmp && export TMPDIR=/tmp
for v in prod ab_t1024 ab_t4096; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_*) lib=$R/fractencode_amd/libfracenc_$v.so ;; esac
  FRAC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/$v.jsonl 2> $O/$v.err
  grep -h "search_mfma16\|resolve_mfma<16>" $(find $O/$v -name '*kernel_stats.csv') | cut -d, -f1-4
done
echo ok
