#!/bin/bash
# round 4 session 38: a level's domain and range bucket keys in one launch (bucket_keys_rows2).  GPU suite, then
# per library (product, committed = libfracenc_ab_orig.so) the C4q and C4 rows, then a C4q kernel trace each.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s38
mkdir -p $O
bash tools/gpu_suite.sh r04s38 && cp gpurun_out/suite_r04s38.log $O/tests.log
tail -1 $O/tests.log
for v in prod ab_orig prod2 ab_orig2; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_orig*) lib=$R/fractencode_amd/libfracenc_ab_orig.so ;; esac
  FRAC_LIB=$lib timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths_$v.jsonl 2> $O/paths_$v.err
  echo "== $v"; cut -c1-330 $O/paths_$v.jsonl
done
cd /tmp && export TMPDIR=/tmp
for v in prod ab_orig; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_*) lib=$R/fractencode_amd/libfracenc_$v.so ;; esac
  FRAC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/$v.jsonl 2> $O/$v.err
  grep -h "bucket_keys" $(find $O/$v -name '*kernel_stats.csv') | cut -d, -f1-4
done
echo ok
