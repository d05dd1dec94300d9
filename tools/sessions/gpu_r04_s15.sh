#!/bin/bash
# round 4 session 15: search_mfma16 with a stage's two tiles software-pipelined, and the n <= 4 float-C loop unrolled with the next tile read ahead — the product library
# (with a forced MFMA/epilogue interleave), the same without the interleave (libfracenc_ab_nosched.so), and the
# committed kernel (libfracenc_ab_orig.so): n = 16 parity tests, then one C4q kernel trace per library.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s15
mkdir -p $O
bash tools/gpu_suite.sh r04s15 && cp gpurun_out/suite_r04s15.log $O/tests.log
tail -3 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in prod ab_nosched ab_orig prod2; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_*) lib=$R/fractencode_amd/libfracenc_$v.so ;; esac
  FRAC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/$v.jsonl 2> $O/$v.err
  grep -h "search_mfma16<4, false>\|resolve_mfma<16>\|search_mfma<4, 4, false" $(find $O/$v -name '*kernel_stats.csv') | cut -d, -f1-4
done
echo ok
