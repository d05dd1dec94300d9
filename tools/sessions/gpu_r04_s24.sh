#!/bin/bash
# round 4 session 24: search_mfma16 merges each wave's transform pair before the integer conversion (resolve_mfma
# merge_span 2) — the GPU suite on the product library, then one C4q kernel trace each for it and for the
# committed kernel (libfracenc_ab_orig.so, tools/build_variant.py --git HEAD), product again last.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s24
mkdir -p $O
bash tools/gpu_suite.sh r04s24 && cp gpurun_out/suite_r04s24.log $O/tests.log
tail -3 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in prod ab_orig prod2; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_*) lib=$R/fractencode_amd/libfracenc_$v.so ;; esac
  FRAC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/$v.jsonl 2> $O/$v.err
  grep -h "search_mfma16<4, false>\|resolve_mfma<16>" $(find $O/$v -name '*kernel_stats.csv') | cut -d, -f1-4
done
echo ok
