#!/bin/bash
# round 4 session 27: resolve_dft issues every load that depends on the slot alone before testing any of them
# (the padding check moved after the entries), and the record's range is read beside them.  GPU suite, then C2
# rates and a C4q kernel trace for the product library and the committed one (libfracenc_ab_orig.so).
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s27
mkdir -p $O
bash tools/gpu_suite.sh r04s27 && cp gpurun_out/suite_r04s27.log $O/tests.log
tail -1 $O/tests.log
for v in prod ab_orig prod2 ab_orig2; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_orig*) lib=$R/fractencode_amd/libfracenc_ab_orig.so ;; esac
  echo "== $v"
  FRAC_LIB=$lib timeout -k 10 200 python3 tools/c2_rate.py > $O/c2_rate_$v.log 2>&1
  grep -v amdgpu.ids $O/c2_rate_$v.log | grep -v Warning | grep -v "self._ctx"
done
cd /tmp && export TMPDIR=/tmp
for v in prod ab_orig; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_*) lib=$R/fractencode_amd/libfracenc_$v.so ;; esac
  FRAC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/$v.jsonl 2> $O/$v.err
  grep -h "resolve_dft" $(find $O/$v -name '*kernel_stats.csv') | cut -d, -f1-4
  cat $O/$v.jsonl
done
echo ok
