#!/bin/bash
# round 4 session 43: search_mfma16 with s_setprio(1) around each tile's MFMA cluster (libfracenc_ab_p16.so)
# against the product build: the n = 16 parity cases on it, then C4q rates and kernel traces.
# The variant: tools/build_variant.py fractencode_amd/libfracenc_ab_p16.so with two substitutions in fracenc_mfma.hip:
#   "acc[j] = zero;" + the following "for (int s = 0; s < KS; ++s)" loop gets __builtin_amdgcn_s_setprio(1) before it,
#   and "uint32_t e[16];" gets __builtin_amdgcn_s_setprio(0) before it.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s43
mkdir -p $O
FRAC_LIB=$R/fractencode_amd/libfracenc_ab_p16.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "16" > $O/tests_p16.log 2>&1
tail -1 $O/tests_p16.log
for v in prod ab_p16 prod2 ab_p162; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_p16*) lib=$R/fractencode_amd/libfracenc_ab_p16.so ;; esac
  FRAC_LIB=$lib timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths_$v.jsonl 2> $O/paths_$v.err
  echo "== $v"; cut -c1-330 $O/paths_$v.jsonl
done
cd /tmp && export TMPDIR=/tmp
for v in prod ab_p16; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_*) lib=$R/fractencode_amd/libfracenc_$v.so ;; esac
  FRAC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/$v.jsonl 2> $O/$v.err
  grep -h "search_mfma16" $(find $O/$v -name '*kernel_stats.csv') | cut -d, -f1-4
done
echo ok
