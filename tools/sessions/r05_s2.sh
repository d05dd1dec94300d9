#!/bin/bash
# round 5 session 2: search_dft merges its domain splits per slot (64-bit atomicMax), resolve_dft reads one
# word per slot instead of the entries' CSR walk.  The GPU suite on the product build, then an interleaved
# A/B (process-alternated) against the previous commit's chain (libfracenc_ab_prev.so): C3 and C2 rates;
# the C2 chain's kernel trace.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s2
mkdir -p $O
bash tools/gpu_suite.sh r05s2
cp gpurun_out/suite_r05s2.log $O/
for k in 1 2 3; do
  for v in prod prev; do
    lib=$R/fractencode_amd/libfracenc.so
    [ $v = prev ] && lib=$R/fractencode_amd/libfracenc_ab_prev.so
    FRAC_LIB=$lib timeout -k 10 200 python3 tools/c3c2_rate.py >> $O/ab.jsonl 2>> $O/ab.err
    tail -1 $O/ab.jsonl
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2kt -o kt --output-format csv -- python3 $R/tools/c2_profile.py > $O/c2kt.log 2>&1
grep -h "dft" $(find $O/c2kt -name '*kernel_stats.csv') | cut -d, -f1-4
echo ok
