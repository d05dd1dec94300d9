#!/bin/bash
# round 5 session 22: the n = 4 / 16 pool rows built in mfma_prep's domain half (no pool_build launch) — parity,
# C4q kernel traces (HEAD vs the working tree), frames interleaved
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s22
mkdir -p $O
python3 -c "import torch" > /dev/null
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_classify.py tests/test_quadtree.py tests/test_gpu_fullsize.py  > $O/tests.log 2>&1
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in head prod; do
  if [ $v = prod ]; then L=$R/fractencode_amd/libfracenc.so; else L=$R/fractencode_amd/ab_$v.so; fi
  FRAC_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o kt --output-format csv -- python3 $R/tools/c4q_emit.py leaves 10 > $O/kt_$v.log 2>&1
done
cd $R
for r in 1 2 3; do
  for v in head prod; do
    if [ $v = prod ]; then L=$R/fractencode_amd/libfracenc.so; else L=$R/fractencode_amd/ab_$v.so; fi
    FRAC_LIB=$L timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths_${v}_$r.jsonl 2> $O/paths_${v}_$r.err
  done
done
echo ok
