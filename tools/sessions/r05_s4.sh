#!/bin/bash
# round 5 session 4: quadtree leaves staged in LDS and written as contiguous 1-KiB runs (records and 32-byte
# leaves) against the per-lane emit (libfracenc_ab_prevemit.so); the fp32-regime probe at C3 size.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s4
mkdir -p $O
python3 -c "import torch" > /dev/null
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_quadtree.py tests/test_gpu_fullsize.py -k "quadtree or c4" > $O/tests.log 2>&1
tail -2 $O/tests.log
for k in 1 2; do
  for v in prod prevemit; do
    lib=$R/fractencode_amd/libfracenc.so
    [ $v != prod ] && lib=$R/fractencode_amd/libfracenc_ab_$v.so
    FRAC_LIB=$lib timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths_${v}_$k.jsonl 2> $O/paths_${v}_$k.err
    echo "$v $k $(cut -c150-420 $O/paths_${v}_$k.jsonl)"
  done
done
timeout -k 10 300 python3 tools/fallback_probe.py 0 1 16 > $O/fallback.jsonl 2>&1 && cat $O/fallback.jsonl
cd /tmp && export TMPDIR=/tmp
for v in prod prevemit; do
  lib=$R/fractencode_amd/libfracenc.so
  [ $v != prod ] && lib=$R/fractencode_amd/libfracenc_ab_$v.so
  for m in records leaves; do
    FRAC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_${v}_$m -o kt --output-format csv -- python3 $R/tools/c4q_emit.py $m 10 > $O/kt_${v}_$m.log 2>&1
    echo "$v $m: $(grep -h qt_split_emit $(find $O/kt_${v}_$m -name '*kernel_stats.csv') | cut -d, -f2-4)"
  done
done
echo ok
