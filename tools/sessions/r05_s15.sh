#!/bin/bash
# round 5 session 15: the direct form at n <= 4 with slot words and a float running minimum per stage —
# GPU parity, C4q kernel traces (HEAD vs the working tree) and C4q frames interleaved
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s15
mkdir -p $O
python3 -c "import torch" > /dev/null
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_quadtree.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
FRAC_LIB=$R/fractencode_amd/ab_head.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_head -o kt --output-format csv -- python3 $R/tools/c4q_emit.py leaves 10 > $O/kt_head.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_prod -o kt --output-format csv -- python3 $R/tools/c4q_emit.py leaves 10 > $O/kt_prod.log 2>&1
for v in head prod; do echo "== $v"; grep -h "search_mfma<4\|resolve_small<4" $(find $O/kt_$v -name '*kernel_stats.csv') | cut -d, -f1-4 | cut -c1-120; done
cd $R
for r in 1 2 3; do
  for v in head prod; do
    if [ $v = prod ]; then L=$R/fractencode_amd/libfracenc.so; else L=$R/fractencode_amd/ab_$v.so; fi
    FRAC_LIB=$L timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths_${v}_$r.jsonl 2> $O/paths_${v}_$r.err
    echo "$v $r $(cut -c150-320 $O/paths_${v}_$r.jsonl)"
  done
done
echo ok
