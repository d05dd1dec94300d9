#!/bin/bash
# round 5 session 18: classifier keys from the planes' block sums (frame_block_sums + bucket_keys_bs) —
# GPU parity (classifier cases, odd plane sides, distinct planes, C4 / C4q full size, the large pool), then
# C4 / C4q interleaved against the previous build and a C4q kernel trace
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s18
mkdir -p $O
python3 -c "import torch" > /dev/null
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_classify.py tests/test_quadtree.py tests/test_gpu_fullsize.py tests/test_integration.py > $O/tests.log 2>&1
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_prod -o kt --output-format csv -- python3 $R/tools/c4q_emit.py leaves 10 > $O/kt_prod.log 2>&1
cd $R
for r in 1 2 3; do
  for v in head prod; do
    if [ $v = prod ]; then L=$R/fractencode_amd/libfracenc.so; else L=$R/fractencode_amd/ab_$v.so; fi
    FRAC_LIB=$L timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths_${v}_$r.jsonl 2> $O/paths_${v}_$r.err
  done
done
echo ok
