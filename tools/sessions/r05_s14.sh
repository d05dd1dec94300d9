#!/bin/bash
# round 5 session 14: slot words for the direct form at n <= 4 (search_mfma -> resolve_small) — GPU parity, and
# C4 / C4q interleaved: HEAD (entries + CSR walk) vs the working tree, plus the never / always tile-mask builds
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s14
mkdir -p $O
python3 -c "import torch" > /dev/null
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_quadtree.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1
tail -3 $O/tests.log
for r in 1 2 3; do
  for v in head prod never always; do
    if [ $v = prod ]; then L=$R/fractencode_amd/libfracenc.so; else L=$R/fractencode_amd/ab_$v.so; fi
    FRAC_LIB=$L timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths_${v}_$r.jsonl 2> $O/paths_${v}_$r.err
    echo "$v $r $(cut -c1-200 $O/paths_${v}_$r.jsonl | tr '\n' ' ')"
  done
done
echo ok
