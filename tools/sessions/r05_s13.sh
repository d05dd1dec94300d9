#!/bin/bash
# round 5 session 13: tile masks (TMASK) on classified pools — C4 and the C4 quadtree with the never / always
# builds, interleaved
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s13
mkdir -p $O
python3 -c "import torch" > /dev/null
for r in 1 2 3; do
  for v in never always; do
    FRAC_LIB=$R/fractencode_amd/ab_$v.so timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths_${v}_$r.jsonl 2> $O/paths_${v}_$r.err
    cut -c1-250 $O/paths_${v}_$r.jsonl
  done
done
echo ok
