#!/bin/bash
# round 4 session 42: kernel traces of the final build — the C4 quadtree frame (both split thresholds) and the
# C2 chain (Lenna 512², T = 8 and 4, back to back) — for profiles/r04/final/.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s42
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c4q -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/c4q.jsonl 2> $O/c4q.err
C2_FRAMES=200 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2 -o kt --output-format csv -- python3 $R/tools/c2_rate.py > $O/c2.log 2> $O/c2.err
echo ok
