#!/bin/bash
# round 4 session 20: pool_build with one lane per D4 row.  Full suite, then the C4 quadtree rate and trace.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s20
mkdir -p $O
bash tools/gpu_suite.sh r04s20
timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
cat $O/paths.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c4q_prof -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/c4q_prof.jsonl 2> $O/c4q_prof.err
echo ok
