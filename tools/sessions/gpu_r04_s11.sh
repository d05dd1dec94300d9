#!/bin/bash
# round 4 session 11: fallback in the resolving wave (no fallback_fp32 launch after fused fits), resolve_dft chunk prefetch,
# at least 8 tiles per work item, quadtree leaves copied on a second stream.  Full suite, C4 / C4q rates, C4q and C2 kernel traces.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s11
mkdir -p $O
bash tools/gpu_suite.sh r04s11
timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
cat $O/paths.jsonl
timeout -k 10 200 python3 tools/c2_rate.py > $O/c2_rate.log 2>&1
cat $O/c2_rate.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c4q_prof -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/c4q_prof.jsonl 2> $O/c4q_prof.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2_prof -o kt --output-format csv -- python3 $R/tools/c2_rate.py > $O/c2_prof.log 2>&1
echo ok
