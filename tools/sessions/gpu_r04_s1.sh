#!/bin/bash
# round 4 session 1: the pruned product build and the device-planned quadtree — GPU parity subset,
# the C4 quadtree path timing, and its kernel trace.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s1
mkdir -p $O
bash tools/gpu_suite.sh r04s1 -k "integration or failure_comes_back or quadtree or new_frame or default_cli or sampled_form or rectangular or fourier_and_direct or operand_extremes or product_form or stress_frame or decoders_agree or goldens or classify"
timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
cat $O/paths.jsonl
QT_CALLS=3 timeout -k 10 120 python3 tools/trace_c4q.py 0.05 > $O/trace_c4q.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c4q_prof -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/c4q_prof.jsonl 2> $O/c4q_prof.err
echo ok
