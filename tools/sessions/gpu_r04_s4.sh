#!/bin/bash
# round 4 session 4: resolve_small (n <= 4), closed-form grid counts.
# direct-form entries, the fit fused into resolve_dft — the full GPU suite, then C4 quadtree / C2 timings
# and the C4 quadtree kernel trace.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s4
mkdir -p $O
bash tools/gpu_suite.sh r04s4
timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
cat $O/paths.jsonl
timeout -k 10 200 python3 tools/c2_rate.py > $O/c2_rate.log 2>&1
timeout -k 10 180 python3 tools/c2_profile.py > $O/c2_profile.log 2>&1
cat $O/c2_rate.log $O/c2_profile.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c4q_prof -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/c4q_prof.jsonl 2> $O/c4q_prof.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2_prof -o kt --output-format csv -- python3 $R/tools/c2_rate.py > $O/c2_prof.log 2>&1
echo ok
