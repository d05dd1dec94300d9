#!/bin/bash
# round 4 session 9: splits in proportion to each bucket's tiles, n = 16 at 2,048 target workgroups,
# the range prep's independent row loads.  Full suite; C4 / C4 quadtree on the product library and on
# the A/B library whose n = 16 resolve gathers the range bytes (libfracenc_ab_bytecopy.so); traces.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s9
mkdir -p $O
bash tools/gpu_suite.sh r04s9
timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
FRAC_LIB=$R/fractencode_amd/libfracenc_ab_bytecopy.so timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths_bytecopy.jsonl 2> $O/paths_bytecopy.err
timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths2.jsonl 2> $O/paths2.err
cat $O/paths.jsonl $O/paths_bytecopy.jsonl $O/paths2.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c4q_prof -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/c4q_prof.jsonl 2> $O/c4q_prof.err
echo ok
