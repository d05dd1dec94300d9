#!/bin/bash
# round 4 session 8: n = 16 with two transforms per wave (search_mfma16), the LDS range prep and the
# resolve's copies from the B fragments; T = 8 paired resolve_dft.  The full GPU suite first, then
# the C4 quadtree / C2 timings and kernel traces, and the Fourier search's stamped timeline (L2 model).
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s8
mkdir -p $O
bash tools/gpu_suite.sh r04s8
timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
cat $O/paths.jsonl
timeout -k 10 200 python3 tools/c2_rate.py > $O/c2_rate.log 2>&1
timeout -k 10 180 python3 tools/c2_profile.py > $O/c2_profile.log 2>&1
cat $O/c2_rate.log $O/c2_profile.log
FRAC_LIB=$R/fractencode_amd/libfracenc_stamps.so timeout -k 10 120 python3 tools/clock_stamp.py 35 --seconds 3 --dump $O/stamps > $O/clock.jsonl 2> $O/clock.err
cat $O/clock.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c4q_prof -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/c4q_prof.jsonl 2> $O/c4q_prof.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2_prof -o kt --output-format csv -- python3 $R/tools/c2_profile.py > $O/c2_prof.log 2>&1
echo ok
