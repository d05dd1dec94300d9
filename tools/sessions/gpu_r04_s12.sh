#!/bin/bash
# round 4 session 12: reverts (leaf stream, resolve_dft prefetch); A/B of search_mfma16 with four
# transforms per wave (libfracenc_ab_tpw4.so, one wave per SIMD) against the product on the C4 quadtree.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s12
mkdir -p $O
bash tools/gpu_suite.sh r04s12
timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
FRAC_LIB=$R/fractencode_amd/libfracenc_ab_tpw4.so timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths_tpw4.jsonl 2> $O/paths_tpw4.err
timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths2.jsonl 2> $O/paths2.err
cat $O/paths.jsonl $O/paths_tpw4.jsonl $O/paths2.jsonl
timeout -k 10 200 python3 tools/c2_rate.py > $O/c2_rate.log 2>&1
cat $O/c2_rate.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c4q_prof -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/c4q_prof.jsonl 2> $O/c4q_prof.err
FRAC_LIB=$R/fractencode_amd/libfracenc_ab_tpw4.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c4q_tpw4_prof -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/c4q_tpw4_prof.jsonl 2> $O/c4q_tpw4_prof.err
echo ok
