#!/bin/bash
# round 4 final measurement of the committed build: the GPU suite, smoke(), the bench line, the search's
# traffic passes (tools/pmc_search_r04.sh, re-keying profiles/pmc_search.json on the box), the bench
# line again (now carrying the traffic), its kernel trace, and the C4 quadtree / C2 rows.
# usage: tools/gpu_r04_final.sh TAG
set -euo pipefail
R=$(pwd)
T=${1:?tag}
O=$R/gpurun_out/r04_$T
mkdir -p $O
bash tools/gpu_suite.sh r04$T
cp gpurun_out/suite_r04$T.log $O/
timeout -k 10 300 python3 -c "import __graft_entry__ as G; G.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
bash tools/pmc_search_r04.sh $O/pmc
timeout -k 10 400 python3 bench.py > $O/bench_traffic.json 2> $O/bench_traffic.err
cat $O/bench_traffic.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bench_prof -o kt --output-format csv -- python3 $R/bench.py --steps 20 > $O/bench_prof.json 2> $O/bench_prof.err
cp $(find $O/bench_prof -name '*kernel_stats.csv') $O/bench_kernel_stats.csv
cd $R
timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
timeout -k 10 200 python3 tools/c2_rate.py > $O/c2_rate.log 2>&1
timeout -k 10 180 python3 tools/c2_profile.py > $O/c2_profile.log 2>&1
cat $O/paths.jsonl $O/c2_rate.log $O/c2_profile.log
echo ok
