#!/bin/bash
# round 5 final measurement of the committed build: GPU suite, smoke(), the bench line, the search's traffic passes
# (re-keying profiles/pmc_search.json, copied out under gpurun_out/), the bench line again (carrying the traffic),
# the headline kernel trace (tools/c3_once.py e2e and device-resident), C2 / C4q / C4 / C5 rows, the shard
# simulation.  usage: tools/sessions/r05_final.sh TAG
set -euo pipefail
R=$(pwd)
T=${1:?tag}
O=$R/gpurun_out/r05_$T
mkdir -p $O
bash tools/gpu_suite.sh r05$T
cp gpurun_out/suite_r05$T.log $O/
timeout -k 10 300 python3 -c "import __graft_entry__ as G; G.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cut -c1-400 $O/bench.json
bash tools/pmc_search_r04.sh $O/pmc
cp profiles/pmc_search.json $O/pmc_search.json
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_traffic.json 2> $O/bench_traffic.err
cut -c1-400 $O/bench_traffic.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c3kt_e2e -o kt --output-format csv -- python3 $R/tools/c3_once.py mfma 20 e2e > $O/c3kt_e2e.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c3kt -o kt --output-format csv -- python3 $R/tools/c3_once.py mfma 20 > $O/c3kt.log 2>&1
grep -h "search_dft\|resolve_dft\|dft_prep" $(find $O/c3kt_e2e -name '*kernel_stats.csv') | cut -d, -f1-4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2kt -o kt --output-format csv -- python3 $R/tools/c2_profile.py > $O/c2kt.log 2>&1
cd $R
timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 c5 --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
timeout -k 10 200 python3 tools/c3c2_rate.py > $O/c3c2_rate.jsonl 2> $O/c3c2_rate.err
timeout -k 10 300 python3 tools/shard_sim.py > $O/shard_sim.log 2>&1
cut -c1-300 $O/paths.jsonl $O/c3c2_rate.jsonl
tail -8 $O/shard_sim.log
echo ok
