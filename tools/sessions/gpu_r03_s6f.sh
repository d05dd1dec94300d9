#!/bin/bash
# round 3 session 6: measurements of the final build (fused Fourier preparation, one timing event
# per run boundary) — headline bench, HBM traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs),
# the counter passes and kernel stats of tools/pmc_search.sh, the bench under rocprofv3
# --kernel-trace --stats, the either-side paths, C2 rates and shard_sim.  The GPU suite ran on
# the same build before (profiles/r03/session6/gpu_suite_summary.txt).
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r03_s6f
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o pmc --output-format csv -- python3 $R/tools/c3_once.py mfma 4 > /dev/null
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/write -o pmc --output-format csv -- python3 $R/tools/c3_once.py mfma 4 > /dev/null
bash $R/tools/pmc_search.sh $O/pmc 4 > $O/pmc.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bstats -o kt --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 > $O/bench_rocprof.json 2> $O/bench_rocprof.err
cd $R
timeout -k 10 300 python3 tools/bench_paths.py > $O/paths.jsonl 2> $O/paths.err
timeout -k 10 200 python3 tools/c2_rate.py > $O/c2_rate.log 2>&1
timeout -k 10 180 python3 tools/c2_profile.py c3t8 > $O/c2_profile.log 2>&1
timeout -k 10 300 python3 tools/shard_sim.py > $O/shard_sim.log 2>&1
echo ok
