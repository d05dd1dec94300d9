#!/bin/bash
# round 3 session 5: the final build end to end — GPU suite, headline bench, HBM traffic
# passes (FETCH_SIZE / WRITE_SIZE, separate runs), the counter passes and kernel stats of
# tools/pmc_search.sh, the bench under rocprofv3 --kernel-trace --stats, and shard_sim.
# A test failure (pytest rc 1) does not stop the measurements; anything else does.
set -uo pipefail
R=$(pwd)
O=$R/gpurun_out/r03_s5f
mkdir -p $O
python3 -c "import torch" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
rc=$?
tail -3 $O/suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o pmc --output-format csv -- python3 $R/tools/c3_once.py mfma 4 > /dev/null
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/write -o pmc --output-format csv -- python3 $R/tools/c3_once.py mfma 4 > /dev/null
bash $R/tools/pmc_search.sh $O/pmc 4 > $O/pmc.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bstats -o kt --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 > $O/bench_rocprof.json 2> $O/bench_rocprof.err
cd $R
timeout -k 10 300 python3 tools/shard_sim.py > $O/shard_sim.log 2>&1
echo ok
