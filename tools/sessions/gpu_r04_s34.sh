#!/bin/bash
# round 4 session 34: two n = 16 parity cases across 8 tiles (ties; threshold hits at T = 4) and the n = 16 VALU
# engine without its dead 4-copy instantiation.  GPU suite, then the C4q and C4 rows.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s34
mkdir -p $O
bash tools/gpu_suite.sh r04s34 && cp gpurun_out/suite_r04s34.log $O/tests.log
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/bench_paths.py --only c4q c4 --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
cat $O/paths.jsonl
echo ok
