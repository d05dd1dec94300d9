#!/bin/bash
# round 5 session 17: the N > 1 frame upload in row stripes + RCCL all-gather (bench.FrameStep stripes) —
# the nccl world-1 tests, and bench.py at N = 1 (unchanged path) as a check
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s17
mkdir -p $O
python3 -c "import torch" > /dev/null
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_multirank.py > $O/tests.log 2>&1
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -12
echo ok
