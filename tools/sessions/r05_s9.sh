#!/bin/bash
# round 5 session 9: the new quadtree tests (fp32 levels, device count), and why the search is slower inside the
# end-to-end step (tools/e2e_probe.py's idle and device-to-device legs).
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s9
mkdir -p $O
python3 -c "import torch" > /dev/null
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_quadtree.py -k "fp32 or device_count" > $O/tests.log 2>&1
tail -4 $O/tests.log
timeout -k 10 300 python3 tools/e2e_probe.py 20 3 > $O/e2e_probe.jsonl 2>&1
grep round $O/e2e_probe.jsonl
echo ok
