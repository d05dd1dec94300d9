#!/bin/bash
# round 5 session 10: the end-to-end step with the tuples packed straight into pinned host memory, and with the
# copies done by blit kernels instead of the SDMA engines (HSA_ENABLE_SDMA=0).
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s10
mkdir -p $O
python3 -c "import torch" > /dev/null
timeout -k 10 300 python3 tools/e2e_probe.py 20 3 e2e,device,e2e_zc > $O/e2e_zc.jsonl 2>&1
grep round $O/e2e_zc.jsonl
HSA_ENABLE_SDMA=0 timeout -k 10 300 python3 tools/e2e_probe.py 20 3 e2e,device,e2e_zc > $O/e2e_zc_nosdma.jsonl 2>&1
grep round $O/e2e_zc_nosdma.jsonl
echo ok
