#!/bin/bash
# round 5 session 23: the tuple sink (frac_set_tuple_sink, ABI 8) — its GPU tests, the multi-rank and
# end-to-end-related tests, then the end-to-end step with and without the sink interleaved (tools/e2e_probe.py)
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s23
mkdir -p $O
python3 -c "import torch" > /dev/null
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tuple_sink.py tests/test_multirank.py tests/test_gpu_parity.py -k "sink or nccl or stripes or two_ranks or fallback or fp32" > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 400 python3 tools/e2e_probe.py 20 3 e2e,e2e_nosink,device > $O/e2e_sink.jsonl 2>&1
grep round $O/e2e_sink.jsonl
echo ok
