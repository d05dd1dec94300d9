#!/bin/bash
# round 5 session 11: search_dft carrying the winning chunk's tile mask (TMASK) — GPU parity on the product build
# (TMASK up to kDftTmaskTiles), a frame-size sweep of never / always TMASK builds interleaved, and the
# end-to-end step with the tuples packed straight into pinned host memory (with and without SDMA copies).
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s11
mkdir -p $O
python3 -c "import torch" > /dev/null
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1
tail -3 $O/tests.log
for r in 1 2 3; do
  for v in never always; do
    FRAC_LIB=$R/fractencode_amd/ab_$v.so timeout -k 10 240 python3 tools/tmask_sweep.py 50 >> $O/sweep.jsonl 2>&1
  done
done
grep '"S"' $O/sweep.jsonl | tail -14
timeout -k 10 300 python3 tools/e2e_probe.py 20 3 e2e,device,e2e_zc > $O/e2e_zc.jsonl 2>&1
grep round $O/e2e_zc.jsonl
HSA_ENABLE_SDMA=0 timeout -k 10 300 python3 tools/e2e_probe.py 20 3 e2e,device,e2e_zc > $O/e2e_zc_nosdma.jsonl 2>&1
grep round $O/e2e_zc_nosdma.jsonl
echo ok
