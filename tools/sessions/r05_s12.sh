#!/bin/bash
# round 5 session 12: TMASK through the guarded six-MFMA tile function (dft_tile_max6g) — parity and the sweep
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s12
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
echo ok
