#!/bin/bash
# round 5: C2 / C3 rates of the product build (TMASK up to kDftTmaskTiles) against the never-TMASK build,
# interleaved (tools/c3c2_rate.py per library, 4 rounds)
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_tmask_ab
mkdir -p $O
for r in 1 2 3 4; do
  FRAC_LIB=$R/fractencode_amd/ab_never.so timeout -k 10 200 python3 tools/c3c2_rate.py >> $O/c3c2_ab.jsonl 2>> $O/c3c2_ab.err
  timeout -k 10 200 python3 tools/c3c2_rate.py >> $O/c3c2_ab.jsonl 2>> $O/c3c2_ab.err
done
cut -c1-300 $O/c3c2_ab.jsonl
echo ok
