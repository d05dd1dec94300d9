#!/bin/bash
# round 5 session 5: the fp32 fallback spread over the whole grid (fallback_grid, settled before records are read)
# instead of one resolving wave per range.  GPU suite; the C3 fp32-regime probe and C3/C2 rates against the
# previous build (libfracenc_ab_prev.so); the headline bench line.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s5
mkdir -p $O
rm -f $O/ab.jsonl
bash tools/gpu_suite.sh r05s5
cp gpurun_out/suite_r05s5.log $O/
for v in prod prev; do
  lib=$R/fractencode_amd/libfracenc.so
  [ $v != prod ] && lib=$R/fractencode_amd/libfracenc_ab_$v.so
  FRAC_LIB=$lib timeout -k 10 300 python3 tools/fallback_probe.py 0 1 16 > $O/fallback_$v.jsonl 2>&1
  echo "$v"; cat $O/fallback_$v.jsonl | grep white
done
for k in 1 2; do
  for v in prod prev; do
    lib=$R/fractencode_amd/libfracenc.so
    [ $v != prod ] && lib=$R/fractencode_amd/libfracenc_ab_$v.so
    FRAC_LIB=$lib timeout -k 10 200 python3 tools/c3c2_rate.py >> $O/ab.jsonl 2>> $O/ab.err
    tail -1 $O/ab.jsonl | cut -c1-330
  done
done
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cut -c1-900 $O/bench.json
echo ok
