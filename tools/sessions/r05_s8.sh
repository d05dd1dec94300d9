#!/bin/bash
# round 5 session 8: resolve_dft prefetching the next tile of its chunk (one tile ahead) against the previous
# build: parity tests, C3/C2 interleaved A/B, C4q rows.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s8
mkdir -p $O
rm -f $O/ab.jsonl
python3 -c "import torch" > /dev/null
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_quadtree.py > $O/tests.log 2>&1
tail -1 $O/tests.log
for k in 1 2 3; do
  for v in prod prev; do
    lib=$R/fractencode_amd/libfracenc.so
    [ $v != prod ] && lib=$R/fractencode_amd/libfracenc_ab_$v.so
    FRAC_LIB=$lib timeout -k 10 200 python3 tools/c3c2_rate.py >> $O/ab.jsonl 2>> $O/ab.err
    tail -1 $O/ab.jsonl | cut -c1-330
  done
done
for v in prod prev; do
  lib=$R/fractencode_amd/libfracenc.so
  [ $v != prod ] && lib=$R/fractencode_amd/libfracenc_ab_$v.so
  FRAC_LIB=$lib timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths_$v.jsonl 2> $O/paths_$v.err
  echo "$v $(cut -c150-330 $O/paths_$v.jsonl)"
done
echo ok
