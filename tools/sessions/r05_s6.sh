#!/bin/bash
# round 5 session 6: the Fourier preparation reads slot / tile-row origins from maps built at layout time
# (fill_range_slots / fill_tile_pos / qt_fill_item) instead of the slot_range → ranges and tile_pos → porig → doms
# chains.  Parity + quadtree tests, C3/C2 A/B against the previous build, the fp32 probe (wall clock), C2 trace.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s6
mkdir -p $O
rm -f $O/ab.jsonl
python3 -c "import torch" > /dev/null
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_quadtree.py tests/test_integration.py > $O/tests.log 2>&1
tail -1 $O/tests.log
for k in 1 2 3; do
  for v in prod prev; do
    lib=$R/fractencode_amd/libfracenc.so
    [ $v != prod ] && lib=$R/fractencode_amd/libfracenc_ab_$v.so
    FRAC_LIB=$lib timeout -k 10 200 python3 tools/c3c2_rate.py >> $O/ab.jsonl 2>> $O/ab.err
    tail -1 $O/ab.jsonl | cut -c1-330
  done
done
timeout -k 10 300 python3 tools/fallback_probe.py 0 1 16 > $O/fallback.jsonl 2>&1 && grep white $O/fallback.jsonl
timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
cut -c150-420 $O/paths.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2kt -o kt --output-format csv -- python3 $R/tools/c2_profile.py > $O/c2kt.log 2>&1
echo ok
