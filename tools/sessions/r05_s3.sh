#!/bin/bash
# round 5 session 3: the resolve carrying the winner's domain origin (tdom) and the range item; the 32-byte
# quadtree leaves.  Quadtree / full-size / parity tests, then the interleaved A/B (prod, notdom = tdom off at
# run time, prev = round 4's chain), C4q paths with the leaves, C2 kernel trace.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s3
mkdir -p $O; rm -f $O/ab.jsonl
python3 -c "import torch" > /dev/null
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_quadtree.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1
[ -n "${SKIP_TESTS:-}" ] || tail -2 $O/tests.log
for k in 1 2 3; do
  for v in prod notdom prev; do
    lib=$R/fractencode_amd/libfracenc.so
    [ $v != prod ] && lib=$R/fractencode_amd/libfracenc_ab_$v.so
    FRAC_LIB=$lib timeout -k 10 200 python3 tools/c3c2_rate.py >> $O/ab.jsonl 2>> $O/ab.err
    tail -1 $O/ab.jsonl | cut -c1-330
  done
done
timeout -k 10 200 python3 tools/e2e_probe.py 20 2 > $O/e2e_probe.jsonl 2>&1 && cat $O/e2e_probe.jsonl
timeout -k 10 300 python3 tools/fallback_probe.py 0 1 16 > $O/fallback.jsonl 2>&1 && cat $O/fallback.jsonl
timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths.jsonl 2> $O/paths.err
cat $O/paths.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2kt -o kt --output-format csv -- python3 $R/tools/c2_profile.py > $O/c2kt.log 2>&1
echo ok
