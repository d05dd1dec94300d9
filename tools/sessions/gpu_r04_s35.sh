#!/bin/bash
# round 4 session 35: the Fourier path's timing boundaries recorded by its kernels' own launch events
# (hipExtLaunchKernelGGL start/stop) instead of marker packets.  GPU suite, C2 rates and profile for the
# product and the committed library (libfracenc_ab_orig.so), then the headline bench line.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s35
mkdir -p $O
bash tools/gpu_suite.sh r04s35 && cp gpurun_out/suite_r04s35.log $O/tests.log
tail -1 $O/tests.log
for v in prod ab_orig prod2; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in ab_*) lib=$R/fractencode_amd/libfracenc_$v.so ;; esac
  echo "== $v"
  FRAC_LIB=$lib timeout -k 10 200 python3 tools/c2_rate.py > $O/c2_rate_$v.log 2>&1
  FRAC_LIB=$lib timeout -k 10 180 python3 tools/c2_profile.py > $O/c2_profile_$v.log 2>&1
  grep -v amdgpu.ids $O/c2_rate_$v.log $O/c2_profile_$v.log | grep -v Warning | grep -v "self._ctx"
done
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
echo ok
