#!/bin/bash
# round 4 session 26: timing events at the run's inner boundaries (start, prep, search) without the system-scope
# fence; the run's last event keeps it.  GPU suite on the product library, then the C2 rates for it, for
# device-scope-release events (libfracenc_ab_dev.so) and for the committed library (libfracenc_ab_orig.so),
# and the headline bench line on the product library.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s26
mkdir -p $O
bash tools/gpu_suite.sh r04s26 && cp gpurun_out/suite_r04s26.log $O/tests.log
tail -1 $O/tests.log
for v in prod ab_dev ab_orig prod2; do
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
