#!/bin/bash
# The GPU test suite in one process, under its own time limit, log under gpurun_out/ (usage:
# tools/gpu_suite.sh TAG [pytest args...]).  Stops there on failure; prints the summary.
set -uo pipefail
tag=${1:?tag}; shift
mkdir -p gpurun_out
python3 -c "import torch" || exit 1
timeout -k 10 1500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" tests > gpurun_out/suite_$tag.log 2>&1
rc=$?
tail -5 gpurun_out/suite_$tag.log
exit $rc
