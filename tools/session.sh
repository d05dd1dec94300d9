#!/bin/bash
# One GPU session on the gpurun box: named steps in order, each under its own time limit, outputs under
# gpurun_out/<TAG>/.  The first failing step ends the session (no GPU step runs after a fault, an abort or
# a time-out).  Replaces the per-session scripts of rounds 3-5 (in git history under tools/sessions/).
# usage: tools/session.sh TAG STEP...
# steps:
#   suite         the whole GPU test suite (pytest -m gpu tests), one process
#   tests:A,B,..  the GPU tests pytest -k "A or B or ..." selects
#   smoke         __graft_entry__.smoke()
#   bench         python bench.py --steps 20 --warmup 5 (the headline line) -> bench.json
#   pmc           the search's HBM-traffic passes (tools/pmc_search_r04.sh), re-keying profiles/pmc_search.json
#                 (copied to the session directory)
#   sqpmc         the search's SQ counter passes (tools/pmc_search.sh)
#   trace         rocprofv3 --kernel-trace --stats of the headline step alone (tools/c3_once.py mfma 20 e2e),
#                 device-resident, and of C2 (tools/c2_profile.py)
#   paths         tools/bench_paths.py --only c4q c4 c5, tools/c3c2_rate.py
#   shard         tools/shard_sim.py (per-shard efficiency on one GPU)
#   py:SCRIPT     python3 tools/SCRIPT (its stdout to SCRIPT.out)
set -uo pipefail
R=$(pwd)
T=${1:?tag}
shift
O=$R/gpurun_out/$T
mkdir -p "$O"
python3 -c "import torch" > /dev/null || exit 1
run() { # SECONDS LOGNAME COMMAND...: one step, stop the session on failure
  local secs=$1 log=$2
  shift 2
  echo "=== [$(date +%T)] $log: $*"
  timeout -k 10 "$secs" "$@" > "$O/$log" 2>&1
  local rc=$?
  tail -3 "$O/$log"
  if [ $rc -ne 0 ]; then
    echo "=== $log failed (rc=$rc): session ends"
    exit $rc
  fi
}
for step in "$@"; do
  case $step in
  suite) run 1500 suite.log python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests ;;
  tests:*) k=${step#tests:}; run 900 "tests_${k//,/_}.log" python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "${k//,/ or }" ;;
  smoke) run 300 smoke.log python3 -c "import __graft_entry__ as G; G.smoke()" ;;
  bench) run 500 bench.log python3 -u bench.py --steps 20 --warmup 5 --out "$O/bench.json" ;;
  pmc) run 600 pmc.log bash tools/pmc_search_r04.sh "$O/pmc" && cp profiles/pmc_search.json "$O/pmc_search.json" ;;
  sqpmc) run 900 sqpmc.log bash tools/pmc_search.sh "$O/sqpmc" ;;
  trace)
    (cd /tmp && export TMPDIR=/tmp &&
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/c3kt_e2e" -o kt --output-format csv -- python3 "$R/tools/c3_once.py" mfma 20 e2e &&
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/c3kt" -o kt --output-format csv -- python3 "$R/tools/c3_once.py" mfma 20 &&
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/c2kt" -o kt --output-format csv -- python3 "$R/tools/c2_profile.py") > "$O/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
    grep -h "search_dft\|resolve_dft\|dft_prep" $(find "$O/c3kt_e2e" -name '*kernel_stats.csv') | cut -d, -f1-4 ;;
  paths)
    run 400 paths.jsonl python3 tools/bench_paths.py --only c4q c4 c5 --steps 20 --warmup 3
    run 200 c3c2_rate.jsonl python3 tools/c3c2_rate.py ;;
  shard) run 300 shard_sim.log python3 tools/shard_sim.py ;;
  py:*) s=${step#py:}; run 900 "${s%% *}.out" python3 tools/$s ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $T ok"
