#!/bin/bash
# The search's traffic passes on the shipped C3 search (tools/c3_once.py, 4 launches), one rocprofv3
# run per pass under its own limit: the sized read requests, FETCH_SIZE, WRITE_SIZE; then
# tools/pmc_traffic.py writes profiles/pmc_search.json keyed to this build.  Stops at the first failure.
# usage: tools/pmc_search_r04.sh OUTDIR
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$(realpath -m "${1:?outdir}")
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d "$out/rdreq" -o pmc --output-format csv -- python3 "$R/tools/c3_once.py" mfma 4 > "$out/rdreq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o pmc --output-format csv -- python3 "$R/tools/c3_once.py" mfma 4 > "$out/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o pmc --output-format csv -- python3 "$R/tools/c3_once.py" mfma 4 > "$out/write.log" 2>&1
cd "$R"
python3 tools/pmc_traffic.py fourier "void fracenc::search_dft<false, 123905, 8u" \
  $(find "$out/rdreq" -name '*counter_collection.csv') $(find "$out/fetch" -name '*counter_collection.csv') \
  $(find "$out/write" -name '*counter_collection.csv') "rocprofv3 --pmc, separate passes, tools/c3_once.py mfma 4 (tools/pmc_search_r04.sh)" > "$out/pmc_traffic.json"
cat "$out/pmc_traffic.json"
