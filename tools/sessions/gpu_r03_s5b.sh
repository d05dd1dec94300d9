#!/bin/bash
# round 3 session 5: search time and HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) against the
# Fourier search's workgroup count (domain splits per block group): FRAC_DFT_WGS values as arguments
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r03_s5b
mkdir -p $O
python3 -c "import torch"
timeout -k 10 300 env AB_REPS=3 python3 tools/ab_env.py FRAC_DFT_WGS $(echo "$@" | tr ' ' ',') 6 > $O/wgs.log 2>&1
cat $O/wgs.log
cd /tmp && export TMPDIR=/tmp
for w in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    FRAC_DFT_WGS=$w timeout -s KILL 150 rocprofv3 --pmc $c -d $O/w${w}_$c -o pmc --output-format csv -- python3 $R/tools/c3_once.py mfma 4 > /dev/null 2>&1
  done
  python3 $R/tools/pmc_summary.py $(find $O -path "*w${w}_*" -name '*counter_collection.csv') > $O/w${w}_pmc.txt
  echo "WGS=$w"; grep -A3 "search_dft" $O/w${w}_pmc.txt
done
echo ok
