#!/bin/bash
# round 5 session 7: counters of the C2 chain (dft_prep, search_dft, resolve_dft at Lenna T = 8 / 4): where the
# resolve's time goes (VALU vs waits), two --pmc passes over tools/c2_profile.py.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s7
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
passes=(
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
  "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES SQ_INSTS_BRANCH"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $p -d $O/pass$i -o pmc --output-format csv -- python3 $R/tools/c2_profile.py > $O/pass$i.log 2>&1
  python3 $R/tools/pmc_summary.py $(find $O/pass$i -name '*counter_collection.csv') > $O/pass$i.txt
  grep -A9 "dft" $O/pass$i.txt
done
echo ok
