#!/bin/bash
# round 3 session 5: wave-state counters of the shipped search (35) against the LDS-prefetch (44)
# and producer-wave (47) variants (usage: tools/gpu_r03_s5.sh VARIANTS...)
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r03_s5
mkdir -p $O
python3 -c "import torch"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  for p in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"; do
    n=$(echo $p | md5sum | cut -c1-6)
    FRAC_MFMA_VARIANT=$v timeout -s KILL 150 rocprofv3 --pmc $p -d $O/v${v}_$n -o pmc --output-format csv -- python3 $R/tools/c3_once.py mfma 4 > /dev/null
  done
  python3 $R/tools/pmc_summary.py $(find $O -path "*v${v}_*" -name '*counter_collection.csv') > $O/v${v}_pmc.txt
  grep -A12 "search_dft" $O/v${v}_pmc.txt | head -24
done
echo ok
