#!/bin/bash
# round 3 session 3: L2 and SQ counters of the issue-cost variant (36) against the six-MFMA form
# (21), and a sweep of the Fourier search's workgroup count (domain splits) for 36
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r03_s3
mkdir -p $O
python3 -c "import torch"
cd /tmp && export TMPDIR=/tmp
for v in 21 36; do
  for p in "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
           "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM"; do
    n=$(echo $p | md5sum | cut -c1-6)
    FRAC_MFMA_VARIANT=$v timeout -s KILL 150 rocprofv3 --pmc $p -d $O/v${v}_$n -o pmc --output-format csv -- python3 $R/tools/c3_once.py mfma 4 > /dev/null
  done
  python3 $R/tools/pmc_summary.py $(find $O -path "*v${v}_*" -name '*counter_collection.csv') > $O/v${v}_pmc.txt
done
cd $R
FRAC_MFMA_VARIANT=36 timeout -k 10 400 python3 tools/ab_env.py FRAC_DFT_WGS 4096,8192,16384,32768 8 > $O/wgs.log 2>&1
echo ok
