#!/bin/bash
# round 4 session 13: counters of the C4 quadtree's kernels (search_mfma16, search_mfma<4>, the
# resolvers): three --pmc passes over a short C4q run, each under its own limit.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s13
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
passes=(
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
  "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM"
  "GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_WAVES SQ_INSTS_VALU_CVT"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $p -d $O/pass$i -o pmc --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 3 --warmup 2 > $O/pass$i.log 2>&1
  python3 $R/tools/pmc_summary.py $(find $O/pass$i -name '*counter_collection.csv') > $O/pass$i.txt
done
echo ok
