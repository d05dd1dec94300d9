#!/bin/bash
# Counter passes on the shipped C3 search (tools/c3_once.py), one rocprofv3 run per pass, each
# under its own time limit; then a kernel-trace --stats pass.  Stops at the first failure.
# usage: tools/pmc_search.sh OUTDIR [reps]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$(realpath -m "${1:?outdir}")
reps=${2:-4}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
passes=(
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
  "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU2 SQ_INSTS_SALU"
  "GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_THREAD_CYCLES_VALU"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  echo "pass $i: $p"
  timeout -s KILL 150 rocprofv3 --pmc $p -d "$out/pass$i" -o pmc --output-format csv -- python3 "$R/tools/c3_once.py" mfma "$reps"
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$out/stats" -o kt --output-format csv -- python3 "$R/tools/c3_once.py" mfma 10
for i in 1 2 3; do
  python3 "$R/tools/pmc_summary.py" $(find "$out/pass$i" -name '*counter_collection.csv') > "$out/pass$i.txt"
done
cp $(find "$out/stats" -name '*kernel_stats.csv') "$out/kernel_stats.csv"
echo done
