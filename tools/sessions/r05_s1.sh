#!/bin/bash
# round 5 session 1: the new bench line (value = end-to-end step), and the n = 16 A/B:
# product vs p16 (s_setprio) vs sc2 (two 8-deep chains) — n = 16 parity on each, C4q rates interleaved,
# kernel traces, and two PMC passes per library.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r05_s1
mkdir -p $O
python3 -c "import torch" > /dev/null
for v in p16 sc2; do
  FRAC_LIB=$R/fractencode_amd/libfracenc_ab_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "16" > $O/tests_$v.log 2>&1
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cat $O/bench.json
for v in prod p16 sc2 prod2 p162 sc22; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in p16*|sc2*) lib=$R/fractencode_amd/libfracenc_ab_${v:0:3}.so ;; esac
  FRAC_LIB=$lib timeout -k 10 300 python3 tools/bench_paths.py --only c4q --steps 20 --warmup 3 > $O/paths_$v.jsonl 2> $O/paths_$v.err
  echo "== $v"; cut -c1-300 $O/paths_$v.jsonl
done
cd /tmp && export TMPDIR=/tmp
passes=(
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
  "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM"
)
for v in prod p16 sc2; do
  lib=$R/fractencode_amd/libfracenc.so
  case $v in p16|sc2) lib=$R/fractencode_amd/libfracenc_ab_$v.so ;; esac
  FRAC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o kt --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 10 --warmup 2 > $O/kt_$v.log 2>&1
  grep -h "search_mfma16\|resolve_mfma<16" $(find $O/kt_$v -name '*kernel_stats.csv') | cut -d, -f1-4 || true
  i=0
  for p in "${passes[@]}"; do
    i=$((i + 1))
    FRAC_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $p -d $O/pmc_${v}_$i -o pmc --output-format csv -- python3 $R/tools/bench_paths.py --only c4q --steps 3 --warmup 2 > $O/pmc_${v}_$i.log 2>&1
    python3 $R/tools/pmc_summary.py $(find $O/pmc_${v}_$i -name '*counter_collection.csv') > $O/pmc_${v}_$i.txt
    grep -A9 "search_mfma16" $O/pmc_${v}_$i.txt || true
  done
done
echo ok
