#!/bin/bash
# round 4 session 7: (a) the in-kernel shader clock of the C3 Fourier search (variant 35, ablations
# 240 / 241; diagnostic library libfracenc_stamps.so); (b) the traffic reconciliation: FETCH_SIZE and
# the sized request counters on the calibration kernel (known bytes) and on the shipped search, and
# on the search with the XCD order off / one domain split (tuning knobs, same diagnostic library);
# (c) the bench headline and its kernel trace.  Every GPU step under its own limit; stops at the
# first failure.
set -euo pipefail
R=$(pwd)
O=$R/gpurun_out/r04_s7
mkdir -p $O
STAMPS=$R/fractencode_amd/libfracenc_stamps.so
FRAC_LIB=$STAMPS timeout -k 10 120 python3 tools/clock_stamp.py 35,240,241,35 --seconds 3 > $O/clock.jsonl 2> $O/clock.err
cat $O/clock.jsonl
cd /tmp && export TMPDIR=/tmp
P1="FETCH_SIZE"
P2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_READ_sum"
# calibration: 1 GiB read once by 4,096 workgroups; then 10.5 MB (one domain split) shared by all
i=0
for p in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 60 rocprofv3 --pmc $p -d $O/cal_once_p$i -o pmc --output-format csv -- $R/tools/fetch_calib once 1073741824 4096 0 > $O/cal_once_p$i.log 2>&1
  timeout -s KILL 60 rocprofv3 --pmc $p -d $O/cal_shared_p$i -o pmc --output-format csv -- $R/tools/fetch_calib shared 11010048 4096 6000 > $O/cal_shared_p$i.log 2>&1
done
# the shipped search (product library), 4 launches
i=0
for p in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $p -d $O/c3_p$i -o pmc --output-format csv -- python3 $R/tools/c3_once.py mfma 4 > $O/c3_p$i.log 2>&1
done
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/c3_w -o pmc --output-format csv -- python3 $R/tools/c3_once.py mfma 4 > $O/c3_w.log 2>&1
# order experiments (diagnostic library): XCD order off; one domain split (1,024 workgroups)
export FRAC_LIB=$STAMPS
i=0
for p in "$P1" "$P2"; do
  i=$((i + 1))
  FRAC_XCD_ORDER=0 timeout -s KILL 120 rocprofv3 --pmc $p -d $O/c3x0_p$i -o pmc --output-format csv -- python3 $R/tools/c3_once.py mfma 4 > $O/c3x0_p$i.log 2>&1
  FRAC_DFT_WGS=1024 timeout -s KILL 120 rocprofv3 --pmc $p -d $O/c3w1k_p$i -o pmc --output-format csv -- python3 $R/tools/c3_once.py mfma 4 > $O/c3w1k_p$i.log 2>&1
done
unset FRAC_LIB
for d in $O/cal_* $O/c3*; do
  [ -d "$d" ] || continue
  python3 $R/tools/pmc_summary.py $(find $d -name '*counter_collection.csv') > $d.txt
done
cd $R
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bench_prof -o kt --output-format csv -- python3 $R/bench.py > $O/bench_prof.json 2> $O/bench_prof.err
cp $(find $O/bench_prof -name '*kernel_stats.csv') $O/bench_kernel_stats.csv
echo ok
