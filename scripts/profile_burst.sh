#!/bin/bash
# Burst evidence at HEAD: the C4 and burst MSK bench lines and their
# rocprofv3 kernel statistics (profile_round.sh part b's burst half).
set -eo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 $R/bench.py --mode burst10500 --steps 10 --cpu-runs 1 > $OUT/bench_burst.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profb_$TAG -o prof -- python3 $R/bench.py --mode burst10500 --steps 6 --no-cpu-baseline > $OUT/bench_burst_prof.log 2>&1
find /tmp/profb_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_burst.csv \;
timeout -k 10 600 python3 $R/bench.py --mode burstmsk1200 --steps 6 --cpu-runs 1 > $OUT/bench_burstmsk.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profm_$TAG -o prof -- python3 $R/bench.py --mode burstmsk1200 --steps 4 --no-cpu-baseline > $OUT/bench_burstmsk_prof.log 2>&1
find /tmp/profm_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_burstmsk.csv \;
ls -la $OUT
