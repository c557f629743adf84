#!/bin/bash
# MSK evidence at HEAD: C3 (MSK 600) and MSK 1200 bench lines with kernel stats.
set -eo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py --mode msk600 --steps 20 --cpu-runs 1 > $OUT/bench_msk600.log 2>&1
timeout -k 10 400 python3 $R/bench.py --mode msk1200 --steps 20 --cpu-runs 1 > $OUT/bench_msk1200.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profk_$TAG -o prof -- python3 $R/bench.py --mode msk1200 --steps 10 --no-cpu-baseline > $OUT/bench_msk1200_prof.log 2>&1
find /tmp/profk_$TAG -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_msk1200.csv \;
ls -la $OUT
