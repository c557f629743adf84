#!/bin/bash
# The non-headline bench modes with their CPU baselines: burst OQPSK (C4),
# burst MSK, MSK 600 (C3), MSK 1200, C5 in process and through the binaries,
# C1.  Usage: bash scripts/gpu_modes.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for m in burst10500 burstmsk1200 msk600 msk1200; do
  timeout -k 10 300 python bench.py --mode $m --steps 20 --cpu-runs 1 > $OUT/bench_$m.log 2>&1 || exit $?
done
timeout -k 10 240 python bench.py --mode c5 --steps 20 > $OUT/bench_c5.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --mode c5bin --steps 3 > $OUT/bench_c5bin.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --mode c1 > $OUT/bench_c1.log 2>&1 || exit $?
