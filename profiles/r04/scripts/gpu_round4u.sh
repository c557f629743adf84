#!/bin/bash
# Burst demods under the memory-clause (bmc) and max-ILP (bilp) scheduling
# strategies against the default: C4 and burst-MSK A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4u
mkdir -p $OUT
cd $R
bash scripts/ab_bench.sh r4u/oq "base bmc bilp base bmc bilp" --mode burst10500 --steps 6 --warmup 2 > $OUT/ab_oq.txt 2>&1 || exit $?
bash scripts/ab_bench.sh r4u/msk "base bmc bilp base bmc bilp" --mode burstmsk1200 --steps 6 --warmup 2 > $OUT/ab_msk.txt 2>&1
