#!/bin/bash
# Burst demods: PLL table entry and msema slot loaded ahead, one soft store
# per bit, exact fmod fast path (variant pf): burst parity, then A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4q
mkdir -p $OUT
cd $R
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_pf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_burst.py tests/test_gpu_burst_msk.py > $OUT/pytest_burst.log 2>&1 || exit $?
bash scripts/ab_bench.sh r4q/oq "base pf base pf" --mode burst10500 --steps 6 --warmup 2 > $OUT/ab_oq.txt 2>&1 || exit $?
bash scripts/ab_bench.sh r4q/msk "base pf base pf" --mode burstmsk1200 --steps 6 --warmup 2 > $OUT/ab_msk.txt 2>&1
