#!/bin/bash
# Round-4 GPU check (g): the full GPU suite, C5 through the binaries with the
# host split, coarse MFMA-adder A/B (bench + parity), burst A/B.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -v --timeout 500 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_mfma.so timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/pytest_mfma.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/ab_bench.sh $TAG/coarse "base mfma base mfma" --steps 8 > $OUT/ab_coarse.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py --mode c5bin --steps 3 > $OUT/bench_c5bin.log 2>&1 || exit $?
bash scripts/ab_bench.sh $TAG "prevburst base" --mode burst10500 --steps 6 > $OUT/ab_burst.txt 2>&1 || exit $?
mkdir -p $OUT/msk && bash scripts/ab_bench.sh $TAG/msk "prevburst base" --mode burstmsk1200 --steps 4 > $OUT/ab_burstmsk.txt 2>&1
