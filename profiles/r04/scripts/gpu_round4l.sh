#!/bin/bash
# Round-4 GPU check (l): the burst front ends' ring traffic cut (bt_d1 in
# registers, peak-detector d1/d2 read from d3, delay slots carried):
# the burst parity tests, then the C4 / burst MSK A/B against the previous
# front ends.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_burst.py tests/test_gpu_burst_msk.py tests/test_gpu_burst_scale.py > $OUT/pytest_burst.log 2>&1 || exit $?
bash scripts/ab_bench.sh $TAG "prevfront base prevfront base" --mode burst10500 --steps 6 > $OUT/ab_burst.txt 2>&1 || exit $?
mkdir -p $OUT/msk && bash scripts/ab_bench.sh $TAG/msk "prevfront base" --mode burstmsk1200 --steps 4 > $OUT/ab_burstmsk.txt 2>&1
