#!/bin/bash
# Round-4 GPU check (o): the MSK demod's ring slots loaded one sample ahead:
# MSK parity, then MSK 600 / MSK 1200 / C5 A/B.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT/m1200 $OUT/m600 $OUT/c5
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_msk.py tests/test_gpu_msk_rate.py tests/test_gpu_c5.py tests/test_gpu_chan.py > $OUT/pytest.log 2>&1 || exit $?
bash scripts/ab_bench.sh $TAG/m600 "mskold base mskold base" --mode msk600 --steps 10 > $OUT/ab_msk600.txt 2>&1 || exit $?
bash scripts/ab_bench.sh $TAG/m1200 "mskold base" --mode msk1200 --steps 10 > $OUT/ab_msk1200.txt 2>&1 || exit $?
bash scripts/ab_bench.sh $TAG/c5 "mskold base" --mode c5 --steps 20 > $OUT/ab_c5.txt 2>&1
