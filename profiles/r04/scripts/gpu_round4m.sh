#!/bin/bash
# Round-4 GPU check (m): the continuous MSK demod built without machine LICM
# (and with the memory-clause scheduler): MSK parity, then C3 / MSK 1200 / C5 A/B.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_msknolicm.so timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_msk.py tests/test_gpu_msk_rate.py tests/test_gpu_c5.py > $OUT/pytest_msknolicm.log 2>&1 || exit $?
bash scripts/ab_bench.sh $TAG/m600 "base msknolicm mskmc base msknolicm mskmc" --mode msk600 --steps 10 > $OUT/ab_msk600.txt 2>&1 || exit $?
mkdir -p $OUT/m1200 && bash scripts/ab_bench.sh $TAG/m1200 "base msknolicm mskmc" --mode msk1200 --steps 10 > $OUT/ab_msk1200.txt 2>&1 || exit $?
mkdir -p $OUT/c5 && bash scripts/ab_bench.sh $TAG/c5 "base msknolicm mskmc" --mode c5 --steps 20 > $OUT/ab_c5.txt 2>&1
