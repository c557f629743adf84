#!/bin/bash
# Round-4 GPU check (k): the OQPSK coarse kernel's |X| + log10 smoothing in
# the transform's register layout (AERO_X_REGY build): parity, then the C2
# bench A/B and the variant's kernel stats.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_regy.so timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullscale.py > $OUT/pytest_regy.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/ab_bench.sh $TAG "base regy base regy" --steps 10 > $OUT/ab.txt 2>&1
