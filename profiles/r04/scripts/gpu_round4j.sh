#!/bin/bash
# Round-4 GPU check (j): the AGC (and clipping) moved into the demod's FIR
# wave: parity of both variants, then the C2 bench A/B.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for v in p1full p1agc; do
  AERO_ENGINE_SO=$R/aero-cli_amd/libaero_engine_$v.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/pytest_$v.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
bash scripts/ab_bench.sh $TAG "base p1full p1agc base p1full p1agc" --steps 8 > $OUT/ab.txt 2>&1
